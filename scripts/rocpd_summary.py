"""Summarise rocprofv3 rocpd databases: kernel durations, and PMC counters of the
timed dispatch of each kernel (the LAST dispatch: bench.py launches the fused kernel
twice, a scratch-copy launch and then the timed one).  Each pass directory's sibling
log (<dir>.log) holds that pass's bench JSON line; its steps / warmup / batch / mean
IP iterations / HIP-event kernel time are written next to every counter row.
usage: python scripts/rocpd_summary.py [--csv out.csv] <pass dir> [...]"""
import argparse, csv, glob, json, os, sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("dirs", nargs="+")
ap.add_argument("--csv")
a = ap.parse_args()


def bench_line(d):
    log = d.rstrip("/") + ".log"
    if not os.path.exists(log):
        return {}
    for line in reversed(open(log).read().splitlines()):
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    return {}


rows = []
for d in a.dirs:
    bl = bench_line(d)
    run = {"steps": bl.get("steps", ""), "warmup": bl.get("warmup", ""),
           "batch": bl.get("config", {}).get("global_batch", ""),
           "ibar": bl.get("mean_ip_iterations", ""),
           "kernel_ms": bl.get("roofline", {}).get("kernel_avg_ms", ""),
           "bench_value": bl.get("value", "")}
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        db = sqlite3.connect(f)
        print(f"== {f}  run: {run}")
        n = db.execute("select count(*) from counters_collection").fetchone()[0]
        if n:
            q = ("select kernel_name, counter_name, value, dispatch_id from counters_collection c "
                 "where dispatch_id = (select max(dispatch_id) from counters_collection c2 "
                 "where c2.kernel_name = c.kernel_name) order by kernel_name")
            for kn, cn, v, did in db.execute(q):
                if "nmpc" in kn:
                    print(f"  {kn[:60]:60s} {cn:24s} dispatch={did} value={v:.6g}")
                    rows.append({"kernel": kn, "counter": cn, "value": v, "dispatch": did, **run})
        else:
            q = ("select name, count(*), avg(duration), min(duration), max(duration), sum(duration) "
                 "from kernels group by name order by sum(duration) desc")
            for name, c, avg, mn, mx, tot in db.execute(q):
                print(f"  {name[:70]:70s} n={c:4d} avg={avg/1e6:10.3f} ms min={mn/1e6:9.3f} "
                      f"max={mx/1e6:9.3f} total={tot/1e6:9.3f} ms")
if a.csv and rows:
    with open(a.csv, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows)
    print("wrote", a.csv)
