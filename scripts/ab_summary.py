"""Dev tool: summarise an r05_ab.sh round: bitwise comparisons and bench values."""
import glob, json, os, sys
tag = sys.argv[1]
O = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
for f in sorted(glob.glob(f"{O}/{tag}_*_cmp*.txt")):
    txt = open(f).read()
    print(os.path.basename(f), "BITWISE EQUAL" if "DIFFERS" not in txt else "DIFFERS:\n" + txt)
rows = {}
for f in sorted(glob.glob(f"{O}/{tag}_*.json")):
    try:
        r = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:
        print(f, "unreadable", e); continue
    name = os.path.basename(f)[len(tag) + 1:-5]
    ch = r["roofline"].get("chain", {})
    print(f"{name:20s} {r['value']:10.0f} steps/s  kernel {r['roofline']['kernel_avg_ms']:8.2f} ms  "
          f"work-bound us/it {r['roofline']['kernel_avg_ms'] * 1e3 / max(1, ch.get('work_bound_iterations_per_slot', 1)):7.2f}")
