"""Dev: summarise gpurun_out/<tag>_<variant>_<rep>.json bench lines of an A/B round."""
import glob, json, re, sys, collections
tag = sys.argv[1]
res = collections.defaultdict(list)
for f in sorted(glob.glob(f"gpurun_out/{tag}_*_[0-9].json")):
    v = re.match(rf"gpurun_out/{tag}_(.+)_\d\.json", f).group(1)
    try:
        d = json.load(open(f))
    except Exception:
        continue
    res[v].append((d["value"], d["roofline"]["kernel_avg_ms"]))
for v, l in res.items():
    print(f"{v:12s} value {[round(a / 1e3, 1) for a, _ in l]}k  kernel ms {[round(b, 1) for _, b in l]}")
