"""Dev tool: per-kernel VGPR / spill / scratch / occupancy of the solver (hipcc remarks)."""
import os, re, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(ROOT, "mpc-implementation_amd", "csrc", "nmpc_solve.hip")
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-mllvm", "-disable-machine-licm",
       "-Wno-unused-result", "-Wno-unused-value", "-I", os.path.join(ROOT, "include"), "--offload-device-only",
       "-c", src, "-o", "/tmp/_res.o", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[1:]
out = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp").stderr
cur, rows = None, {}
for line in out.splitlines():
    m = re.search(r"remark: (Function Name|[\w \[\]/]+?): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2)
    if k == "Function Name":
        cur = v
        rows[cur] = {}
    elif cur:
        rows[cur][k] = v
for name, r in rows.items():
    short = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", name)[:60]
    print(f"{short:60s} VGPR {r.get('VGPRs','?'):>4} AGPR {r.get('AGPRs','?'):>3} vspill {r.get('VGPRs Spill','?'):>3} "
          f"sspill {r.get('SGPRs Spill','?'):>4} scratch {r.get('ScratchSize [bytes/lane]','?'):>4} "
          f"occ {r.get('Occupancy [waves/SIMD]','?')} LDS {r.get('LDS Size [bytes/block]','?')}")
