"""Golden fixtures for the feasibility-restoration path: inputs captured from the
config-3 closed loop (seed 1003, 4096 scenarios, steps 0-11; solves whose line
search fails, so IPOPT enters restoration) and the oracle's outcome on each.

Inputs (w = warm start, p = [x0; xs]) are data; this script recomputes every
expected output from them with oracle/nmpc_oracle.py:
    python tests/golden/gen_resto_cases.py <captured.npz>
"""
import os
import sys
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mpc-implementation_amd"))
from oracle import nmpc_oracle as orc  # noqa: E402

warnings.filterwarnings("ignore", category=RuntimeWarning)


def main(src):
    F = np.load(src)
    idx = np.arange(0, len(F["k"]), 6)
    prob = orc.make_problem("race_track_2", N=20, T=0.2)
    lbx, ubx, lbg, ubg = orc.bounds(prob)
    sol = orc.IpoptDense(prob, orc.REFERENCE_OPTS)
    out = {"w": F["w"][idx], "p": F["p"][idx], "step": F["k"][idx], "status": [], "iter": [], "x": [],
           "first_resto": [], "trace": []}
    for j in idx:
        r = sol.solve(F["w"][j], lbx, ubx, lbg, ubg, F["p"][j], trace=True)
        tr = np.array([[t["iter"], t["mu"], t["theta"], t["alpha_p"], t["alpha_d"], float(t.get("resto", False))]
                       for t in r["trace"]] + [[0.0] * 6] * (100 - len(r["trace"])))
        fr = next((int(t["iter"]) for t in r["trace"] if t.get("resto")), -1)
        out["status"].append(r["status"]); out["iter"].append(r["iter"]); out["x"].append(r["x"])
        out["first_resto"].append(fr); out["trace"].append(tr)
        print(j, r["status"], r["iter"], fr)
    np.savez_compressed(os.path.join(HERE, "resto_cases.npz"), **{k: np.asarray(v) for k, v in out.items()})


if __name__ == "__main__":
    main(sys.argv[1])
