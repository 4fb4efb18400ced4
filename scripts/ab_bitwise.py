"""Dev tool: dump every output of a cold batched solve and a fused closed loop
(config 3, B scenarios, K steps) to an .npz, so two builds of the library
(NMPC_LIB=...) can be compared bit for bit:

    python scripts/ab_bitwise.py out_a.npz        # default library
    NMPC_LIB=exp/other.so python scripts/ab_bitwise.py out_b.npz
    python scripts/ab_bitwise.py --compare out_a.npz out_b.npz
"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-implementation_amd"))


def compare(a, b):
    A, Bz = np.load(a), np.load(b)
    bad = 0
    for k in A.files:
        x, y = A[k], Bz[k]
        same = x.shape == y.shape and np.ascontiguousarray(x).tobytes() == np.ascontiguousarray(y).tobytes()
        ndiff = int(np.sum(x != y)) if not same else 0
        print(f"{k:14s} {'bitwise equal' if same else f'DIFFERS in {ndiff} entries'}")
        bad += not same
    return bad


def main():
    if sys.argv[1] == "--compare":
        sys.exit(1 if compare(sys.argv[2], sys.argv[3]) else 0)
    import torch
    from nmpc_amd import nlpsol, config_spec, draw_scenarios, REFERENCE_OPTS
    B = int(os.environ.get("AB_B", "4096")); K = int(os.environ.get("AB_K", "20"))
    cfg = int(os.environ.get("AB_CONFIG", "3"))
    spec = config_spec(cfg)
    P = draw_scenarios(spec, B, seed=1000 + cfg)
    lbx, ubx, lbg, ubg = spec.bounds()
    s = nlpsol("solver", "ipopt", spec, REFERENCE_OPTS)
    sol = s(x0=np.zeros(spec.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=P.T)
    st = s.stats()
    out = {"cold_x": sol["x"], "cold_f": sol["f"], "cold_status": np.asarray(st["status_code"]),
           "cold_iters": np.asarray(st["iter_count"])}
    dev = dict(dtype=torch.float64, device="cuda")
    bnd = [torch.tensor(v, **dev) for v in (lbx, ubx, lbg, ubg)]
    p = torch.tensor(P, **dev).contiguous()
    w = torch.zeros(B, spec.nw, **dev)
    hist = {"u": torch.empty(K, B, 6, **dev), "f": torch.empty(K, B, **dev), "fov": torch.zeros(K, B, **dev),
            "status": torch.empty(K, B, dtype=torch.int32, device="cuda"),
            "iters": torch.empty(K, B, dtype=torch.int32, device="cuda")}
    s.closed_loop_device(K, *bnd, p, w, torch.full((B,), 12.0, **dev), torch.full((B,), 0.01, **dev), hist)
    torch.cuda.synchronize()
    for k, v in hist.items():
        out["cl_" + k] = v.cpu().numpy()
    out["cl_p_final"] = p.cpu().numpy()
    out["cl_w_final"] = w.cpu().numpy()
    np.savez(sys.argv[1], **out)
    print("saved", sys.argv[1], "mean cold iters", out["cold_iters"].mean(), "closed-loop iters",
          out["cl_iters"].mean())


if __name__ == "__main__":
    main()
