"""Multi-GPU sharding of independent scenarios.

Scenarios are independent NLPs: each rank (one process per GPU) solves a
contiguous block of the global scenario stream with no data-path collective.
The only exchange is the per-step gather of each scenario's applied control,
cost and status (8 doubles = 64 B per scenario) so that every rank -- in
particular the controller on rank 0 -- holds the whole batch's result.  Over
RCCL (backend "nccl") this is one all-gather of B*64 bytes per rank.
"""
from __future__ import annotations


def shard(total: int, world: int, rank: int) -> slice:
    """Contiguous block of the global scenario index range for `rank`."""
    base, rem = divmod(total, world)
    lo = rank * base + min(rank, rem)
    return slice(lo, lo + base + (1 if rank < rem else 0))


def pack_result(x, f, status, nu: int = 6):
    """(B, 8) float64 rows: u0 (the first nu entries of x, the first control column,
    zero-padded to 6 like the closed loop's u history), f, status.  nu = 3 for the
    no-gimbal model, whose x holds 3 controls per stage."""
    import torch

    u0 = x[:, :nu]
    if nu < 6:
        u0 = torch.cat([u0, torch.zeros(x.shape[0], 6 - nu, dtype=x.dtype, device=x.device)], dim=1)
    return torch.cat([u0, f[:, None], status[:, None].to(x.dtype)], dim=1).contiguous()


def gather_rows(local, world: int, group=None):
    """All-gather equal-sized (B, k) row blocks from every rank -> (world*B, k)."""
    import torch
    import torch.distributed as dist

    out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, local, group=group)
    else:  # gloo (CPU tests, single-GPU rehearsal): staged through host memory
        host = local.cpu()
        parts = [torch.empty_like(host) for _ in range(world)]
        dist.all_gather(parts, host, group=group)
        out.copy_(torch.cat(parts, dim=0))
    return out


def pack_closed_loop(hist):
    """(B, 8K) float64 rows of a fused closed-loop launch's histories: every step's u0
    (6), f and status, scenario-major -- the per-scenario record rank 0 needs."""
    import torch

    u, f, st = hist["u"], hist["f"], hist["status"]
    B = u.shape[1]
    return torch.cat([u.permute(1, 0, 2).reshape(B, -1), f.t(), st.t().to(u.dtype)], dim=1).contiguous()


def gather_closed_loop(hist, world: int, group=None):
    """The fused mode's only exchange: one all-gather of every rank's packed
    histories after its K-step launch -> (world*B, 8K) on every rank."""
    return gather_rows(pack_closed_loop(hist), world, group)
