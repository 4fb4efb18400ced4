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


def shard_sizes(total: int, world: int) -> list[int]:
    """Rows each rank holds under shard(): the first total % world ranks one more."""
    return [shard(total, world, r).stop - shard(total, world, r).start for r in range(world)]


def gather_rows(local, world: int, group=None, total: int | None = None):
    """All-gather the (B_r, k) row blocks of every rank -> (sum B_r, k), in rank order.

    ``total`` (the global row count) gives the per-rank sizes of shard(); omitted, every
    block must have the same size.  Unequal blocks (total % world != 0) are padded to the
    largest one, gathered in one collective (all_gather_into_tensor over RCCL needs equal
    sizes), and the padding is dropped again."""
    import torch
    import torch.distributed as dist

    sizes = shard_sizes(total, world) if total is not None else [local.shape[0]] * world
    rank = dist.get_rank(group)
    if local.shape[0] != sizes[rank]:
        raise ValueError(f"rank {rank} holds {local.shape[0]} rows, shard() gives it {sizes[rank]}")
    bmax = max(sizes)
    if local.shape[0] < bmax:
        pad = torch.zeros((bmax - local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        local = torch.cat([local, pad], dim=0)
    local = local.contiguous()
    out = torch.empty((world * bmax,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, local, group=group)
    else:  # gloo (CPU tests, single-GPU rehearsal): staged through host memory
        host = local.cpu()
        parts = [torch.empty_like(host) for _ in range(world)]
        dist.all_gather(parts, host, group=group)
        out.copy_(torch.cat(parts, dim=0))
    if all(n == bmax for n in sizes):
        return out
    return torch.cat([out[r * bmax:r * bmax + n] for r, n in enumerate(sizes)], dim=0)


def pack_closed_loop(hist):
    """(B, 8K) float64 rows of a fused closed-loop launch's histories: every step's u0
    (6), f and status, scenario-major -- the per-scenario record rank 0 needs."""
    import torch

    u, f, st = hist["u"], hist["f"], hist["status"]
    K, B = u.shape[0], u.shape[1]  # B may be 0 (a rank with an empty shard)
    return torch.cat([u.permute(1, 0, 2).reshape(B, K * u.shape[2]), f.t(), st.t().to(u.dtype)], dim=1).contiguous()


def gather_closed_loop(hist, world: int, group=None, total: int | None = None):
    """The fused mode's only exchange: one all-gather of every rank's packed
    histories after its K-step launch -> (total, 8K) on every rank (``total``
    scenarios over all ranks, sharded by shard(); None = equal shards)."""
    return gather_rows(pack_closed_loop(hist), world, group, total)
