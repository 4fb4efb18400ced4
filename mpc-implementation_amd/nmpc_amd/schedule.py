"""Dispatch order for the fused closed-loop launch (nmpc_closed_loop_dev `order`).

A fused launch runs each scenario's K MPC steps back to back on one wavefront,
and workgroups start roughly in blockIdx order as slots free up.  A scenario
whose chain is long (locally infeasible steps that run to max_iter, as
Python/NMPC_TT.py's IPOPT options make them) and that happens to start after
the first wave of slots has drained finishes last and sets the launch time.
Longest-expected-first order (classic LPT list scheduling) removes that: the
expected chain length comes from iterations already observed in earlier MPC
steps of the same scenarios (never from the launch being ordered).
"""
from __future__ import annotations


def longest_first(cost):
    """int32 permutation of range(B), scenarios with the largest `cost` first
    (ties keep index order).  `cost`: (B,) or (k, B) torch tensor of observed
    per-step iterations (summed over steps); the result lives on cost's device."""
    import torch

    c = cost.to(torch.float64)
    if c.dim() == 2:
        c = c.sum(0)
    assert c.dim() == 1, tuple(cost.shape)
    return torch.argsort(-c, stable=True).to(torch.int32).contiguous()
