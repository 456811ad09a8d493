"""Random-restart sweep across GPUs: one process per GPU, restarts sharded in contiguous
blocks, no communication inside the evaluation loop, one exchange per sweep step
(SURVEY.md 8(e)):

  1. all_gather of (best F, restart id) from every rank (world x 16 B over RCCL/xGMI);
  2. broadcast of the winning control vector from the rank that owns it.

The evaluation itself is `GrapePlan.fidelity_grad_device_async` on each rank's block
of restarts; nothing here touches the kernels.  Works with the "nccl" (RCCL) backend on
device tensors and with "gloo" on host tensors (the CPU tests use gloo, world_size 2).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous block of restarts owned by `rank`: (first, count). Blocks differ in
    size by at most one; every restart is owned by exactly one rank."""
    if n_total < 0 or world < 1 or not 0 <= rank < world:
        raise ValueError("bad shard arguments")
    base, extra = divmod(n_total, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def local_best(F: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
    """(F_best, id) of this rank as a 2-vector (float64); an empty shard reports (-inf, -1).
    Ties go to the smallest restart id; NaN scores count as -inf."""
    if F.numel() == 0:
        return torch.tensor([float("-inf"), -1.0], dtype=torch.float64, device=F.device)
    # a NaN score (a diverged restart) ranks last instead of poisoning the max
    F = torch.nan_to_num(F.to(torch.float64), nan=float("-inf"), posinf=float("inf"), neginf=float("-inf"))
    fmax = torch.max(F)
    cand = torch.where(F == fmax, ids.to(torch.float64), torch.full_like(F, float("inf")))
    return torch.stack([fmax.to(torch.float64), torch.min(cand)])


def gather_best(F: torch.Tensor, ids: torch.Tensor, X: torch.Tensor | None = None, group=None):
    """Global best over all ranks. Returns (F_best, restart_id, owner_rank, x_best or None).

    One all_gather of every rank's (F_best, id); ties go to the smallest restart id (so the
    answer does not depend on the world size). When X (this rank's (count, n_x) block, rows
    in `ids` order) is given, the owner broadcasts the winning row to every rank."""
    world = dist.get_world_size(group)
    mine = local_best(F, ids)
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine, group=group)
    allp = torch.stack(parts)                                  # (world, 2)
    fbest = torch.max(allp[:, 0])
    cand = torch.where(allp[:, 0] == fbest, allp[:, 1], torch.full_like(allp[:, 1], float("inf")))
    rid = torch.min(cand)
    owner = int(torch.nonzero(allp[:, 1] == rid)[0, 0].item())
    xb = None
    if X is not None:
        if dist.get_rank(group) == owner:
            row = int(torch.nonzero(ids.to(torch.float64) == rid)[0, 0].item())
            xb = X[row].clone()
        else:
            xb = torch.empty(X.shape[1], dtype=X.dtype, device=X.device)
        dist.broadcast(xb, src=dist.get_global_rank(group, owner) if group is not None else owner, group=group)
    return float(fbest.item()), int(rid.item()), owner, xb


def optimize_sweep(fidelity_problem, fidelity_parameters, n_restarts: int, initial_x, device: int = 0,
                   group=None, evaluate=None):
    """Random-restart optimisation sweep: the restarts are cut into
    contiguous shards, one per rank; each rank runs ALL of its restarts as one batched L-BFGS
    on its own GPU (robustgrape_amd.optimize.optimize_restarts, no communication inside the
    loop), then one exchange finds the global best and broadcasts its control vector.

    initial_x(r) -> the n_x control vector of restart r (e.g. seeded per restart, as
    examples/time_optimal_cz.jl:32).  Returns (best_cost, restart_id, owner_rank, x_best,
    local BatchResult).  Ranking is by the optimiser's cost (1 - F + sensitivities +
    regularisers), so the exchanged value is -cost through gather_best's max."""
    import numpy as np

    from .optimize import optimize_restarts
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    first, count = shard(n_restarts, world, rank)
    X0 = np.stack([np.asarray(initial_x(r), dtype=np.float64) for r in range(first, first + count)]) \
        if count else None
    res = optimize_restarts(fidelity_problem, fidelity_parameters, X0, device=device, evaluate=evaluate) \
        if count else None
    dev = res.minimizer.device if res is not None else torch.device("cpu")
    if evaluate is None and res is None:
        dev = torch.device("cuda", device)
    ids = torch.arange(first, first + count, device=dev)
    score = -res.minimum if res is not None else torch.empty(0, dtype=torch.float64, device=dev)
    X = res.minimizer if res is not None else None
    if world == 1:
        if count == 0:
            return float("inf"), -1, 0, None, res
        fbest, rid, owner, xb = gather_best_local(score, ids, X)
    else:
        if X is None:
            nx = len(np.asarray(initial_x(0)))
            X = torch.empty(0, nx, dtype=torch.float64, device=dev)
        fbest, rid, owner, xb = gather_best(score, ids, X, group=group)
    return -fbest, rid, owner, xb, res


def gather_best_local(F: torch.Tensor, ids: torch.Tensor, X: torch.Tensor):
    """Single-process form of gather_best (same tie rule)."""
    fb, rid = local_best(F, ids).tolist()
    row = int(torch.nonzero(ids.to(torch.float64) == rid)[0, 0].item())
    return fb, int(rid), 0, X[row].clone()
