"""Restart-sweep sharding and exchange on CPU: gloo, world_size 2 and 3.

The device evaluation is replaced by a closed-form per-restart score here; what is under
test is the partition and the exchange, which are the same code the GPU bench runs over
RCCL."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from robustgrape_amd.sweep import gather_best, local_best, shard

NX = 13


def _score(r):
    # deterministic per-restart "fidelity" with a planted tie at the maximum (ids 7 and 29)
    return 1.0 if r in (7, 29) else 0.5 + 0.01 * ((r * 37) % 41) / 41.0


def _xrow(r):
    return torch.arange(NX, dtype=torch.float64) + 1000.0 * r


@pytest.mark.parametrize("n,world", [(0, 1), (1, 2), (7, 3), (256, 8), (1024, 8), (5, 8)])
def test_shard_partitions_every_restart_once(n, world):
    seen = []
    sizes = []
    for rank in range(world):
        first, count = shard(n, world, rank)
        seen.extend(range(first, first + count))
        sizes.append(count)
    assert seen == list(range(n))
    assert max(sizes) - min(sizes) <= 1


def test_shard_rejects_bad_arguments():
    with pytest.raises(ValueError):
        shard(4, 0, 0)
    with pytest.raises(ValueError):
        shard(4, 2, 2)


def test_local_best_tie_goes_to_smallest_id():
    F = torch.tensor([0.3, 0.9, 0.9, 0.1], dtype=torch.float64)
    ids = torch.tensor([10, 12, 11, 13])
    assert local_best(F, ids).tolist() == [0.9, 11.0]
    assert local_best(F[:0], ids[:0]).tolist()[1] == -1.0


def test_local_best_nan_ranks_last():
    """A diverged restart (NaN score) must not poison the exchange (torch.max
    propagates NaN and the winning id became inf)."""
    F = torch.tensor([0.3, float("nan"), 0.7, 0.1], dtype=torch.float64)
    ids = torch.tensor([4, 5, 6, 7])
    assert local_best(F, ids).tolist() == [0.7, 6.0]
    allnan = torch.full((3,), float("nan"), dtype=torch.float64)
    fb, rid = local_best(allnan, torch.tensor([9, 8, 10])).tolist()
    assert fb == float("-inf") and rid == 8.0


def _worker(rank, world, port, n_total, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        first, count = shard(n_total, world, rank)
        ids = torch.arange(first, first + count)
        F = torch.tensor([_score(int(r)) for r in ids], dtype=torch.float64)
        X = torch.stack([_xrow(int(r)) for r in ids]) if count else torch.empty(0, NX, dtype=torch.float64)
        fbest, rid, owner, xb = gather_best(F, ids, X)
        q.put((rank, fbest, rid, owner, xb.tolist()))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,n_total", [(2, 64), (3, 40), (2, 1)])
def test_gather_best_matches_single_process(world, n_total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    scores = [_score(r) for r in range(n_total)]
    best = max(scores)
    rid = scores.index(best)                     # smallest id among ties
    owner = next(r for r in range(world) if shard(n_total, world, r)[0] <= rid
                 < sum(shard(n_total, world, r)))
    for rank, fbest, got_id, got_owner, xb in out:
        assert fbest == best and got_id == rid and got_owner == owner
        assert xb == _xrow(rid).tolist()


# ---------------------------------------------------------------- optimiser sweep (C4 + row f1)
def _opt_worker(rank, world, port, n_total, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank,) + _run_sweep(n_total))
    finally:
        if world > 1:
            dist.destroy_process_group()


def _run_sweep(n_total):
    import numpy as np
    from oracle import grape_oracle as O
    from robustgrape_amd.regularization import regularization_cost_phase
    from robustgrape_amd.sweep import optimize_sweep
    from robustgrape_amd.types import FidelityRobustGRAPEParameters
    from tests import problems as P
    fp = P.sym_problem(24, t0=P.T0_TO, device=False)

    def ev(X):
        outs = [O.calculate_fidelity_and_derivatives(fp, x.numpy()) for x in X]
        t = lambda v: torch.as_tensor(np.asarray(v, dtype=np.float64))
        return (t([o[0] for o in outs]), t(np.stack([o[1] for o in outs])),
                torch.zeros(len(X), 0, dtype=torch.float64), torch.zeros(len(X), X.shape[1], 0, dtype=torch.float64))
    params = FidelityRobustGRAPEParameters(
        x_initial=np.zeros(25), regularization_functions=[regularization_cost_phase],
        regularization_coeff1=[1e-6], regularization_coeff2=[1e-6], error_source_coeff=[], iterations=6)
    cost, rid, owner, xb, _ = optimize_sweep(fp, params, n_total, lambda r: P.random_x(24, 1000 + r, small=True),
                                             evaluate=ev)
    return cost, rid, owner, xb.tolist()


@pytest.mark.parametrize("world,n_total", [(2, 5)])
def test_optimize_sweep_two_ranks_equals_one(world, n_total):
    """The sharded sweep (gloo, 2 ranks) finds the same best restart, cost and pulse as one
    process running every restart: restarts are independent and rows of a batched L-BFGS
    do not interact."""
    single = _run_sweep(n_total)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_opt_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, cost, rid, owner, xb in out:
        assert rid == single[1] and abs(cost - single[0]) < 1e-12
        assert max(abs(a - b) for a, b in zip(xb, single[3])) < 1e-12
