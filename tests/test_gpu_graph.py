"""The host-array entry grape_fidelity_grad replays small batches (<= 64 evaluations: the
reference's one-x-per-call Optim pattern, FidelityCalculations.jl:177) as captured HIP graphs.
The replay must give exactly the stream path's numbers, for every batch size, across the
graph cache's eviction, for error sources and for the dense engine."""
import numpy as np
import pytest

from robustgrape_amd import synthetic as S
from tests import problems as P

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _plan(fp, nparam, max_batch):
    from robustgrape_amd.engine import GrapePlan
    return GrapePlan(fp, nparam=nparam, device=0, max_batch=max_batch)


@pytest.mark.parametrize("nerr", [0, 2])
def test_graph_replay_equals_stream_path(nerr):
    fp = P.full9_problem(40, nerr=nerr)
    X = np.stack([P.random_x(40, s) for s in range(80)])
    plan = _plan(fp, 1, 128)
    try:
        ref = plan.fidelity_grad(X)        # 80 > 64: the stream path, one launch sequence
        for nb in (1, 2, 3, 5, 7, 11, 13, 17, 64, 1, 3):  # > 8 sizes: the cache evicts and recaptures
            out = plan.fidelity_grad(X[:nb])
            for a, r in zip(out, ref):
                assert np.array_equal(a, r[:nb]), nb
        for b in (0, 41, 79):             # single evaluations, replayed
            out = plan.fidelity_grad(X[b:b + 1])
            for a, r in zip(out, ref):
                assert np.array_equal(a, r[b:b + 1])
    finally:
        plan.close()


def test_graph_replay_dense_engine():
    fp = S.dense_error_problem(16, 5, rank=13, nerr=1)
    X = np.stack([S.dense_x(5, seed=s) for s in range(3)])
    plan = _plan(fp, 2, 4)
    try:
        ref = [plan.fidelity_grad(X[b:b + 1]) for b in range(3)]
        again = [plan.fidelity_grad(X[b:b + 1]) for b in range(3)]
        for r, a in zip(ref, again):
            for u, v in zip(r, a):
                assert np.array_equal(u, v)
        from oracle import grape_oracle as O
        F0 = O.calculate_fidelity_and_derivatives(fp, X[1])[0]
        assert abs(ref[1][0][0] - F0) < 1e-12
    finally:
        plan.close()
