"""Device-pointer calls (grape_fidelity_grad_device_async, the optimiser's line-search rounds) against
the host-array entry on the same plan (grape_fidelity_grad: captured graphs for <= 64 evaluations,
the stream path above), bitwise: fresh output tensors per call, row counts through and past the
graph limit, error sources (F_d2err, F_d2err_dx).  And the optimiser's cost (RobustCost) on a few
rows equals the same rows inside a large call, bitwise, through the fused cost and the torch cost.

(Round 4 also replayed small device-pointer calls from captured graphs; it measured no faster than
the stream path -- 0.104 vs 0.100 ms for one row, scripts/probes/cost_call_latency.py -- and was
removed.)"""
import numpy as np
import pytest

from tests import problems as P

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _call(plan, X, ne):
    import torch
    dev = torch.device("cuda", 0)
    Xd = torch.as_tensor(np.ascontiguousarray(X), device=dev)
    r, nx = X.shape
    nan = float("nan")
    F = torch.full((r,), nan, dtype=torch.float64, device=dev)
    Fdx = torch.full((r, nx), nan, dtype=torch.float64, device=dev)
    Fd2 = torch.full((r, max(1, ne)), nan, dtype=torch.float64, device=dev)
    Fd2dx = torch.full((r, max(1, ne), nx), nan, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    plan.fidelity_grad_device_async(Xd.data_ptr(), F.data_ptr(), Fdx.data_ptr(), r,
                                    Fd2.data_ptr() if ne else 0, Fd2dx.data_ptr() if ne else 0)
    plan.synchronize()
    out = [F.cpu().numpy(), Fdx.cpu().numpy()]
    if ne:
        out += [Fd2.cpu().numpy(), Fd2dx.cpu().numpy()]
    return out


CASES = [
    ("c2", lambda: P.full9_problem(512), 0, (1, 3, 4, 7, 16, 33, 64, 100, 2, 1)),
    ("c3", lambda: P.full9_problem(64, nerr=4), 4, (1, 5, 8, 3, 100, 1)),
    ("sym5", lambda: P.sym_problem(40), 0, (1, 2, 13, 64, 1)),
]


@pytest.mark.parametrize("name,mk,ne,sizes", CASES)
def test_device_calls_are_the_host_calls(name, mk, ne, sizes):
    from robustgrape_amd.engine import GrapePlan
    fp = mk()
    nt = fp.unitary_problem.ntimes
    X = np.stack([P.random_x(nt, 300 + s) for s in range(128)])
    plan = GrapePlan(fp, nparam=1, device=0, max_batch=128)
    try:
        for i, nb in enumerate(sizes):
            rows = X[(5 * i) % 20:(5 * i) % 20 + nb]
            got = _call(plan, rows, ne)
            F, Fdx, Fd2, Fd2dx = plan.fidelity_grad(rows)
            want = [F, Fdx] + ([Fd2, np.ascontiguousarray(Fd2dx.transpose(0, 2, 1))] if ne else [])
            for g, w in zip(got, want):
                assert np.all(np.isfinite(g)), (name, nb)
                assert np.array_equal(g, w), (name, nb, float(np.max(np.abs(g - w))))
    finally:
        plan.close()


@pytest.mark.parametrize("fused", [True, False])
def test_robust_cost_small_rounds_match_large_round(fused):
    """The optimiser's cost on a few rows (device graph) equals the same rows inside a large call
    (stream path) bitwise, through the fused cost (grape_robust_cost: one regulariser per control)
    and the torch cost (no regulariser)."""
    import torch

    from robustgrape_amd import optimize as OPT
    from robustgrape_amd import regularization as REG
    from robustgrape_amd.types import FidelityRobustGRAPEParameters
    fp = P.full9_problem(128)
    X = torch.as_tensor(np.stack([P.random_x(128, 70 + s) for s in range(96)]), device="cuda:0")
    regs = [REG.regularization_cost_phase] if fused else []
    params = FidelityRobustGRAPEParameters(x_initial=X[0].cpu().numpy(), regularization_functions=regs,
                                           regularization_coeff1=[1e-7] * len(regs),
                                           regularization_coeff2=[1e-7] * len(regs), error_source_coeff=[])
    cost = OPT.RobustCost(fp, params, nparam=1, max_batch=96, device=0)
    assert (cost._fused is not None) == fused
    try:
        c_all, g_all = cost(X)
        for r0, n in ((0, 1), (7, 5), (40, 33)):
            c, g = cost(X[r0:r0 + n])
            assert torch.equal(c, c_all[r0:r0 + n]) and torch.equal(g, g_all[r0:r0 + n])
    finally:
        cost.close()
