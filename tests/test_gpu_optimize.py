"""The optimiser (FidelityCalculations.jl:161-218) with its
evaluations on the GPU: the cost assembly against the oracle's calculate_common!
restatement, the reference's optimisation testset (runtests.jl:356-416), and
batched restarts equal to independent runs."""
import numpy as np
import pytest
import torch

from robustgrape_amd import optimize as OPT
from robustgrape_amd import regularization as REG
from robustgrape_amd.types import FidelityRobustGRAPEParameters
from tests import problems as P

pytestmark = pytest.mark.gpu
T2, T2_ABS, T3 = 1e-6, 1e-7, 1e-5


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _params(x0, nerr=0, iterations=40, **extra):
    return FidelityRobustGRAPEParameters(
        x_initial=x0, regularization_functions=[REG.regularization_cost_phase], regularization_coeff1=[1e-6],
        regularization_coeff2=[1e-6], error_source_coeff=[0.5] * nerr, iterations=iterations,
        additional_parameters=dict(f_abstol=1e-11, g_tol=3e-10, **extra))


def test_device_cost_matches_oracle_cost():
    from oracle import grape_oracle as O
    fpd = P.sym_problem(50, errors=("amp", "freq"))
    fph = P.sym_problem(50, errors=("amp", "freq"), device=False)
    X = np.stack([P.random_x(50, s) for s in (11, 12, 13)])
    params = _params(X[0], nerr=2)
    cost = OPT.RobustCost(fpd, params, nparam=1, max_batch=3)
    c, g = cost(torch.as_tensor(X, device="cuda"))
    cost.close()
    for b in range(3):
        ref = O.optimization_cost(fph, X[b], [O.regularization_cost_phase], [1e-6], [1e-6], [0.5, 0.5])
        assert abs(float(c[b]) - ref[0]) <= T3 * abs(ref[0]) + 1e-9
        gb = g[b].cpu().numpy()
        assert np.max(np.abs(gb - ref[1:])) <= T3 * np.max(np.abs(ref[1:])) + T2_ABS


def test_reference_optimisation_testset_on_gpu():
    """runtests.jl:356-416: N = 200, 40 L-BFGS iterations from 2pi*0.001*U reach 1 - F < 1e-6."""
    from robustgrape_amd import calculate_fidelity_and_derivatives
    fp = P.sym_problem(200)
    rng = np.random.default_rng(42)
    x0 = np.concatenate([2 * np.pi * 0.001 * rng.uniform(size=200), [2 * np.pi * rng.uniform()]])
    res = OPT.optimize_fidelity_and_error_sources(fp, _params(x0))
    F = calculate_fidelity_and_derivatives(fp, OPT.minimizer(res))[0]
    assert 1 - F < 1e-6 and res.iterations <= 40


def test_batched_restarts_equal_independent_runs():
    """Rows advance independently: a restart's trajectory in a batch of 6 equals its own run
    (deterministic kernels: a batch element is bitwise the single evaluation)."""
    fp = P.sym_problem(100, t0=P.T0_TO)
    X0 = np.stack([P.random_x(100, 1000 + r, small=True) for r in range(6)])
    res = OPT.optimize_restarts(fp, _params(X0[0], iterations=25), X0)
    for r in (0, 4):
        one = OPT.optimize_restarts(fp, _params(X0[r], iterations=25), X0[r:r + 1])
        assert int(one.iterations[0]) == int(res.iterations[r])
        assert torch.equal(one.minimizer[0], res.minimizer[r])
    assert float(torch.min(res.minimum)) < 1e-3


def test_optimise_with_error_sources():
    """examples/time_optimal_cz.jl:60-71 pattern: the error sensitivity joins the cost
    (error_source_coeff); the optimiser lowers that cost and reports it consistently."""
    from robustgrape_amd import calculate_fidelity_and_derivatives
    fp = P.sym_problem(100, t0=P.T0_TO, errors=("amp",))
    x0 = P.random_x(100, 77, small=True)
    params = _params(x0, nerr=1, iterations=30)
    cost = OPT.RobustCost(fp, params, nparam=1, max_batch=1)
    c0 = float(cost(torch.as_tensor(x0[None, :], device="cuda"))[0][0])
    cost.close()
    res = OPT.optimize_fidelity_and_error_sources(fp, params)
    F, _, d2, _ = calculate_fidelity_and_derivatives(fp, res.minimizer)
    reg = REG.regularization_cost_phase(res.minimizer[:100])
    assert res.minimum < c0
    assert abs(res.minimum - (1 - F + 0.5 * d2[0] ** 2 + 1e-6 * (reg[0] + reg[2]))) < 1e-12


def test_optimize_sweep_single_gpu():
    """C4-style sweep on one GPU: the returned best is the batch minimum and its pulse."""
    from robustgrape_amd.sweep import optimize_sweep
    fp = P.sym_problem(100, t0=P.T0_TO)
    params = _params(np.zeros(101), iterations=15)
    cost, rid, owner, xb, res = optimize_sweep(fp, params, 8, lambda r: P.random_x(100, 1000 + r, small=True))
    assert owner == 0 and cost == float(torch.min(res.minimum)) and rid == int(torch.argmin(res.minimum))
    assert torch.equal(xb, res.minimizer[rid])


def test_device_lbfgs_direction_matches_torch_two_loop():
    """grape_lbfgs_direction (one launch) against the batched torch two-loop recursion:
    ragged histories (0..m pairs), wrapped ring-buffer heads, n not a multiple of 256."""
    import torch
    from robustgrape_amd.optimize import _device_direction, _torch_direction
    gen = torch.Generator().manual_seed(3)
    m, R, n = 10, 37, 513
    S = torch.randn(m, R, n, generator=gen, dtype=torch.float64)
    Y = S + 0.3 * torch.randn(m, R, n, generator=gen, dtype=torch.float64)
    rho = 1.0 / (S * Y).sum(-1)
    head = torch.randint(0, m, (R,), generator=gen)
    hist = torch.randint(0, m + 1, (R,), generator=gen)
    hist[0], hist[1] = 0, m
    gamma = torch.rand(R, generator=gen, dtype=torch.float64) + 0.5
    g = torch.randn(R, n, generator=gen, dtype=torch.float64)
    ref = _torch_direction(S, Y, rho, head, hist, gamma, g)
    dev = [t.cuda() for t in (S, Y, rho, head, hist, gamma, g)]
    out = _device_direction(*dev).cpu()
    assert torch.equal(out[0], -gamma[0] * g[0])  # empty history: steepest descent, scaled
    err = (out - ref).abs().max() / ref.abs().max()
    assert err <= 1e-12, float(err)


def test_optimiser_on_closure_problem():
    """a closure problem (the reference's native Types.jl form) takes the host-table
    plan; the optimiser's cost must evaluate through it and equal the operator-basis cost."""
    fpd = P.sym_problem(40, errors=("amp",))
    fph = P.sym_problem(40, errors=("amp",), device=False)
    X = np.stack([P.random_x(40, s) for s in (21, 22)])
    params = _params(X[0], nerr=1)
    costs = []
    for fp in (fpd, fph):
        cost = OPT.RobustCost(fp, params, nparam=1, max_batch=2)
        assert cost.plan.tables == (fp is fph)
        c, g = cost(torch.as_tensor(X, device="cuda"))
        cost.close()
        costs.append((c.cpu().numpy(), g.cpu().numpy()))
    # the cost carries c_e F_d2err^2: an eps-FD quantity (tier T2; the two paths round the
    # sensitivity differently at ~2e-9 relative), not a T1 one
    np.testing.assert_allclose(costs[1][0], costs[0][0], rtol=1e-8, atol=0)
    assert np.max(np.abs(costs[1][1] - costs[0][1])) <= T3 * np.max(np.abs(costs[0][1])) + T2_ABS
    res = OPT.optimize_fidelity_and_error_sources(fph, _params(X[0], nerr=1, iterations=3))
    assert np.isfinite(res.minimum)
