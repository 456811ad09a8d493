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


def _rosen(X, rows=None):
    a, b = X[:, :-1], X[:, 1:]
    f = torch.sum(100 * (b - a * a) ** 2 + (1 - a) ** 2, dim=1)
    g = torch.zeros_like(X)
    g[:, :-1] += -400 * a * (b - a * a) - 2 * (1 - a)
    g[:, 1:] += 200 * (b - a * a)
    return f, g


def test_device_line_search_matches_torch_line_search(monkeypatch):
    """grape_lbfgs_ls_* / grape_lbfgs_step (the state machine as HIP kernels, one sync per round)
    against the torch implementation on the same GPU tensors: the same iterates and call counts
    over the first iterations (row sums reduce in a different order: 1e-12), the same stopping
    behaviour over whole runs, and rows independent of the batch."""
    rng = np.random.default_rng(5)
    X0 = torch.as_tensor(rng.uniform(-2, 2, size=(9, 6)), device="cuda")
    short = {}
    for torch_ls in (False, True):
        monkeypatch.setattr(OPT, "_TORCH_LS", torch_ls)
        res = OPT.lbfgs_batched(_rosen, X0, iterations=4)
        assert bool(res.extra.get("device_ls", False)) == (not torch_ls)
        short[torch_ls] = res
    a, b = short[False], short[True]
    assert torch.equal(a.iterations, b.iterations) and torch.equal(a.f_calls, b.f_calls)
    assert torch.allclose(a.minimizer, b.minimizer, rtol=1e-10, atol=1e-12)
    monkeypatch.setattr(OPT, "_TORCH_LS", False)
    X2 = X0[:, :2].contiguous()  # 2-D: one minimum, at (1, 1) (from 4-D on there is a second one)
    full = OPT.lbfgs_batched(_rosen, X2, iterations=2000, g_tol=1e-8)
    assert bool(full.g_converged.all())
    assert torch.max(torch.abs(full.minimizer - 1)) < 1e-6
    for r in (0, 5):  # a row's run does not depend on its batch
        one = OPT.lbfgs_batched(_rosen, X2[r:r + 1], iterations=2000, g_tol=1e-8)
        assert int(one.iterations[0]) == int(full.iterations[r])
        assert torch.equal(one.minimizer[0], full.minimizer[r])
    # stopping rules: iteration cap, converged at x0
    res = OPT.lbfgs_batched(_rosen, torch.full((2, 4), -1.5, dtype=torch.float64, device="cuda"), iterations=3)
    assert list(res.iterations.cpu()) == [3, 3] and not bool(res.g_converged.any())
    res = OPT.lbfgs_batched(_rosen, torch.ones(1, 4, dtype=torch.float64, device="cuda"))
    assert int(res.iterations[0]) == 0 and bool(res.g_converged[0])


@pytest.mark.parametrize("case", ["sym_err_phase", "dense2_plain"])
def test_fused_cost_matches_torch_cost(case):
    """grape_robust_cost (cost assembly + the reference's regularisers in one launch) against the
    torch assembly of the same engine outputs: error penalty, regularization_cost_phase and
    regularization_cost, two controls per step."""
    from robustgrape_amd import synthetic as S
    if case == "sym_err_phase":
        fp = P.sym_problem(40, errors=("amp", "freq"))
        X = np.stack([P.random_x(40, s) for s in range(5)])
        regs, ce = [REG.regularization_cost_phase], [0.3, 0.7]
    else:
        fp = S.dense_problem(d=6, ntimes=16, dt=0.5, rank=3)
        X = np.stack([S.dense_x(ntimes=16, seed=s) for s in range(5)])
        regs, ce = [REG.regularization_cost, REG.regularization_cost_phase], []
    np_ = len(regs)
    params = FidelityRobustGRAPEParameters(x_initial=X[0], regularization_functions=regs,
                                           regularization_coeff1=[1e-3] * np_, regularization_coeff2=[2e-3] * np_,
                                           error_source_coeff=ce)
    cost = OPT.RobustCost(fp, params, nparam=np_, max_batch=8)
    try:
        assert cost._fused is not None
        Xd = torch.as_tensor(X, device="cuda")
        c_f, g_f = cost(Xd)
        fused, cost._fused = cost._fused, None
        c_t, g_t = cost(Xd)
        cost._fused = fused
    finally:
        cost.close()
    assert torch.allclose(c_f, c_t, rtol=1e-13, atol=1e-15), float((c_f - c_t).abs().max())
    assert torch.allclose(g_f, g_t, rtol=1e-12, atol=1e-14), float((g_f - g_t).abs().max())


@pytest.mark.parametrize("steepest", [False, True])
def test_asynchronous_rows_are_the_synchronous_trajectories(steepest):
    """grape_lbfgs_async_advance: rows advance without waiting for each other at iteration
    boundaries; each row's arithmetic is the synchronous loop's, so iterations, call counts, flags
    and minimisers are bitwise equal (Rosenbrock rows that need very different numbers of line-search
    rounds, and the GRAPE cost of a Rydberg batch)."""
    rng = np.random.default_rng(11)
    X0 = torch.as_tensor(rng.uniform(-2, 2, size=(13, 4)), device="cuda")
    res = {}
    for asy in (False, True):
        res[asy] = OPT.lbfgs_batched(_rosen, X0, iterations=60 if steepest else 300, g_tol=1e-9,
                                     steepest=steepest, asynchronous=asy)
    a, b = res[False], res[True]
    assert torch.equal(a.iterations, b.iterations) and torch.equal(a.f_calls, b.f_calls)
    assert torch.equal(a.minimizer, b.minimizer) and torch.equal(a.minimum, b.minimum)
    for k in ("g_converged", "f_converged", "x_converged", "ls_failed"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k
    if steepest:
        return
    fp = P.sym_problem(60, t0=P.T0_TO)
    Xg = torch.as_tensor(np.stack([P.random_x(60, 2000 + r, small=True) for r in range(7)]), device="cuda")
    params = _params(Xg[0].cpu().numpy(), iterations=15)
    out = {}
    for asy in (False, True):
        cost = OPT.RobustCost(fp, params, nparam=1, max_batch=7)
        try:
            out[asy] = OPT.lbfgs_batched(cost, Xg, iterations=15, g_tol=1e-12, asynchronous=asy)
        finally:
            cost.close()
    a, b = out[False], out[True]
    assert torch.equal(a.iterations, b.iterations) and torch.equal(a.f_calls, b.f_calls)
    assert torch.equal(a.minimizer, b.minimizer)
