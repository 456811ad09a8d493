"""Host logic of the optimiser on the CPU: the regularisers and
the cost assembly against the oracle's restatement of Regularization.jl and
calculate_common! (FidelityCalculations.jl:172-196), the batched L-BFGS on
synthetic objectives, and the reference's optimisation testset
(runtests.jl:356-416) with the oracle standing in for the GPU evaluation."""
import math

import numpy as np
import pytest
import torch

from oracle import grape_oracle as O
from robustgrape_amd import optimize as OPT
from robustgrape_amd import regularization as REG
from robustgrape_amd.types import FidelityRobustGRAPEParameters
from tests import problems as P


def _close(a, b, tol=1e-13):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    assert np.max(np.abs(a - b)) <= tol * max(1.0, np.max(np.abs(b))), np.max(np.abs(a - b))


@pytest.mark.parametrize("n", [4, 5, 9, 200])
def test_regularizers_match_oracle(n):
    rng = np.random.default_rng(n)
    x = rng.normal(size=n)
    for ours, ref in ((REG.regularization_cost(x), O.regularization_cost(x)),
                      (REG.regularization_cost_phase(x), O.regularization_cost_phase(x)),
                      (REG.regularization_cost(x, torch.sin, torch.cos), O.regularization_cost(x, math.sin, math.cos))):
        for a, b in zip(ours, ref):
            _close(a, b)
    # batched rows == the 1-D calls
    X = torch.as_tensor(rng.normal(size=(3, n)))
    r1, j1, r2, j2 = REG.regularization_cost_phase(X)
    for i in range(3):
        ref = O.regularization_cost_phase(X[i].numpy())
        _close(r1[i], ref[0]), _close(j1[i], ref[1]), _close(r2[i], ref[2]), _close(j2[i], ref[3])


def test_regularizer_gradients_are_derivatives():
    x = np.random.default_rng(3).normal(size=12)
    r = O.regularization_cost_phase(x)
    for k, j in ((0, 1), (2, 3)):
        for i in (0, 1, 5, 10, 11):
            e = 1e-6
            xp, xm = x.copy(), x.copy()
            xp[i] += e
            xm[i] -= e
            fd = (O.regularization_cost_phase(xp)[k] - O.regularization_cost_phase(xm)[k]) / (2 * e)
            assert abs(fd - r[j][i]) < 1e-7


def _oracle_eval(fp):
    ne = len(fp.unitary_problem.error_sources)

    def ev(X):
        outs = [O.calculate_fidelity_and_derivatives(fp, x.numpy()) for x in X]
        t = lambda v: torch.as_tensor(np.asarray(v, dtype=np.float64))
        return (t([o[0] for o in outs]), t(np.stack([o[1] for o in outs])),
                t(np.stack([o[2] for o in outs])).reshape(len(X), ne),
                t(np.stack([o[3] for o in outs])).reshape(len(X), X.shape[1], ne))
    return ev


def test_cost_assembly_matches_oracle_with_errors_and_regularizers():
    fp = P.sym_problem(12, errors=("amp", "freq"), device=False)
    params = FidelityRobustGRAPEParameters(
        x_initial=P.random_x(12, 5), regularization_functions=[REG.regularization_cost_phase],
        regularization_coeff1=[1e-3], regularization_coeff2=[2e-3], error_source_coeff=[0.5, 0.25])
    cost = OPT.RobustCost(fp, params, nparam=1, max_batch=2, evaluate=_oracle_eval(fp))
    X = np.stack([P.random_x(12, 5), P.random_x(12, 6)])
    c, g = cost(torch.as_tensor(X))
    for b in range(2):
        ref = O.optimization_cost(fp, X[b], [O.regularization_cost_phase], [1e-3], [2e-3], [0.5, 0.25])
        _close(c[b], ref[0], 1e-14)
        _close(g[b], ref[1:], 1e-14)


def test_cost_two_controls_regularised_per_control():
    """nparam = 2: each control's regulariser gradient lands on its own entries."""
    fp = P.sym_problem(8, device=False)
    X = np.concatenate([np.random.default_rng(1).uniform(size=16), [0.3]])
    params = FidelityRobustGRAPEParameters(
        x_initial=X, regularization_functions=[REG.regularization_cost, REG.regularization_cost_phase],
        regularization_coeff1=[0.1, 0.2], regularization_coeff2=[0.3, 0.4], error_source_coeff=[])
    f64 = dict(dtype=torch.float64)
    zero = lambda Xb: (torch.ones(len(Xb), **f64), torch.zeros(Xb.shape, **f64), torch.zeros(len(Xb), 0, **f64),
                       torch.zeros(Xb.shape[0], Xb.shape[1], 0, **f64))
    c, g = OPT.RobustCost(fp, params, nparam=2, max_batch=1, evaluate=zero)(torch.as_tensor(X[None, :]))
    a = O.regularization_cost(X[0:16:2])
    b = O.regularization_cost_phase(X[1:16:2])
    _close(c[0], 0.1 * a[0] + 0.3 * a[2] + 0.2 * b[0] + 0.4 * b[2])
    _close(g[0, 0:16:2], 0.1 * a[1] + 0.3 * a[3])
    _close(g[0, 1:16:2], 0.2 * b[1] + 0.4 * b[3])
    assert g[0, 16] == 0


def test_shape_assertions():
    fp = P.sym_problem(8, errors=("amp",), device=False)
    params = FidelityRobustGRAPEParameters(
        x_initial=np.zeros(9), regularization_functions=[REG.regularization_cost_phase],
        regularization_coeff1=[0.0], regularization_coeff2=[0.0], error_source_coeff=[])
    with pytest.raises(AssertionError):
        OPT.optimize_fidelity_and_error_sources(fp, params, evaluate=_oracle_eval(fp))


def _rosenbrock(X, rows=None):
    a, b = X[:, :-1], X[:, 1:]
    f = torch.sum(100 * (b - a * a) ** 2 + (1 - a) ** 2, dim=1)
    g = torch.zeros_like(X)
    g[:, :-1] += -400 * a * (b - a * a) - 2 * (1 - a)
    g[:, 1:] += 200 * (b - a * a)
    return f, g


def test_lbfgs_batched_rosenbrock_rows_independent():
    rng = np.random.default_rng(0)
    X0 = torch.as_tensor(rng.uniform(-2, 2, size=(5, 2)))  # 2-D: one minimum, at (1, 1)
    res = OPT.lbfgs_batched(_rosenbrock, X0, iterations=500, g_tol=1e-8)
    assert bool(res.g_converged.all())
    assert torch.max(torch.abs(res.minimizer - 1)) < 1e-6
    for r in (0, 3):
        one = OPT.lbfgs_batched(_rosenbrock, X0[r:r + 1], iterations=500, g_tol=1e-8)
        assert int(one.iterations[0]) == int(res.iterations[r])
        assert torch.allclose(one.minimizer[0], res.minimizer[r], rtol=0, atol=1e-12)


def test_lbfgs_stopping_rules():
    X0 = torch.full((2, 4), -1.5, dtype=torch.float64)
    res = OPT.lbfgs_batched(_rosenbrock, X0, iterations=3)
    assert list(res.iterations) == [3, 3] and not bool(res.g_converged.any())
    res = OPT.lbfgs_batched(_rosenbrock, torch.ones(1, 4, dtype=torch.float64))
    assert int(res.iterations[0]) == 0 and bool(res.g_converged[0])  # converged at x0


def test_reference_optimisation_testset_with_oracle():
    """runtests.jl:356-416: 40 L-BFGS iterations from a small random pulse reach 1-F < 1e-6
    (N = 200, regularization_cost_phase 1e-6/1e-6, f_abstol 1e-11, g_tol 3e-10; numpy seed 42
    replaces Random.seed!(42))."""
    fp = P.sym_problem(200, device=False)
    rng = np.random.default_rng(42)
    x0 = np.concatenate([2 * np.pi * 0.001 * rng.uniform(size=200), [2 * np.pi * rng.uniform()]])
    params = FidelityRobustGRAPEParameters(
        x_initial=x0, regularization_functions=[REG.regularization_cost_phase], regularization_coeff1=[1e-6],
        regularization_coeff2=[1e-6], error_source_coeff=[], iterations=40,
        additional_parameters=dict(f_abstol=1e-11, g_tol=3e-10, show_trace=False))
    res = OPT.optimize_fidelity_and_error_sources(fp, params, evaluate=_oracle_eval(fp))
    F = O.calculate_fidelity_and_derivatives(fp, OPT.minimizer(res))[0]
    assert 1 - F < 1e-6 and res.iterations <= 40


def _small_params(fp, **ap):
    rng = np.random.default_rng(7)
    x0 = np.concatenate([2 * np.pi * 0.01 * rng.uniform(size=fp.unitary_problem.ntimes), [0.3]])
    return FidelityRobustGRAPEParameters(
        x_initial=x0, regularization_functions=[REG.regularization_cost_phase], regularization_coeff1=[1e-6],
        regularization_coeff2=[1e-6], error_source_coeff=[], iterations=6, additional_parameters=ap)


def test_optim_trace_options(capsys):
    """The Optim.Options the reference's examples pass through additional_parameters
    (examples/time_optimal_cz.jl:38-42: show_trace, show_every; FidelityCalculations.jl:211-216):
    Optim's trace table every show_every iterations, store_trace, a stopping callback."""
    fp = P.sym_problem(16, device=False)
    ev = _oracle_eval(fp)
    res = OPT.optimize_fidelity_and_error_sources(
        fp, _small_params(fp, show_trace=True, show_every=2, store_trace=True), evaluate=ev)
    lines = capsys.readouterr().out.splitlines()
    assert lines[0].split() == ["Iter", "Function", "value", "Gradient", "norm"]
    rows = [ln.split() for ln in lines if ln.strip() and ln.split()[0].isdigit()]
    assert [int(r[0]) for r in rows] == list(range(0, res.iterations + 1, 2))
    assert [t["iteration"] for t in res.trace] == list(range(res.iterations + 1))
    assert res.trace[-1]["value"] == pytest.approx(res.minimum, rel=0, abs=0)
    for r, t in zip(rows, res.trace[::2]):
        assert float(r[1]) == pytest.approx(t["value"], rel=1e-6)
    # the callback sees every iteration and can stop the run (Optim: callback returns true)
    seen = []
    res = OPT.optimize_fidelity_and_error_sources(
        fp, _small_params(fp, callback=lambda st: seen.append(st["iteration"]) or st["iteration"] >= 2),
        evaluate=ev)
    assert seen == [0, 1, 2] and res.iterations == 2


def test_optim_options_stopping_and_unknown():
    fp = P.sym_problem(16, device=False)
    ev = _oracle_eval(fp)
    res = OPT.optimize_fidelity_and_error_sources(fp, _small_params(fp, f_calls_limit=3), evaluate=ev)
    assert res.f_calls <= 3 + OPT.MAX_LS_ROUNDS
    big = OPT.optimize_fidelity_and_error_sources(fp, _small_params(fp, g_reltol=0.9), evaluate=ev)
    assert big.g_converged and big.iterations < 6
    with pytest.raises(TypeError, match="unsupported Optim option"):
        OPT.optimize_fidelity_and_error_sources(fp, _small_params(fp, show_tracee=True), evaluate=ev)
    # Julia-style symbol keys and the no-effect options are accepted
    OPT.optimize_fidelity_and_error_sources(fp, _small_params(fp, **{":show_trace": False, "allow_f_increases": True}),
                                            evaluate=ev)


def test_solver_algorithm_is_honoured():
    """FidelityRobustGRAPEParameters.solver_algorithm (Types.jl:82, FidelityCalculations.jl:211-213):
    LBFGS(m) sets the memory, GradientDescent() steps along -g, anything else raises TypeError
    instead of silently running L-BFGS."""
    assert OPT.solver_config("LBFGS") == (10, False)
    assert OPT.solver_config("LBFGS()") == (10, False)
    assert OPT.solver_config(OPT.LBFGS(m=3)) == (3, False)
    assert OPT.solver_config(OPT.GradientDescent) == (1, True)
    assert OPT.solver_config("GradientDescent()") == (1, True)
    for bad in ("BFGS", "ConjugateGradient()", "NelderMead", 42, OPT.LBFGS(m=0)):
        with pytest.raises((TypeError, ValueError)):
            OPT.solver_config(bad)
    fp = P.sym_problem(16, device=False)
    ev = _oracle_eval(fp)
    with pytest.raises(TypeError, match="solver_algorithm"):
        p = _small_params(fp)
        p.solver_algorithm = "ConjugateGradient()"
        OPT.optimize_fidelity_and_error_sources(fp, p, evaluate=ev)
    # GradientDescent: every accepted step is a multiple of -g at the previous iterate
    seen = []
    rec = lambda X, f, g, it: seen.append((X[0].clone(), g[0].clone())) and False  # noqa: E731
    X0 = torch.full((1, 4), -1.2, dtype=torch.float64)
    res = OPT.lbfgs_batched(_rosenbrock, X0, iterations=8, steepest=True, callback=rec)
    assert int(res.iterations[0]) == 8
    for (x0, g0), (x1, _) in zip(seen, seen[1:]):
        step = x1 - x0
        a = -float(step @ g0) / float(g0 @ g0)
        assert a > 0 and torch.max(torch.abs(step + a * g0)) <= 1e-12 * max(1.0, float(torch.max(torch.abs(step))))
    # ... and L-BFGS does not (curvature pairs change the direction after the first step)
    seen.clear()
    OPT.lbfgs_batched(_rosenbrock, X0, iterations=8, callback=rec)
    (x0, g0), (x1, _), (x2, g1) = seen[0], seen[1], seen[2]
    step = x2 - x1
    a = -float(step @ g1) / float(g1 @ g1)
    assert torch.max(torch.abs(step + a * g1)) > 1e-6
    # through the driver: GradientDescent lowers the cost from x_initial; LBFGS(m=3) is m = 3
    p = _small_params(fp)
    p.solver_algorithm = OPT.GradientDescent()
    r_gd = OPT.optimize_fidelity_and_error_sources(fp, p, evaluate=ev)
    c0 = O.optimization_cost(fp, p.x_initial, [O.regularization_cost_phase], [1e-6], [1e-6], [])[0]
    assert r_gd.minimum < c0
    p.solver_algorithm = OPT.LBFGS(m=3)
    r3 = OPT.optimize_restarts(fp, p, p.x_initial[None, :], evaluate=ev)
    r3b = OPT.optimize_restarts(fp, _small_params(fp), p.x_initial[None, :], evaluate=ev, m=3)
    assert torch.equal(r3.minimizer, r3b.minimizer)
