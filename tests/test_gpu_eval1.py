"""One workgroup per evaluation (csrc/grape_eval1.hip, round 5): latency-bound plans of the Rydberg
sector layout (one 3-level and two 2-level phase-covariant classes) run each evaluation --
propagators, chain scan, head, gradient -- inside one workgroup.

Checked: which plans take it (grape_plan_eval1), that its F / F_dx equal the pair-kernel pipeline's
(GRAPE_OPT_NO_EVAL1: the same per-step arithmetic, the chain products associated differently, so
to rounding -- T_PAIR -- not bit for bit), the exact forward difference (oracle/grape_exact.py) at
the phase-covariant tier of test_gpu_gauge.py, the goldens, that a single evaluation equals the same
evaluation inside any batch bit for bit (one workgroup each), and that the host-array call (mapped
pinned buffers) equals the device-pointer call bit for bit.  Reference: FidelityCalculations.jl:19-119,
UnitaryCalculations.jl:44-56.
"""
import os

import numpy as np
import pytest

from tests import problems as P

pytestmark = pytest.mark.gpu
T1 = 1e-12
# eval1 vs the pair pipeline: F absolute; F_dx relative to max|F_dx| plus an absolute floor
T_PAIR = (1e-13, 1e-11, 1e-13)
T_EXACT = (1e-9, 2e-11)


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _plan(fp, max_batch, options=0, nparam=1):
    from robustgrape_amd.engine import GrapePlan
    return GrapePlan(fp, nparam=nparam, device=0, max_batch=max_batch, options=options)


def _inputs(nt, n, seed):
    rng = np.random.default_rng(seed)
    X = np.stack([P.random_x(nt, seed * 1000 + s, small=(s % 2 == 0)) for s in range(n)])
    if n > 1:
        X[1, :nt] = rng.uniform(-40.0, 40.0, size=nt)  # large phases: argument reduction
    return X


def _record(test, what, err, scale, tol):
    from tests.parity_log import record
    record(test, what, err, scale, tol)


def test_which_plans_run_one_workgroup_per_evaluation():
    from robustgrape_amd.operators import OPT_NO_EVAL1, OPT_NO_GAUGE, OPT_NO_SYMMETRY
    cases = [(P.full9_problem(64), 1, 0, True), (P.full9_problem(64), 256, 0, True),
             (P.full9_problem(64), 2048, 0, True),            # round 6: up to 2 048 (GRAPE_EVAL1_MAX_BATCH)
             (P.full9_problem(64), 2049, 0, False),           # a throughput plan: the walks
             (P.full9_problem(64), 8, OPT_NO_EVAL1, False),
             (P.full9_problem(64), 8, OPT_NO_GAUGE, False),   # per-step exponentials: the pair kernels
             (P.full9_problem(64), 8, OPT_NO_SYMMETRY, False),  # 4-level permutation sectors
             (P.full9_problem(64, nerr=2), 8, 0, False),      # error sources
             (P.full9_problem(2048), 8, 0, True), (P.full9_problem(2049), 8, 0, False)]
    for fp, mb, opts, want in cases:
        pl = _plan(fp, mb, opts)
        try:
            assert pl.sector_info()["eval1"] == want, (mb, opts, fp.unitary_problem.ntimes, pl.sector_info())
        finally:
            pl.close()


def _kernel_launches(pl, X):
    pl.set_profiling(True)
    pl.kernel_times(reset=True)
    out = pl.fidelity_grad(X)
    kt = pl.kernel_times(reset=True)
    pl.set_profiling(False)
    return out, kt


def test_profiled_call_runs_the_one_kernel():
    fp = P.full9_problem(512)
    X = _inputs(512, 4, 3)
    pl = _plan(fp, 4)
    try:
        out, kt = _kernel_launches(pl, X)
        ref = pl.fidelity_grad(X)  # (the unprofiled host path: mapped pinned buffers)
    finally:
        pl.close()
    assert kt["k_eval1"][1] == 1
    assert sum(n for k, (_, n) in kt.items() if k != "k_eval1") == 0, kt
    assert np.array_equal(out[0], ref[0]) and np.array_equal(out[1], ref[1])


@pytest.mark.parametrize("nt", [1, 2, 3, 255, 256, 257, 512, 1000, 2048])
def test_eval1_matches_pair_pipeline_exact_and_oracle(nt):
    """Every chunking regime: fewer steps than lanes (one step per lane, idle lanes), L = 2 .. 8,
    a ragged last chunk (257, 1000)."""
    from oracle import grape_exact as E
    from oracle import grape_oracle as O
    from robustgrape_amd.operators import OPT_NO_EVAL1
    fp = P.full9_problem(nt)
    n = 5
    X = _inputs(nt, n, 40 + nt)
    pe, pp = _plan(fp, n), _plan(fp, n, OPT_NO_EVAL1)
    try:
        assert pe.sector_info()["eval1"] and not pp.sector_info()["eval1"]
        out, ref = pe.fidelity_grad(X), pp.fidelity_grad(X)
    finally:
        pe.close()
        pp.close()
    ef = float(np.max(np.abs(out[0] - ref[0])))
    _record(f"eval1_vs_pair_nt{nt}", "F", ef, 1.0, T_PAIR[0])
    assert ef <= T_PAIR[0], ef
    for b in range(n):
        err, scale = float(np.max(np.abs(out[1][b] - ref[1][b]))), float(np.max(np.abs(ref[1][b])))
        tol = T_PAIR[1] * scale + T_PAIR[2]
        _record(f"eval1_vs_pair_nt{nt}_{b}", "F_dx", err, scale, tol)
        assert err <= tol, (b, err, scale)
    for b in (0, 1):
        if nt > 600 and b == 1:
            continue  # (the longdouble evaluator's cost)
        Fe, ge = E.fidelity_and_gradient(fp, X[b])
        assert abs(out[0][b] - Fe) <= T1
        floor = T_EXACT[1] * 2.0 ** E.squarings(P.max_step_norm(fp, X[b]))
        err = float(np.max(np.abs(out[1][b][:nt] - ge[:nt])))
        scale = float(np.max(np.abs(ge[:nt])))
        _record(f"eval1_vs_exact_nt{nt}_{b}", "F_dx", err, scale, T_EXACT[0] * scale + floor)
        assert err <= T_EXACT[0] * scale + floor, (b, err, scale)
        # the x_add entry: the target's forward difference formed in double, as the reference (and
        # the pair pipeline's head) does -- no farther from the exact value than the pair pipeline's
        assert abs(out[1][b][nt] - ge[nt]) <= abs(ref[1][b][nt] - ge[nt]) + 1e-12
        t2, t2a = P.fd_tier(fp, X[b])
        if nt <= 256:
            F0, g0 = O.calculate_fidelity_and_derivatives(fp, X[b])[:2]
            assert abs(out[0][b] - F0) <= T1
            tol = t2 * float(np.max(np.abs(g0))) + t2a + float(np.max(np.abs(np.asarray(g0) - ge)))
            assert float(np.max(np.abs(out[1][b] - g0))) <= tol


def test_single_evaluation_equals_batch_rows_bitwise():
    fp = P.full9_problem(512)
    X = _inputs(512, 256, 9)
    pl = _plan(fp, 256)
    try:
        F, G, _, _ = pl.fidelity_grad(X)
        for b in (0, 1, 77, 255):
            f1, g1, _, _ = pl.fidelity_grad(X[b:b + 1])
            assert f1[0] == F[b] and np.array_equal(g1[0], G[b]), b
        f3, g3, _, _ = pl.fidelity_grad(X[10:13])
        assert np.array_equal(f3, F[10:13]) and np.array_equal(g3, G[10:13])
    finally:
        pl.close()


def test_device_pointer_call_equals_host_call_bitwise():
    import torch
    fp = P.full9_problem(512)
    X = _inputs(512, 32, 11)
    pl = _plan(fp, 32)
    try:
        F, G, _, _ = pl.fidelity_grad(X)
        xd = torch.from_numpy(X).to("cuda:0")
        Fd = torch.empty(32, dtype=torch.float64, device="cuda:0")
        Gd = torch.empty((32, X.shape[1]), dtype=torch.float64, device="cuda:0")
        torch.cuda.synchronize()
        pl.fidelity_grad_device_async(xd.data_ptr(), Fd.data_ptr(), Gd.data_ptr(), 32)
        pl.synchronize()
        assert np.array_equal(Fd.cpu().numpy(), F) and np.array_equal(Gd.cpu().numpy(), G)
    finally:
        pl.close()


def test_c2_golden_through_one_workgroup():
    g2 = dict(np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c2.npz"),
                      allow_pickle=False))
    pl = _plan(P.full9_problem(512), 1)
    try:
        assert pl.sector_info()["eval1"]
        F, G, _, _ = pl.fidelity_grad(g2["x"][None, :])
    finally:
        pl.close()
    err, scale = float(np.max(np.abs(G[0] - g2["F_dx"]))), float(np.max(np.abs(g2["F_dx"])))
    _record("eval1_c2_golden", "F_dx", err, scale, 1e-7 * scale + 1e-9)
    assert abs(F[0] - g2["F"]) <= T1
    assert err <= 1e-7 * scale + 1e-9, (err, scale)


def test_c4_restart_sweep_point_matches_pair_pipeline():
    """The C4 latency point (32 restarts per GPU): one call of 32 evaluations."""
    from robustgrape_amd.operators import OPT_NO_EVAL1
    fp = P.full9_problem(512)
    X = _inputs(512, 32, 21)
    pe, pp = _plan(fp, 32), _plan(fp, 32, OPT_NO_EVAL1)
    try:
        out, ref = pe.fidelity_grad(X), pp.fidelity_grad(X)
    finally:
        pe.close()
        pp.close()
    assert float(np.max(np.abs(out[0] - ref[0]))) <= T_PAIR[0]
    err = np.max(np.abs(out[1] - ref[1]), axis=1)
    scale = np.max(np.abs(ref[1]), axis=1)
    assert np.all(err <= T_PAIR[1] * scale + T_PAIR[2]), float(np.max(err / scale))
