"""Phase-covariant walk classes (csrc/grape_walk.hpp GAUGE, round 5).

When the one control enters H only as a phase -- the laser phase of every Rydberg model of the
reference (RydbergTools.jl:31-130) -- H(x) = D(a x) H(0) D(a x)^dag with D(t) = diag(e^{i t N_j}),
so E_k = D_k exp(-i dt H(0)) D_k^dag exactly and the eps-variant E'_k = D'_k exp(-i dt H(0)) D'_k^dag.
The walks then compute one exponential per lane instead of one per step and variant, and form the
reference's forward difference (E' - E) / eps (UnitaryCalculations.jl:48-56) from the level phases.

Checked here: which plans take it (grape_plan_gauge_info), and that its F / F_dx equal those of the
per-step exponentials (GRAPE_OPT_NO_GAUGE) and the oracle -- F at T1; F_dx at the FD tier of the
problem's step norms (tests/problems.py fd_tier): both sides are forward differences with eps = 1e-8,
so they differ by the u / eps rounding noise of the per-step exponentials, the gauge side carrying
almost none.  The golden C2 / C4 checks inside the bench-size plan (test_gpu_walk.py
test_bench_size_plan_matches_goldens) run the gauge walks too: they are the default.
"""
import numpy as np
import pytest

from tests import problems as P

pytestmark = pytest.mark.gpu
T1 = 1e-12
# gauge walks against the exact (longdouble) forward difference: F_dx relative to max|F_dx| + absolute
T_EXACT = (1e-9, 2e-11)


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _plan(fp, max_batch, options=0, nparam=1):
    from robustgrape_amd.engine import GrapePlan
    return GrapePlan(fp, nparam=nparam, device=0, max_batch=max_batch, options=options)


def _check(test, F, Fdx, F0, g0, tier):
    from tests.parity_log import record
    ef = float(np.max(np.abs(np.asarray(F) - np.asarray(F0))))
    record(test, "F", ef, 1.0, T1)
    assert ef <= T1, (test, ef)
    err, scale = float(np.max(np.abs(Fdx - g0))), float(np.max(np.abs(g0)))
    record(test, "F_dx", err, scale, tier[0] * scale + tier[1])
    print(f"{test}: |dF| {ef:.2e} max|dF_dx| {err:.2e} (scale {scale:.2e}, rel {err / scale:.2e})")
    assert err <= tier[0] * scale + tier[1], (test, err, scale)


def test_which_plans_are_phase_covariant():
    """Every Rydberg model with the phase as its control is, with or without its Rabi / detuning
    error sources; NO_GAUGE, two controls per step and whole matrices are not."""
    from robustgrape_amd.operators import OPT_NO_GAUGE, OPT_NO_SECTORS, OPT_NO_SYMMETRY
    cases = [(P.full9_problem(16), 0, 1, (True, True)), (P.full9_problem(16), OPT_NO_SYMMETRY, 1, (True, True)),
             (P.sym_problem(16), 0, 1, (True,)), (P.fullblk_problem(16), 0, 1, (True,)),
             (P.full9_problem(16), OPT_NO_GAUGE, 1, (False, False)),
             (P.full9_problem(16, nerr=2), 0, 1, (True, True)),   # Rabi / detuning errors: covariant too
             (P.full9_problem(16, nerr=2), OPT_NO_GAUGE, 1, (False, False)),
             (P.full9_problem(16), OPT_NO_SECTORS, 1, (False,))]
    for fp, opts, nparam, want in cases:
        pl = _plan(fp, 4, opts, nparam)
        try:
            assert pl.sector_info()["gauge"] == want, (opts, pl.sectors(), pl.sector_info())
        finally:
            pl.close()


def test_two_controls_per_step_are_not_phase_covariant():
    from tests.test_gpu_walk import _high_norm_problem
    fp = _high_norm_problem(8)[0]  # phase and an amplitude control per step (np = 2)
    pl = _plan(fp, 4, 0, 2)
    try:
        assert not any(pl.sector_info()["gauge"])
    finally:
        pl.close()


@pytest.mark.parametrize("name,fp,opts", [
    ("full9-sym", lambda: P.full9_problem(96), 0),
    ("full9-perm", lambda: P.full9_problem(96), "perm"),
    ("full9-one-step", lambda: P.full9_problem(1), 0),     # |dt H(0)|_1 ~ 76: E~ by Taylor 30 + squarings
    ("full9-chunk-starts", lambda: P.full9_problem(3), 0),
    ("full9-c1-label", lambda: P.full9_problem(256), 0),
    ("sym5", lambda: P.sym_problem(40), 0),
    ("fullblk7", lambda: P.fullblk_problem(40), 0),
])
@pytest.mark.parametrize("batch", [5, 300])
def test_gauge_walks_match_per_step_exponentials_and_oracle(name, fp, opts, batch):
    """Throughput (300: 8-wave scans) and latency-bound (5: 16-wave scans, pair kernels) plans,
    and a single call (the graph path)."""
    from oracle import grape_exact as E
    from oracle import grape_oracle as O
    from robustgrape_amd.operators import OPT_NO_GAUGE, OPT_NO_SYMMETRY
    f = fp()
    nt = f.unitary_problem.ntimes
    rng = np.random.default_rng(77 + nt)
    X = np.stack([P.random_x(nt, 900 + s, small=(s % 2 == 0)) for s in range(batch)])
    X[1, :nt] = rng.uniform(-40.0, 40.0, size=nt)  # large phases: argument reduction in the level phases
    so = OPT_NO_SYMMETRY if opts == "perm" else 0
    pg, pn = _plan(f, batch, so), _plan(f, batch, so | OPT_NO_GAUGE)
    try:
        assert all(pg.sector_info()["gauge"]) and not any(pn.sector_info()["gauge"])
        out, ref = pg.fidelity_grad(X), pn.fidelity_grad(X)
        one = pg.fidelity_grad(X[2:3])
    finally:
        pg.close()
        pn.close()
    assert one[0][0] == out[0][2] and np.array_equal(one[1][0], out[1][2])  # single call == batch row
    for b in range(min(batch, 6)):
        _check(f"gauge_vs_exp_{name}_{batch}_{b}", out[0][b], out[1][b], ref[0][b], ref[1][b], P.fd_tier(f, X[b]))
    for b in (0, 1):
        F0, g0 = O.calculate_fidelity_and_derivatives(f, X[b])[:2]
        Fe, ge = E.fidelity_and_gradient(f, X[b])
        # against the reference's forward difference evaluated without rounding (oracle/grape_exact.py):
        # the phase sandwiches carry no exponential per step, hence none of its u / eps noise
        # (the controls' entries; the x_add entry is the target's forward difference, which the head
        # forms in double like the reference: the FD tier)
        # (absolute floor: the longdouble evaluator's own noise, ~1e-19 2^s / eps with s its squarings)
        floor = T_EXACT[1] * 2.0 ** E.squarings(P.max_step_norm(f, X[b]))
        _check(f"gauge_vs_exact_{name}_{batch}_{b}", out[0][b], out[1][b][:nt], Fe, ge[:nt], (T_EXACT[0], floor))
        _check(f"gauge_vs_exact_add_{name}_{batch}_{b}", out[0][b], out[1][b], Fe, ge, P.fd_tier(f, X[b]))
        # against the oracle: the FD tier plus the oracle's own measured distance from the exact value
        # (the reference's algorithm carries up to 2.3e-7 of max|F_dx| of u / eps noise on small
        # gradients: scripts/probes/fd_exact_probe.py)
        t2, t2a = P.fd_tier(f, X[b])
        _check(f"gauge_vs_oracle_{name}_{batch}_{b}", out[0][b], out[1][b], F0, g0,
               (t2, t2a + float(np.max(np.abs(np.asarray(g0) - ge)))))


def test_gauge_bench_size_plan_against_c2_golden():
    """The bench's configuration (32 768 per pass selects the same kernels as 2 048) with the C2
    golden at scattered positions, and the whole batch against the per-step exponentials."""
    import os
    from robustgrape_amd.operators import OPT_NO_EVAL1, OPT_NO_GAUGE
    g2 = dict(np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c2.npz"),
                      allow_pickle=False))
    n = 2048  # (plans of <= 2 048 take one workgroup per evaluation since round 6: OPT_NO_EVAL1 keeps the walks)
    X = np.stack([P.random_x(512, 5000 + s, small=True) for s in range(n)])
    for p in (0, 777, n - 1):
        X[p] = g2["x"]
    pg, pn = _plan(P.full9_problem(512), n, OPT_NO_EVAL1), _plan(P.full9_problem(512), n, OPT_NO_GAUGE)
    try:
        F, G, _, _ = pg.fidelity_grad(X)
        Fn, Gn, _, _ = pn.fidelity_grad(X)
    finally:
        pg.close()
        pn.close()
    for p in (0, 777, n - 1):
        _check(f"gauge_big_c2_at{p}", F[p], G[p], g2["F"], g2["F_dx"], (1e-7, 1e-9))
    assert float(np.max(np.abs(F - Fn))) <= T1
    err = np.max(np.abs(G - Gn), axis=1)
    scale = np.max(np.abs(Gn), axis=1)
    assert np.all(err <= 1e-7 * scale + 1e-9), float(np.max(err / scale))


def _check_err(test, out, b, ref, tier):
    from tests.test_gpu_walk_err import _check_all
    _check_all(test, out, b, ref, tier, len(ref[1]) - 1)


@pytest.mark.parametrize("name,fp", [
    ("c3", lambda: P.full9_problem(64, nerr=4)),
    ("c3-one-step", lambda: P.full9_problem(1, nerr=4)),
    ("full9-2err", lambda: P.full9_problem(40, nerr=2)),
    ("sym5-amp-freq", lambda: P.sym_problem(24, errors=("amp", "freq"))),
    ("fullblk7-amp-freq", lambda: P.fullblk_problem(24, errors=("amp", "freq"))),
])
@pytest.mark.parametrize("batch", [3, 300])
def test_gauge_image_walk_matches_per_step_exponentials_and_oracle(name, fp, batch):
    """Error sources on phase-covariant classes (round 6: the lab-frame walks k_walk_wsum_lab /
    k_walk_err_lab; k_walk_img_gauge with GRAPE_WALK_ERR_LAB=0): F, F_dx, F_d2err,
    F_d2err_dx against the per-step image walk (GRAPE_OPT_NO_GAUGE) and the oracle
    (UnitaryCalculations.jl:66-151, FidelityCalculations.jl:78-117); the mixed stencil is formed without
    its four-term cancellation, so the comparison carries the per-step side's eps2 noise (T3 tier).
    Batches of 3 (latency scans, 128 / 256 chunks) and 300 (4-wave scans); the throughput chunking
    (one-wave scans, 6 / 8 chunks) runs in test_gpu_walk.py test_bench_size_plan_c3_golden."""
    from oracle import grape_oracle as O
    from robustgrape_amd.operators import OPT_NO_GAUGE
    f = fp()
    nt = f.unitary_problem.ntimes
    X = np.stack([P.random_x(nt, 1300 + s, small=(s % 2 == 1)) for s in range(batch)])
    pg, pn = _plan(f, batch), _plan(f, batch, OPT_NO_GAUGE)
    try:
        assert all(pg.sector_info()["gauge"]) and not any(pn.sector_info()["gauge"])
        out, ref = pg.fidelity_grad(X), pn.fidelity_grad(X)
        one = pg.fidelity_grad(X[1:2])
    finally:
        pg.close()
        pn.close()
    assert one[0][0] == out[0][1] and np.array_equal(one[1][0], out[1][1])
    assert np.array_equal(one[3][0], out[3][1])
    for b in range(min(batch, 4)):
        _check_err(f"gauge_img_vs_exp_{name}_{batch}_{b}", out, b, tuple(o[b] for o in ref), P.fd_tier(f, X[b]))
    for b in (0, 1):
        ro = O.calculate_fidelity_and_derivatives(f, X[b])
        _check_err(f"gauge_img_vs_oracle_{name}_{batch}_{b}", out, b, ro, P.fd_tier(f, X[b]))


@pytest.mark.parametrize("n", [2048, 4100])
def test_merged_walks_match_per_class_walks(n):
    """Throughput passes walk both sector classes of an (evaluation, chunk) in one lane
    (grape_walk.hpp k_walk_fwd_m / k_walk_grad_m) at the per-class walks' chunking and scan the chunk
    totals one lane per evaluation (k_scan_seq); with GRAPE_OPT_NO_MERGE the same chunking runs one
    walk kernel per class and the Hillis-Steele scan: the same per-step arithmetic, the chain
    associated differently, so F to T1 and F_dx to 1e-11 of max|F_dx| (4 100: a ragged last
    workgroup).  Against the per-step exponentials at the FD tier, and the C2 golden inside the
    batch."""
    import os
    from robustgrape_amd.operators import OPT_NO_EVAL1, OPT_NO_GAUGE, OPT_NO_MERGE
    g2 = dict(np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c2.npz"),
                      allow_pickle=False))
    f = P.full9_problem(512)
    X = np.stack([P.random_x(512, 7000 + s, small=(s % 3 != 0)) for s in range(n)])
    X[5] = g2["x"]
    pm, pu, pn = (_plan(f, n, OPT_NO_EVAL1), _plan(f, n, OPT_NO_MERGE | OPT_NO_EVAL1),  # (the throughput walks)
                  _plan(f, n, OPT_NO_GAUGE))
    try:
        F, G, _, _ = pm.fidelity_grad(X)
        Fu, Gu, _, _ = pu.fidelity_grad(X)
        Fn, Gn, _, _ = pn.fidelity_grad(X[:64])
    finally:
        pm.close()
        pu.close()
        pn.close()
    assert float(np.max(np.abs(F - Fu))) <= T1
    err_u = np.max(np.abs(G - Gu), axis=1)
    assert np.all(err_u <= 1e-11 * np.max(np.abs(Gu), axis=1) + 1e-13), float(np.max(err_u))
    _check(f"merged_c2_golden_{n}", F[5], G[5], g2["F"], g2["F_dx"], (1e-7, 1e-9))
    assert float(np.max(np.abs(F[:64] - Fn))) <= T1
    err = np.max(np.abs(G[:64] - Gn), axis=1)
    scale = np.max(np.abs(Gn), axis=1)
    assert np.all(err <= 1e-7 * scale + 1e-9), float(np.max(err / scale))
