"""Chunk walks (robustgrape_amd/csrc/grape_walk.hpp) and the kernel configurations the bench times.

The walks serve the sector classes of <= 4 levels without error sources (the Rydberg C1 / C2 /
C4 problems): one lane per (sub-evaluation, chunk) recomputes the propagators of its chunk, once
for the chunk total and once for the gradient walk X <- E X E^dag with the eps-variants
contracted on the spot (UnitaryCalculations.jl:44-56, FidelityCalculations.jl:54-76).

Bench-size plans: the bench evaluates 32 768 evaluations per device pass; a plan of
max_batch >= 2048 already selects the same kernel configuration (one-wave k_scan<S,1> /
k_err_scan<S,1> once the sub-evaluations reach 8 x CUs, the walks' 16 chunks of 32 steps at
S = 4 and 32 chunks of 16 steps at S = 2), so these plans are checked against the goldens
(C2, C4 and C3) and the oracle -- with the walks and with the round-2 stored-intermediate
kernels (GRAPE_OPT_NO_WALK: k_expm_chain_lane's 16-step chunk chains, k_expm_grad), including
high-norm steps inside multi-step chunks (the walks' scaling-and-squaring path; the
stored-intermediate path's parked steps, NaN-poisoned chunk chains and k_scan's rechain)."""
import os

import numpy as np
import pytest

from tests import problems as P

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
T1 = 1e-12
T2, T2_ABS = 1e-6, 1e-7
T2S, T2S_ABS = 1e-7, 1e-9
T3, T3_ABS, T3_XADD_ABS = 1e-5, 1e-7, 1e-5
BIG = 2048  # >= 8 x 256 CUs sub-evaluations: the bench's kernel configuration


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _golden(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


def _plan(fp, max_batch, options=0, nparam=1):
    from robustgrape_amd.engine import GrapePlan
    return GrapePlan(fp, nparam=nparam, device=0, max_batch=max_batch, options=options)


def _check(test, F, Fdx, F0, g0, tight):
    """tight: True (T2s), False (T2) or a (relative, absolute) pair (tests/problems.py fd_tier)."""
    from tests.parity_log import record
    if isinstance(tight, tuple):
        t2, t2a = tight
    else:
        t2, t2a = (T2S, T2S_ABS) if tight else (T2, T2_ABS)
    ef = abs(float(F) - float(F0))
    record(test, "F", ef, 1.0, T1)
    assert ef <= T1, (test, F, F0)
    err, scale = float(np.max(np.abs(Fdx - g0))), float(np.max(np.abs(g0)))
    record(test, "F_dx", err, scale, t2 * scale + t2a)
    print(f"{test}: |dF| {ef:.2e}  max|dF_dx| {err:.2e} (scale {scale:.2e}, rel {err / scale:.2e})")
    assert err <= t2 * scale + t2a, (test, err, scale)


@pytest.mark.parametrize("name,fp,layout", [
    ("full9", lambda: P.full9_problem(40), P.FULL9_SYM),
    ("full9-one-step", lambda: P.full9_problem(1), P.FULL9_SYM),
    ("full9-chunk-starts", lambda: P.full9_problem(3), P.FULL9_SYM),
    ("full9-c1-label", lambda: P.full9_problem(256), P.FULL9_SYM),  # |dt H|_1 = 0.327: Taylor 30, no squaring
    ("full9-perm", lambda: P.full9_problem(40), P.FULL9_PERM),
    ("full9-one-step-perm", lambda: P.full9_problem(1), P.FULL9_PERM),
    ("full9-chunk-starts-perm", lambda: P.full9_problem(3), P.FULL9_PERM),
    ("sym5", lambda: P.sym_problem(24), ((2, 2),)),
    ("fullblk7", lambda: P.fullblk_problem(24), ((2, 3),)),
    ("c1-evered", lambda: P.sym_problem(1000), ((2, 2),)),
])
def test_walk_matches_oracle_and_stored_path(name, fp, layout):
    """Walks vs the oracle and vs the stored-intermediate sector kernels (GRAPE_OPT_NO_WALK); -perm:
    the permutation sectors (GRAPE_OPT_NO_SYMMETRY: the 4-level walk), else the symmetry-adapted ones."""
    from oracle import grape_oracle as O
    from robustgrape_amd.operators import OPT_NO_SYMMETRY, OPT_NO_WALK
    f = fp()
    nt = f.unitary_problem.ntimes
    X = np.stack([P.evered_pulse(nt) if name == "c1-evered" and s == 0 else P.random_x(nt, 700 + s)
                  for s in range(5)])
    so = OPT_NO_SYMMETRY if name.endswith("-perm") else 0
    pw, ps = _plan(f, len(X), so), _plan(f, len(X), OPT_NO_WALK | so)
    try:
        assert pw.sectors() == layout
        out, ref = pw.fidelity_grad(X), ps.fidelity_grad(X)
    finally:
        pw.close()
        ps.close()
    for b in range(len(X)):
        tier = P.fd_tier(f, X[b])  # long steps: the scaled T2 tier (tests/problems.py fd_tier)
        _check(f"walk_vs_stored_{name}_{b}", out[0][b], out[1][b], ref[0][b], ref[1][b], tier)
    for b in (0, 3):
        F0, g0 = O.calculate_fidelity_and_derivatives(f, X[b])[:2]
        tier = P.fd_tier(f, X[b])
        if name == "c1-evered" and b == 0:  # at the optimum max|F_dx| ~ 2e-4: the absolute FD floor
            tier = (tier[0], 1e-8)         # u / eps ~ 1.1e-8 of the reference itself decides
        _check(f"walk_vs_oracle_{name}_{b}", out[0][b], out[1][b], F0, g0, tier)
    if name == "c1-evered":  # runtests.jl:115-165 known answer through the walks
        assert out[0][0] > 0.9999 and abs(out[0][0] - 0.999996184760959) < 1e-12


@pytest.mark.parametrize("walk,sym", [(True, True), (True, False), (False, True)])
def test_bench_size_plan_matches_goldens(walk, sym):
    """C2 and C4 goldens inside one 2 048-evaluation launch (the bench's kernel configuration),
    at scattered batch positions, with the walks (symmetry-adapted sectors, the bench's default,
    and the permutation sectors) and with the round-2 stored-intermediate path."""
    from robustgrape_amd.operators import OPT_NO_EVAL1, OPT_NO_SYMMETRY, OPT_NO_WALK
    g2, g4 = _golden("c2"), _golden("c4")
    rng = np.random.default_rng(5)
    X = np.stack([P.random_x(512, 3000 + s, small=True) for s in range(BIG)])
    pos2 = [0, 1023, BIG - 1]
    pos4 = [17, 640, 1500, 2046]
    for p in pos2:
        X[p] = g2["x"]
    for j, p in enumerate(pos4):
        X[p] = g4["x"][j]
    # (OPT_NO_EVAL1: plans of <= 2 048 run one workgroup per evaluation since round 6; the bench's
    # throughput passes take the walks)
    opts = (0 if walk else OPT_NO_WALK) | (0 if sym else OPT_NO_SYMMETRY) | OPT_NO_EVAL1
    pl = _plan(P.full9_problem(512), BIG, opts)
    try:
        assert pl.sectors() == (P.FULL9_SYM if sym else P.FULL9_PERM)
        F, Fdx, _, _ = pl.fidelity_grad(X)
    finally:
        pl.close()
    tag = ("walk" if walk else "stored") + ("" if sym else "_perm")
    for p in pos2:
        _check(f"big_{tag}_c2_at{p}", F[p], Fdx[p], g2["F"], g2["F_dx"], tight=True)
    for j, p in enumerate(pos4):
        _check(f"big_{tag}_c4_{j}_at{p}", F[p], Fdx[p], g4["F"][j], g4["F_dx"][j], tight=True)
    # the rest of the batch: rows are independent and deterministic -> a re-run of a slice in a
    # small plan (other kernel widths) agrees at the T2s tier
    idx = rng.choice(BIG, size=6, replace=False)
    small = _plan(P.full9_problem(512), 8, opts)
    try:
        Fs, gs, _, _ = small.fidelity_grad(X[idx])
    finally:
        small.close()
    for j, b in enumerate(idx):
        _check(f"big_{tag}_vs_small_{b}", F[b], Fdx[b], Fs[j], gs[j], P.fd_tier(P.full9_problem(512), X[b]))


def test_bench_size_plan_c3_golden():
    """C3 (4 error sources) at a 2 048-evaluation pass: k_err_scan<S,1> and the sector error path."""
    from tests.parity_log import record
    g = _golden("c3")
    fp = P.full9_problem(512, nerr=4)
    X = np.stack([P.random_x(512, 5000 + s, small=True) for s in range(BIG)])
    pos = [3, 1111, BIG - 1]
    for p in pos:
        X[p] = g["x"]
    pl = _plan(fp, BIG)
    try:
        F, Fdx, d2, d2dx = pl.fidelity_grad(X)
    finally:
        pl.close()
    nmain = 512
    from tests.xadd_pin import check_xadd, exact_rows
    xe = exact_rows(fp, g["x"])
    for p in pos:
        _check(f"big_c3_at{p}", F[p], Fdx[p], g["F"], g["F_dx"], tight=True)
        e0, s0 = np.max(np.abs(d2[p] - g["F_d2err"])), np.max(np.abs(g["F_d2err"]))
        record(f"big_c3_at{p}", "F_d2err", e0, s0, T3 * s0 + T3_ABS)
        assert e0 <= T3 * s0 + T3_ABS
        err, sc = np.max(np.abs(d2dx[p][:nmain] - g["F_d2err_dx"][:nmain])), np.max(np.abs(g["F_d2err_dx"][:nmain]))
        record(f"big_c3_at{p}", "F_d2err_dx", err, sc, T3 * sc + T3_ABS)
        assert err <= T3 * sc + T3_ABS
        # the x_add rows against their exact value (tests/xadd_pin.py), the golden within T3 plus its
        # own distance from exact (the reference's stencil residue)
        check_xadd(f"big_c3_at{p}", d2dx[p], g["F_d2err_dx"], nmain, xe)


def _high_norm_problem(nt):
    """C2's model plus a detuning control on the Rydberg levels (n_p = 2): x[1, k] = +-900 at a few
    steps gives |dt H|_1 ~ 27 there (Pade 13 with squarings in the reference; the walks' scaling
    and squaring), every other step is C2's ordinary low-norm step."""
    from robustgrape_amd import rydberg as R
    from robustgrape_amd.operators import FN_LINEAR, VAR_X, OperatorBasisHamiltonian, Term
    from robustgrape_amd.types import FidelityRobustGRAPEProblem, UnitaryRobustGRAPEProblem
    Nr = np.diag([0, 0, 0, 0, 1, 1, 1, 1, 2]).astype(np.complex128)
    H0 = OperatorBasisHamiltonian(list(R.rydberg_full_operator_basis().terms)
                                  + [Term(Nr, var=VAR_X, index=1, func=FN_LINEAR)])
    up = UnitaryRobustGRAPEProblem(t0=P.T0_TO, ntimes=nt, ndim=9, H0=H0, nb_additional_param=1)
    fp = FidelityRobustGRAPEProblem(up, P.W_FULL9, R.cz_full_target())
    Hc = lambda t, x, xa: H0(t, x, xa)  # noqa: E731
    fo = FidelityRobustGRAPEProblem(UnitaryRobustGRAPEProblem(t0=P.T0_TO, ntimes=nt, ndim=9, H0=Hc,
                                                              nb_additional_param=1),
                                    P.W_FULL9, lambda xa: R.cz_with_1q_phase_full(xa[0]))
    return fp, fo


@pytest.mark.parametrize("walk", [True, False])
def test_high_norm_steps_inside_long_chunks(walk):
    """N_t = 512 in a 2 048-evaluation plan (chunks of 32 / 16 steps) with five high-norm steps
    scattered through the chunks: the walks square inside the lane; the stored path parks the
    steps for k_expm_high / k_grad_high, poisons the S = 2 chunk chains after them with NaN and
    k_scan rechains those chunks from E.  Checked against the oracle (long steps: T2 tier)."""
    from oracle import grape_oracle as O
    from robustgrape_amd.operators import OPT_NO_WALK
    nt = 512
    fp, fo = _high_norm_problem(nt)
    rng = np.random.default_rng(11)
    hot = [5, 40, 200, 333, 511]

    def mkx(seed, with_hot):
        r = np.random.default_rng(seed)
        xm = np.stack([2 * np.pi * r.uniform(size=nt), r.uniform(-0.5, 0.5, size=nt)])
        if with_hot:
            xm[1, hot] = r.choice([-900.0, 900.0], size=len(hot))
        return np.concatenate([xm.T.reshape(-1), [2 * np.pi * r.uniform()]])
    X = np.stack([mkx(100 + s, s % 3 == 0) for s in range(BIG)])
    pl = _plan(fp, BIG, 0 if walk else OPT_NO_WALK, nparam=2)
    try:
        F, Fdx, _, _ = pl.fidelity_grad(X)
    finally:
        pl.close()
    tag = "walk" if walk else "stored"
    for b in (0, 1, 999, BIG - 2):  # hot rows (b % 3 == 0) and ordinary rows
        F0, g0 = O.calculate_fidelity_and_derivatives(fo, X[b])[:2]
        _check(f"hot_{tag}_{b}", F[b], Fdx[b], F0, g0, P.fd_tier(fp, X[b], nparam=2))
    assert np.all(np.isfinite(F)) and np.all(np.isfinite(Fdx))
    del rng


def test_walk_single_calls_are_the_batch():
    """Graph-replayed single evaluations through the walks are bitwise the batch's rows."""
    fp = P.full9_problem(64)
    X = np.stack([P.random_x(64, 40 + s) for s in range(70)])
    pl = _plan(fp, 128)
    try:
        ref = pl.fidelity_grad(X)
        for b in (0, 31, 69):
            one = pl.fidelity_grad(X[b:b + 1])
            assert one[0][0] == ref[0][b] and np.array_equal(one[1][0], ref[1][b])
    finally:
        pl.close()


@pytest.mark.parametrize("name,fp", [("full9", lambda: P.full9_problem(96)), ("sym5", lambda: P.sym_problem(40)),
                                     ("full9-hot", lambda: _high_norm_problem(64)[0])])
def test_walk_propagator_modes_bitwise(name, fp):
    """The gradient walk reading the forward walk's stored propagators (default for the 4-level class)
    and recomputing them (GRAPE_OPT_WALK_RECOMPUTE) run the same exponential code on the same inputs:
    F and F_dx agree bit for bit.  (Permutation sectors: the stored propagators serve the 4-level
    class, which the symmetry-adapted C2 layout does not have.)"""
    from robustgrape_amd.operators import OPT_NO_GAUGE, OPT_NO_SYMMETRY, OPT_WALK_RECOMPUTE
    f = fp()
    nparam = 2 if name == "full9-hot" else 1
    nt = f.unitary_problem.ntimes
    rng = np.random.default_rng(3)
    X = rng.uniform(0, 2 * np.pi, size=(300, nparam * nt + 1))
    if name == "full9-hot":
        X[::7, 1::2][:, 5] = 700.0  # one high-norm step in every 7th row (the squaring path)
    outs = []
    for opts in (0, OPT_WALK_RECOMPUTE):  # (per-step exponentials: the phase-covariant walks store nothing)
        pl = _plan(f, 300, opts | OPT_NO_SYMMETRY | OPT_NO_GAUGE, nparam=nparam)
        try:
            outs.append(pl.fidelity_grad(X)[:2])
        finally:
            pl.close()
    for o in outs[1:]:
        assert np.array_equal(o[0], outs[0][0]) and np.array_equal(o[1], outs[0][1])


@pytest.mark.parametrize("name,fp", [("full9", lambda: P.full9_problem(64)), ("sym5", lambda: P.sym_problem(40)),
                                     ("fullblk7", lambda: P.fullblk_problem(40)),
                                     ("c3", lambda: P.full9_problem(40, nerr=4)),
                                     ("sym5-amp-freq", lambda: P.sym_problem(30, errors=("amp", "freq"))),
                                     ("fullblk7-amp", lambda: P.fullblk_problem(30, errors=("amp",)))])
def test_diagonal_head_matches_general_head(name, fp):
    """Diagonal projector and target (every Rydberg CZ problem): the one-thread-per-evaluation sector
    heads (grape_projector.hip k_sec_head_diag, k_sec_err_head_diag) against the general d x d heads
    (GRAPE_OPT_GENERAL_HEAD)
    -- F, the target part of F_dx_add and, through M, every F_dx / F_d2err / F_d2err_dx entry, at the
    rounding level of the two summation orders."""
    from robustgrape_amd.operators import OPT_GENERAL_HEAD
    f = fp()
    nt = f.unitary_problem.ntimes
    X = np.stack([P.random_x(nt, 4000 + s, small=(s % 2 == 0)) for s in range(130)])
    outs = []
    for opts in (0, OPT_GENERAL_HEAD):
        pl = _plan(f, len(X), opts)
        try:
            outs.append(pl.fidelity_grad(X))
        finally:
            pl.close()
    for a, b in zip(outs[0], outs[1]):
        if a.size:
            scale = max(float(np.max(np.abs(b))), 1e-300)
            assert float(np.max(np.abs(a - b))) <= 1e-12 * scale + 1e-15, (name, float(np.max(np.abs(a - b))), scale)


@pytest.mark.parametrize("gauge", [True, False])
@pytest.mark.parametrize("sym", [True, False])
@pytest.mark.parametrize("name,fp,nparam", [("full9", lambda: P.full9_problem(512), 1),
                                            ("full9-hot", lambda: _high_norm_problem(64)[0], 2)])
def test_pair_launches_bitwise(name, fp, nparam, sym, gauge):
    """Latency-bound calls (16-wave scans) of the Rydberg layout run both sector classes' walks and
    scans in one launch per stage (k_walk_fwd_pair, k_scan_pair, k_walk_grad_pair): the same
    arithmetic as one launch per class (GRAPE_OPT_NO_PAIR), so F and F_dx agree bit for bit --
    batched (stream path) and single (graph path) calls; the C2-size problem also against the
    oracle at the T2s tier."""
    from robustgrape_amd.operators import OPT_NO_EVAL1, OPT_NO_GAUGE, OPT_NO_PAIR, OPT_NO_SYMMETRY
    if not gauge and name == "full9-hot":
        pytest.skip("two controls per step: never phase-covariant")
    f = fp()
    nt = f.unitary_problem.ntimes
    rng = np.random.default_rng(11)
    X = rng.uniform(0, 2 * np.pi, size=(5, nparam * nt + 1))
    if name == "full9":
        X[:, :nt] *= 0.001  # the C2 start: a 2 pi 0.001 U pulse
    elif name == "full9-hot":
        X[::2, 1::2][:, 5] = 700.0  # a high-norm step (squaring path) in every other row
    outs = []
    for opts in (0, OPT_NO_PAIR):
        # (OPT_NO_EVAL1: the pair kernels themselves, not one workgroup per evaluation)
        pl = _plan(f, 8, opts | OPT_NO_EVAL1 | (0 if sym else OPT_NO_SYMMETRY) | (0 if gauge else OPT_NO_GAUGE),
                   nparam=nparam)
        try:
            batch = pl.fidelity_grad(X)[:2]
            single = pl.fidelity_grad(X[3:4])[:2]
            outs.append((batch, single))
        finally:
            pl.close()
    (b0, s0), (b1, s1) = outs
    assert np.array_equal(b0[0], b1[0]) and np.array_equal(b0[1], b1[1])
    assert np.array_equal(s0[0], s1[0]) and np.array_equal(s0[1], s1[1])
    assert s0[0][0] == b0[0][3] and np.array_equal(s0[1][0], b0[1][3])
    if name == "full9":
        from oracle import grape_oracle as O
        F0, g0 = O.calculate_fidelity_and_derivatives(f, X[0])[:2]
        _check(f"pair_full9_{'gauge' if gauge else 'exp'}", b0[0][0], b0[1][0], F0, g0, True)


@pytest.mark.parametrize("gauge", [True, False])
@pytest.mark.parametrize("nb,max_batch", [(300, 300), (3, 8)])
def test_twin_sectors_bitwise(nb, max_batch, gauge):
    """Twin sectors (grape_walk.hpp TWIN: the 2-level Rydberg sectors {01, 0r} and {10, r0} have
    identical operator blocks at equal Rabi frequencies): one exponential per step serves both.
    The shared propagators are the ones each sector would compute from the same inputs, so F and
    F_dx equal those of GRAPE_OPT_NO_TWIN bit for bit -- a throughput-size batch and a latency-bound
    one (16-wave scans, pair kernels), plus a single call."""
    from robustgrape_amd.operators import OPT_NO_GAUGE, OPT_NO_TWIN
    f = P.full9_problem(128)
    rng = np.random.default_rng(21)
    X = rng.uniform(0, 2 * np.pi, size=(nb, 129))
    outs = []
    for opts in (0, OPT_NO_TWIN):
        pl = _plan(f, max_batch, opts | (0 if gauge else OPT_NO_GAUGE))
        try:
            outs.append((pl.fidelity_grad(X)[:2], pl.fidelity_grad(X[:1])[:2]))
        finally:
            pl.close()
    (b0, s0), (b1, s1) = outs
    assert np.array_equal(b0[0], b1[0]) and np.array_equal(b0[1], b1[1])
    assert np.array_equal(s0[0], s1[0]) and np.array_equal(s0[1], s1[1])
