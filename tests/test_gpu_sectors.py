"""Sectors (include/grape.h grape_plan_sectors): problems whose H0 operators are block-diagonal
in a common permutation run each evaluation as independent sector problems.  The Rydberg
Hamiltonians of the reference all have this structure (the laser couples |1> <-> |r> only):
rydberg_hamiltonian_full (d = 9) splits into blocks of 4, 2, 2 and the untouched |00> -> one
sector of 4 levels and two of 2 (two sector classes), the symmetric blockaded one (d = 5) into
2, 2 (+ |00>) -> 2 sectors of 2, the full blockaded one (d = 7) into 2, 2, 2 (+ |00>) -> 3
sectors of 2.

The sector path must give the whole-matrix path's numbers (GRAPE_OPT_NO_SECTORS) and the
oracle's, for diagonal and general projectors (which mix sectors in the fidelity head),
x_add-dependent H0, parked high-norm steps, and the graph-replayed single evaluations."""
import numpy as np
import pytest

from tests import problems as P

pytestmark = pytest.mark.gpu
T1 = 1e-12
T2S, T2S_ABS = 1e-7, 1e-9     # short-step eps-FD tier (test_gpu_parity.py)
T2, T2_ABS = 1e-6, 1e-7


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _plan(fp, max_batch, monkeypatch, whole=False, nparam=1, options=0):
    from robustgrape_amd.engine import GrapePlan
    from robustgrape_amd.operators import OPT_NO_SECTORS
    return GrapePlan(fp, nparam=nparam, device=0, max_batch=max_batch,
                     options=options | (OPT_NO_SECTORS if whole else 0))


def _both(fp, X, monkeypatch, options=0):
    ps, pw = _plan(fp, len(X), monkeypatch, options=options), _plan(fp, len(X), monkeypatch, whole=True)
    try:
        return ps.sectors(), pw.sectors(), ps.fidelity_grad(X), pw.fidelity_grad(X)
    finally:
        ps.close()
        pw.close()


def _close(a, b, tight=True):
    """tight: the short-step T2s tier; the chunk walks square a scaled Taylor 12 where the row
    groups (and the reference) take Pade 7 / 9 / 13, so problems with |dt H|_1 > 0.25 compare at
    the long-step T2 tier (tests/problems.py max_step_norm)."""
    if isinstance(tight, tuple):  # tests/problems.py fd_tier
        t2, t2a = tight
    else:
        t2, t2a = (T2S, T2S_ABS) if tight else (T2, T2_ABS)
    assert np.max(np.abs(a[0] - b[0])) <= T1, np.max(np.abs(a[0] - b[0]))
    err, scale = np.max(np.abs(a[1] - b[1])), np.max(np.abs(b[1]))
    print(f"F {np.max(np.abs(a[0] - b[0])):.2e}  F_dx {err:.2e} (scale {scale:.2e})")
    assert err <= t2 * scale + t2a, (err, scale)


@pytest.mark.parametrize("name,fp,layout", [
    ("full9", lambda: P.full9_problem(40), P.FULL9_SYM),
    ("full9-perm", lambda: P.full9_problem(40), P.FULL9_PERM),
    ("sym5", lambda: P.sym_problem(24), ((2, 2),)),
    ("fullblk7", lambda: P.fullblk_problem(24), ((2, 3),)),
])
def test_sectors_match_whole_matrices_and_oracle(name, fp, layout, monkeypatch):
    """-perm: the permutation sectors (GRAPE_OPT_NO_SYMMETRY); full9: the symmetry-adapted ones."""
    from oracle import grape_oracle as O
    from robustgrape_amd.operators import OPT_NO_SYMMETRY
    f = fp()
    nt, d = f.unitary_problem.ntimes, f.unitary_problem.ndim
    X = np.stack([P.random_x(nt, 40 + s) for s in range(6)])
    sec, whole, out, ref = _both(f, X, monkeypatch, OPT_NO_SYMMETRY if name.endswith("-perm") else 0)
    assert sec == layout and whole == ((d, 1),)
    tight = P.fd_tier(f, X)
    _close(out, ref, tight)
    for b in (0, 5):
        F0, g0 = O.calculate_fidelity_and_derivatives(f, X[b])[:2]
        _close((out[0][b], out[1][b]), (F0, g0), tight)


T3, T3_ABS = 1e-5, 1e-7      # eps2 mixed stencils (F_d2err_dx)


def _close_err(a, b, label, fac=1.0):
    """F, F_dx, F_d2err, F_d2err_dx of two paths (T1, T2, T2, T3); fac scales the F_dx tier
    (tests/problems.py fd_tier: max(1, |dt H|_1) on long steps)."""
    errs = {}
    assert np.max(np.abs(a[0] - b[0])) <= T1
    for n, (x, y, t, ta) in enumerate([(a[1], b[1], T2 * fac, T2_ABS * fac), (a[2], b[2], T2, T2_ABS),
                                       (a[3], b[3], T3, T3_ABS)]):
        if np.size(y) == 0:  # no error sources
            continue
        err, scale = np.max(np.abs(x - y)), np.max(np.abs(y))
        errs[("F_dx", "F_d2err", "F_d2err_dx")[n]] = f"{err:.2e}/{scale:.2e}"
        assert err <= t * scale + ta, (label, n, err, scale)
    print(label, errs)


@pytest.mark.parametrize("name,fp,fo,layout", [
    ("full9-C3", lambda: P.full9_problem(24, nerr=4), lambda: P.full9_problem(24, nerr=4, device=False),
     P.FULL9_PERM),
    ("sym5-amp-freq", lambda: P.sym_problem(20, errors=("amp", "freq")),
     lambda: P.sym_problem(20, errors=("amp", "freq"), device=False), ((2, 2),)),
    ("fullblk7-amp", lambda: P.fullblk_problem(16, errors=("amp",)),
     lambda: P.fullblk_problem(16, errors=("amp",), device=False), ((2, 3),)),
])
def test_sectors_with_error_sources(name, fp, fo, layout, monkeypatch):
    """The error path on sectors: local-frame images, error scans and F_d2err_dx walks per
    sector, F_d2err and M_e from the assembled U and Tot in the sector error head."""
    from oracle import grape_oracle as O
    f = fp()
    nt = f.unitary_problem.ntimes
    X = np.stack([P.random_x(nt, 300 + s) for s in range(4)])
    sec, whole, out, ref = _both(f, X, monkeypatch)
    assert sec == layout and whole[0][1] == 1
    _close_err(out, ref, name + " vs whole")
    o = O.calculate_fidelity_and_derivatives(fo(), X[1])
    _close_err((out[0][1], out[1][1], out[2][1], out[3][1]), tuple(np.asarray(v) for v in o), name + " vs oracle")


@pytest.mark.parametrize("d", [5, 9])
def test_sectors_errors_xadd_and_general_projector(d, monkeypatch):
    """Error sources with an x_add-dependent H0 / Herror (per-step x_add terms of F_dx and
    F_d2err_dx summed over sectors and steps) and a general projector coupling sectors."""
    from oracle import grape_oracle as O
    nt = 12
    rng = np.random.default_rng(d)
    Qm, _ = np.linalg.qr(rng.standard_normal((d, 3)))
    P0 = Qm @ Qm.T
    fp = P.xadd_err_problem(d, nt, nerr=2).replace(projector=P0)
    X = np.stack([P.xadd_x(nt, 400 + s) for s in range(3)])
    sec, _, out, ref = _both(fp, X, monkeypatch)
    assert sec[0][0] < d
    _close_err(out, ref, f"xadd d={d} vs whole")
    o = O.calculate_fidelity_and_derivatives(P.xadd_err_problem(d, nt, nerr=2, device=False).replace(projector=P0), X[0])
    _close_err((out[0][0], out[1][0], out[2][0], out[3][0]), tuple(np.asarray(v) for v in o), f"xadd d={d} vs oracle")


@pytest.mark.parametrize("d", [5, 9])
def test_sectors_with_xadd_dependent_h0(d, monkeypatch):
    """H0 reading x_add (a diagonal term: the sectors survive): the per-step x_add terms are
    summed over sectors, then over steps, on top of the head's target part."""
    from oracle import grape_oracle as O
    nt = 16
    fp = P.xadd_err_problem(d, nt, nerr=0)
    X = np.stack([P.xadd_x(nt, 70 + s) for s in range(4)])
    sec, _, out, ref = _both(fp, X, monkeypatch)
    assert sec[0][0] < d
    _close(out, ref, P.fd_tier(fp, X))  # dt = t0 / 16 with x_main = 2 pi U: long steps, the T2 tier
    fo = P.xadd_err_problem(d, nt, nerr=0, device=False)
    F0, g0 = O.calculate_fidelity_and_derivatives(fo, X[2])[:2]
    _close((out[0][2], out[1][2]), (F0, g0), P.fd_tier(fp, X))


@pytest.mark.parametrize("sym", [True, False])
def test_general_projector_mixing_sectors(sym, monkeypatch):
    """A projector coupling levels of different sectors: only the head sees it (the sector
    blocks of M feed the contractions).  sym: the symmetry-adapted sectors, whose head takes the
    rotated P0' = V^dag P0 V with the rotated pattern P' = V^dag (P0 .!= 0) V (general form)."""
    from oracle import grape_oracle as O
    from robustgrape_amd.operators import OPT_NO_SYMMETRY
    nt = 20
    rng = np.random.default_rng(9)
    Qm, _ = np.linalg.qr(rng.standard_normal((9, 3)))
    P0 = Qm @ Qm.T
    fp = P.full9_problem(nt).replace(projector=P0)
    X = np.stack([P.random_x(nt, 90 + s) for s in range(3)])
    sec, _, out, ref = _both(fp, X, monkeypatch, 0 if sym else OPT_NO_SYMMETRY)
    assert sec == (P.FULL9_SYM if sym else P.FULL9_PERM)
    _close(out, ref, P.fd_tier(fp, X))
    fo = P.full9_problem(nt, device=False).replace(projector=P0)
    F0, g0 = O.calculate_fidelity_and_derivatives(fo, X[1])[:2]
    _close((out[0][1], out[1][1]), (F0, g0), P.fd_tier(fp, X))


def test_sectors_parked_high_norm_steps(monkeypatch):
    """Long steps (|A|_1 large): the sector exponentials take Pade 7/9/13 with squarings in
    k_expm_high / k_grad_high."""
    from oracle import grape_oracle as O
    nt = 6
    fp = P.full9_problem(nt, t0=40.0)
    X = np.stack([P.random_x(nt, 120 + s) for s in range(3)])
    _, _, out, ref = _both(fp, X, monkeypatch)
    _close(out, ref, P.fd_tier(fp, X))
    fo = P.full9_problem(nt, t0=40.0, device=False)
    F0, g0 = O.calculate_fidelity_and_derivatives(fo, X[0])[:2]
    _close((out[0][0], out[1][0]), (F0, g0), P.fd_tier(fp, X))


def test_sector_single_calls_are_the_batch(monkeypatch):
    """Graph-replayed single evaluations (<= 64 per call) and the stream path agree bitwise."""
    fp = P.full9_problem(32)
    X = np.stack([P.random_x(32, 200 + s) for s in range(70)])
    pl = _plan(fp, 128, monkeypatch)
    try:
        ref = pl.fidelity_grad(X)
        for b in (0, 33, 69):
            one = pl.fidelity_grad(X[b:b + 1])
            assert one[0][0] == ref[0][b] and np.array_equal(one[1][0], ref[1][b])
    finally:
        pl.close()


@pytest.mark.parametrize("nt", [1, 3])
def test_sectors_tiny_step_counts(nt, monkeypatch):
    """N_t = 1 and 3: one chunk per sector, chunk starts everywhere."""
    from oracle import grape_oracle as O
    for nerr in (0, 2):
        f = P.full9_problem(nt, nerr=nerr)
        X = np.stack([P.random_x(nt, 500 + s) for s in range(3)])
        sec, _, out, ref = _both(f, X, monkeypatch)
        assert sec == (P.FULL9_SYM if nerr == 0 else P.FULL9_PERM)
        fac = max(1.0, P.max_step_norm(f, X) / P.JULIA_THETA13)  # (tests/problems.py fd_tier)
        _close_err(out, ref, f"nt={nt} ne={nerr} vs whole", fac)
        o = O.calculate_fidelity_and_derivatives(P.full9_problem(nt, nerr=nerr, device=False), X[2])
        _close_err((out[0][2], out[1][2], out[2][2], out[3][2]), tuple(np.asarray(v) for v in o),
                   f"nt={nt} ne={nerr} vs oracle", fac)


def test_sectors_two_controls(monkeypatch):
    """n_p = 2 (phase and a detuning on the Rydberg levels, both read from x): two eps-variants
    per step and sector, F_dx interleaved per step."""
    from oracle import grape_oracle as O
    from robustgrape_amd import rydberg as R
    from robustgrape_amd.operators import FN_LINEAR, VAR_X, OperatorBasisHamiltonian, Term
    from robustgrape_amd.types import FidelityRobustGRAPEProblem, UnitaryRobustGRAPEProblem
    nt = 10
    Nr = np.diag([0, 0, 0, 0, 1, 1, 1, 1, 2]).astype(np.complex128)
    H0 = OperatorBasisHamiltonian(list(R.rydberg_full_operator_basis().terms)
                                  + [Term(Nr, var=VAR_X, index=1, func=FN_LINEAR, scale=0.3)])
    up = UnitaryRobustGRAPEProblem(t0=P.T0_TO, ntimes=nt, ndim=9, H0=H0, nb_additional_param=1)
    fp = FidelityRobustGRAPEProblem(up, P.W_FULL9, R.cz_full_target())
    rng = np.random.default_rng(77)
    X = np.stack([np.concatenate([rng.uniform(-3, 3, 2 * nt), [rng.uniform(0, 6)]]) for _ in range(3)])
    from robustgrape_amd.engine import GrapePlan
    from robustgrape_amd.operators import OPT_NO_SECTORS
    ps = GrapePlan(fp, nparam=2, device=0, max_batch=3)
    pw = GrapePlan(fp, nparam=2, device=0, max_batch=3, options=OPT_NO_SECTORS)
    try:
        # the detuning control keeps the swap symmetry; the dark level (1r - r1)/sqrt2 now has a
        # diagonal (Nr = 1 there): a 1-level sector in the 2-level class
        assert ps.sectors() == ((3, 1), (2, 3)) and pw.sectors() == ((9, 1),)
        out, ref = ps.fidelity_grad(X), pw.fidelity_grad(X)
    finally:
        ps.close()
        pw.close()
    _close(out, ref, P.fd_tier(fp, X, nparam=2))
    Hc = lambda t, x, xa: H0(t, x, xa)  # noqa: E731  (closure form for the oracle)
    fo = FidelityRobustGRAPEProblem(UnitaryRobustGRAPEProblem(t0=P.T0_TO, ntimes=nt, ndim=9, H0=Hc,
                                                              nb_additional_param=1),
                                    P.W_FULL9, lambda xa: R.cz_with_1q_phase_full(xa[0]))
    F0, g0 = O.calculate_fidelity_and_derivatives(fo, X[1])[:2]
    _close((out[0][1], out[1][1]), (F0, g0), P.fd_tier(fp, X, nparam=2))
