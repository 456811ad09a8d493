"""General (non-diagonal) projectors, which the reference accepts as any real matrix
(Types.jl:54 `projector::Matrix{<:Real}`, FidelityCalculations.jl:47-51: P0 = projector,
tr_mod(X) = tr(P0 X), P = P0 with its nonzero entries set to 1, D = Re tr(P0)).

The engines' hot kernels specialise to a diagonal P0; any other matrix takes the general heads
of grape_projector.hip after the scans.  Checked against the live oracle (which evaluates the
reference's expressions literally) on every device path: the small-d operator basis with and
without error sources (H0 reading x_add included), the closure fallback, the dense engine with
and without error sources, the expectation values and the fidelity response."""
import numpy as np
import pytest

from robustgrape_amd import synthetic as S
from tests import problems as P

pytestmark = pytest.mark.gpu
T1 = 1e-12
T2, T2_ABS = 1e-6, 1e-8      # eps-FD tier (long-step problems; see test_gpu_xadd_err.py)
T3, T3_ABS = 1e-5, 1e-7      # eps2 mixed stencils


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def sparse_projector(W, seed):
    """The problem's diagonal weights plus a few off-diagonal (non-symmetric) entries: P then
    differs from P0's pattern of a diagonal projector and A = P0 P mixes rows."""
    rng = np.random.default_rng(seed)
    P0 = np.array(W, dtype=np.float64)
    d = P0.shape[0]
    for _ in range(3):
        i, j = rng.integers(0, d, 2)
        if i != j:
            P0[i, j] = rng.uniform(-0.5, 0.5)
    return P0


def dense_projector(d, rank, seed):
    """Orthogonal projector onto a random real rank-`rank` subspace: every entry nonzero (P is the
    all-ones matrix), trace = rank."""
    rng = np.random.default_rng(seed)
    Qm, _ = np.linalg.qr(rng.standard_normal((d, rank)))
    return Qm @ Qm.T


def _cmp(out, ref, label, errors=True):
    F, g, e, ed = out
    F0, g0, e0, ed0 = ref
    errs = {"F": abs(F - F0), "F_dx": np.max(np.abs(g - g0)) / np.max(np.abs(g0))}
    if errors:
        errs["F_d2err"] = np.max(np.abs(e - e0)) / np.max(np.abs(e0))
        errs["F_d2err_dx"] = np.max(np.abs(ed - ed0)) / np.max(np.abs(ed0))
    print(label, {k: f"{v:.2e}" for k, v in errs.items()})
    assert abs(F - F0) <= T1, (F, F0)
    assert np.max(np.abs(g - g0)) <= T2 * np.max(np.abs(g0)) + T2_ABS
    if errors:
        assert np.max(np.abs(e - e0)) <= T2 * np.max(np.abs(e0)) + T2_ABS
        assert np.max(np.abs(ed - ed0)) <= T3 * np.max(np.abs(ed0)) + T3_ABS


def _with_projector(fp, P0):
    return fp.replace(projector=P0)


@pytest.mark.parametrize("kind", ["sparse", "dense"])
@pytest.mark.parametrize("nerr", [0, 2])
def test_small_d_operator_basis(kind, nerr):
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_fidelity_and_derivatives
    nt = 13
    errors = ("amp", "freq")[:nerr]
    fp = P.sym_problem(nt, errors=errors)
    fo = P.sym_problem(nt, errors=errors, device=False)
    P0 = sparse_projector(P.W_SYM, 3) if kind == "sparse" else dense_projector(5, 2, 4)
    x = P.random_x(nt, 11)
    ref = O.calculate_fidelity_and_derivatives(_with_projector(fo, P0), x)
    out = calculate_fidelity_and_derivatives(_with_projector(fp, P0), x)
    _cmp(out, ref, f"d=5 {kind} ne={nerr}", errors=nerr > 0)
    # really general: the diagonal-projector result differs
    diag = calculate_fidelity_and_derivatives(fp, x)
    assert abs(diag[0] - out[0]) > 1e-6


@pytest.mark.parametrize("device", [True, False], ids=["operator-basis", "closures"])
@pytest.mark.parametrize("d,nt", [(5, 9), (9, 7)])
def test_xadd_dependent_h0_with_errors(device, d, nt):
    """H0 and an error generator reading x_add, two additional parameters, two error sources:
    every head output (F, M'_c, F_dx_add's target part, F_d2err, M'_{c,e}, F_d2err_dx_add's
    target part) is exercised."""
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_fidelity_and_derivatives
    P0 = dense_projector(d, 3, 20 + d) + sparse_projector(np.zeros((d, d)), 21)
    x = P.xadd_x(nt, 60 + nt)
    ref = O.calculate_fidelity_and_derivatives(_with_projector(P.xadd_err_problem(d, nt, device=False), P0), x)
    out = calculate_fidelity_and_derivatives(_with_projector(P.xadd_err_problem(d, nt, device=device), P0), x)
    _cmp(out, ref, f"d={d} xadd {'ob' if device else 'tables'}")


def test_small_d_batch_is_bitwise_the_single_calls():
    from robustgrape_amd import calculate_fidelity_and_derivatives
    fp = _with_projector(P.full9_problem(24, nerr=2), dense_projector(9, 4, 5))
    X = np.stack([P.random_x(24, s) for s in range(5)])
    F, Fdx, d2, d2dx = calculate_fidelity_and_derivatives(fp, X)
    for b in (0, 4):
        Fs, gs, es, eds = calculate_fidelity_and_derivatives(fp, X[b])
        assert Fs == F[b] and np.array_equal(gs, Fdx[b]) and np.array_equal(es, d2[b])
        assert np.array_equal(eds, d2dx[b])


@pytest.mark.parametrize("d,ntimes,nerr,phase", [(13, 4, 0, False), (16, 5, 2, True), (24, 7, 1, False)])
def test_dense_engine(d, ntimes, nerr, phase):
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_fidelity_and_derivatives
    if nerr:
        fp = S.dense_error_problem(d, ntimes, rank=min(16, d - 3), nerr=nerr, phase=phase)
    else:
        fp = S.dense_problem(d, ntimes, rank=min(16, d - 3))
    fp = _with_projector(fp, dense_projector(d, 6, 30 + d))
    x = S.dense_x(ntimes, seed=500 + ntimes)
    if phase:
        x = np.concatenate([x, [0.7]])
    ref = O.calculate_fidelity_and_derivatives(fp, x)
    out = calculate_fidelity_and_derivatives(fp, x)
    _cmp(out, ref, f"dense d={d} ne={nerr}", errors=nerr > 0)


def test_analysis_entry_points():
    """calculate_expectation_values (tr_mod over the HIP interaction operators) and the fidelity
    response, direct and FFT (FidelityCalculations.jl:246-343, 368-390), with a general P0."""
    from oracle import grape_oracle as O
    from robustgrape_amd import analysis as A
    nt = 16
    P0 = sparse_projector(P.W_SYM, 8)
    fp = _with_projector(P.sym_problem(nt, errors=("amp", "freq")), P0)
    fo = _with_projector(P.sym_problem(nt, errors=("amp", "freq"), device=False), P0)
    x = P.random_x(nt, 3)
    ev0 = O.calculate_expectation_values(fo, x)
    ev = A.calculate_expectation_values(fp, x)
    assert np.max(np.abs(ev - ev0)) <= T2 * np.max(np.abs(ev0)) + T2_ABS
    w = np.linspace(0.0, 2.0, 5)
    r0 = O.calculate_fidelity_response(fo, x, w)
    r = A.calculate_fidelity_response(fp, x, w)
    assert np.max(np.abs(r - r0)) <= T2 * np.max(np.abs(r0)) + T2_ABS
    f0, fr0 = O.calculate_fidelity_response_fft(fo, x, 2)
    f, fr = A.calculate_fidelity_response_fft(fp, x, 2)
    np.testing.assert_allclose(fr, fr0)
    assert np.max(np.abs(f - f0)) <= T2 * np.max(np.abs(f0)) + T2_ABS
