"""Pin the CPU oracle (oracle/grape_oracle.py) to the reference's own tests.

The reference's Julia toolchain is absent here, so its test/runtests.jl
testsets are re-run against the oracle with numpy seeds (Julia's RNG stream is
not reproducible), with the reference's tolerances.  Each test cites the
testset it restates.
"""
import os

import numpy as np
import pytest
import scipy.linalg as sl

from oracle import grape_oracle as O
from tests import problems as P


def test_known_answer_evered_pulse():
    """runtests.jl:115-165 -- the Evered et al. pulse reaches F > 0.9999."""
    fp = P.sym_problem(1000, device=False)
    F = O.calculate_fidelity_and_derivatives(fp, P.evered_pulse(1000))[0]
    assert F > 0.9999
    # value of an independent numpy restatement recorded in SURVEY.md section 4
    assert abs(F - 0.999996184760959) < 1e-12


def test_fidelity_gradient_matches_forward_difference():
    """runtests.jl:292-354 -- (F(x+eps e_i)-F(x))/eps vs F_dx[i], rtol=atol=1e-3."""
    ntimes = 50
    fp = P.sym_problem(ntimes, device=False)
    rng = np.random.default_rng(42)
    for ntest in range(5):
        idx = int(rng.integers(ntimes)) if ntest < 4 else ntimes
        xs = 2 * np.pi * rng.uniform(size=ntimes + 1)
        F0, g0, _, _ = O.calculate_fidelity_and_derivatives(fp, xs)
        xs[idx] += fp.unitary_problem.eps
        F1 = O.calculate_fidelity_and_derivatives(fp, xs)[0]
        np.testing.assert_allclose((F1 - F0) / fp.unitary_problem.eps, g0[idx], rtol=1e-3, atol=1e-3)


def test_error_sensitivity_gradient_matches_difference():
    """runtests.jl:48-113 -- (F_d2err(x+1e-4 e_i)-F_d2err(x))/1e-4 vs F_d2err_dx[i]."""
    ntimes = 200
    fp = P.sym_problem(ntimes, errors=("amp",), device=False)
    rng = np.random.default_rng(42)
    for ntest in range(2):
        idx = ntimes if ntest == 1 else int(rng.integers(ntimes))
        xs = 2 * np.pi * rng.uniform(size=ntimes + 1)
        _, _, d0, d0dx = O.calculate_fidelity_and_derivatives(fp, xs)
        xs[idx] += 1e-4
        _, _, d1, _ = O.calculate_fidelity_and_derivatives(fp, xs)
        np.testing.assert_allclose((d1[0] - d0[0]) / 1e-4, d0dx[idx, 0], rtol=1e-3, atol=1e-5)


GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def pulse200():
    """LBFGS-optimised pulse, N=200, t0=2pi*1.22 (tests/golden/make_golden.py)."""
    return np.load(os.path.join(GOLDEN, "opt_pulse_sym_n200.npy"))


@pytest.fixture(scope="module")
def pulse500():
    """LBFGS-optimised pulse, N=500, t0=7.613 (tests/golden/make_golden.py)."""
    return np.load(os.path.join(GOLDEN, "opt_pulse_sym_n500_t7613.npy"))


def test_optimised_pulses_are_optimal(pulse200, pulse500):
    """runtests.jl:356-416 asks an optimiser to reach 1-F < 1e-6; the fixtures do."""
    assert 1 - O.calculate_fidelity_and_derivatives(P.sym_problem(200, device=False), pulse200)[0] < 1e-6
    fp = P.sym_problem(500, t0=P.T0_TO, device=False)
    assert 1 - O.calculate_fidelity_and_derivatives(fp, pulse500)[0] < 1e-6


def test_sensitivity_matches_second_difference(pulse200):
    """runtests.jl:167-290 -- F_d2err vs (F(+e2)+F(-e2)-2F)/e2^2 on an optimised pulse."""
    x = pulse200
    base = P.sym_problem(200, device=False)
    up = base.unitary_problem
    e2 = up.eps2
    Fs = []
    for err in (0.0, e2, -e2):
        H = (lambda err: lambda t, p, xa: O.rydberg_hamiltonian_symmetric_blockaded(p[0], err, 0))(err)
        Fs.append(O.calculate_fidelity_and_derivatives(base.replace(unitary_problem=up.replace(H0=H)), x)[0])
    robust = P.sym_problem(200, errors=("amp",), device=False)
    _, _, d2, _ = O.calculate_fidelity_and_derivatives(robust, x)
    numerical = (Fs[1] + Fs[2] - 2 * Fs[0]) / e2 ** 2
    np.testing.assert_allclose(numerical, d2[0], rtol=1e-3, atol=1e-2)


def test_reduced_vs_full_hamiltonian_sensitivity(pulse500):
    """runtests.jl:418-529 -- d=5 symmetric and d=7 full models give the same sensitivities."""
    x = pulse500
    sym = P.sym_problem(500, t0=P.T0_TO, errors=("amp", "freq"), device=False)
    full = P.fullblk_problem(500, t0=P.T0_TO, errors=("amp", "freq"), device=False)
    _, _, ds, _ = O.calculate_fidelity_and_derivatives(sym, x)
    _, _, df, _ = O.calculate_fidelity_and_derivatives(full, x)
    np.testing.assert_allclose(ds, df, rtol=1e-3, atol=1e-3)


def test_response_at_zero_frequency_matches_sensitivity(pulse500):
    """runtests.jl:531-619 -- -F_d2err = 2 * response(omega = 0)."""
    x = pulse500
    fp = P.sym_problem(500, t0=P.T0_TO, errors=("amp", "freq"), device=False)
    _, _, d2, _ = O.calculate_fidelity_and_derivatives(fp, x)
    resp = O.calculate_fidelity_response(fp, x, [0.0])
    np.testing.assert_allclose(-d2, 2 * resp[0], rtol=1e-3, atol=1e-3)
    resp_fft, freqs = O.calculate_fidelity_response_fft(fp, x, oversampling=2)
    assert freqs[0] == 0.0
    np.testing.assert_allclose(resp_fft[0], resp[0], rtol=1e-10, atol=1e-12)


def test_published_time_optimal_values(pulse500):
    """docs/src/examples.md:200-240, 287-310 (examples/time_optimal_cz.jl) print, for the
    reference's own optimised time-optimal pulse (N = 500, t0 = 7.613): infidelity 1.39e-13,
    amplitude sensitivity -F_d2err[1]/2 = 4.211625822890814, frequency sensitivity
    -F_d2err[2]/2 = 2.8602011006871577 and integrated Rydberg population
    calculate_expectation_values(...)[end, 1] = 2.963973401634995 (2.963781384493184 in a
    second run, :394 -- the optimiser's end point varies between runs).  Our fixture is a
    different optimiser run (scipy L-BFGS, tests/golden/make_golden.py) reaching 6.7e-14, so the
    published numbers are not bit-level vectors; they pin the oracle's conventions (sign,
    the factor 2 of F_d2err, the eps normalisation of Herror, the time integration of the
    expectation values) to within the spread of near-optimal pulses (measured: amp 1.9 %,
    freq 0.31 %, Rydberg population 0.33 %)."""
    from robustgrape_amd.types import ErrorSource
    x = pulse500
    fp = P.sym_problem(500, t0=P.T0_TO, errors=("amp", "freq"), device=False)
    F, _, d2, _ = O.calculate_fidelity_and_derivatives(fp, x)
    assert 1 - F < 1.4e-13
    np.testing.assert_allclose(-d2[0] / 2, 4.211625822890814, rtol=0.025)
    np.testing.assert_allclose(-d2[1] / 2, 2.8602011006871577, rtol=0.005)
    decay = np.diag([0, 0, 0, 1.0, 1.0]).astype(complex)
    fd = fp.replace(unitary_problem=fp.unitary_problem.replace(
        error_sources=[ErrorSource(lambda t, p, xa, e: e * decay)]))
    ev = O.calculate_expectation_values(fd, x)
    np.testing.assert_allclose(ev[-1, 0], 2.963973401634995, rtol=0.005)


@pytest.mark.parametrize("norm,m", [(0.01, 3),(0.2, 5), (0.5, 7), (1.5, 9), (4.0, 13), (60.0, 13)])
def test_julia_exp_degree_and_accuracy(norm, m):
    """Julia exp! restatement: Pade degree thresholds and accuracy vs scipy.linalg.expm."""
    rng = np.random.default_rng(int(norm * 100))
    H = rng.normal(size=(9, 9)) + 1j * rng.normal(size=(9, 9))
    H = (H + H.conj().T) / 2
    A = -1j * H / np.abs(H).sum(axis=0).max() * norm
    stats = {}
    E = O.julia_exp(A, stats)
    assert list(stats)[0][0] == m
    assert np.abs(E - sl.expm(A)).max() < 1e-13 * max(1.0, norm)
    assert np.abs(E.conj().T @ E - np.eye(9)).max() < 1e-13 * max(1.0, norm)


def test_julia_exp_balancing_and_diagonal_paths():
    """zgebal permutation isolates the decoupled |00> row/column; isdiag early exit."""
    H = O.rydberg_hamiltonian_full(0.3, 1, 1, 0, 0, 10)
    Ab, ilo, ihi, scale = O.zgebal_b(-1j * 0.015 * H)
    assert ihi == 8 and ilo == 1 and scale[8] == 1.0  # row/col 1 (|00>) pushed to position 9
    E = O.julia_exp(-1j * 0.015 * H)
    assert E[0, 0] == 1.0 and np.all(E[0, 1:] == 0) and np.all(E[1:, 0] == 0)
    D = np.diag([0.1j, -0.3j, 2.0])
    np.testing.assert_array_equal(O.julia_exp(D), np.diag(np.exp(np.diag(D))))
