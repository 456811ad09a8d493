"""Oracle vs committed golden fixtures, and the two CPU restatements against each other.

* the numpy oracle reproduces every golden fixture (regression guard on the
  generator, cheap cases recomputed here);
* the reference-faithful C++ port (oracle/cref, the CPU baseline) agrees with
  the numpy oracle within the SURVEY.md 8c tiers on every config, with error
  sources, and on the materialised unitary derivatives.
"""
import os

import numpy as np
import pytest

from oracle import grape_oracle as O
from tests import problems as P

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def g(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


# Tiers with absolute floors for the reference's own rounding noise:
#  T2 eps-FD:   1e-6 * max|ref| + 1e-7   (~10 u/eps: at an optimum max|F_dx| itself is ~1e-8 noise)
#  T3 eps2:     1e-5 * max|ref| + 1e-7 on the control rows; the x_add rows of the
#               mixed stencil are ((a+b)-a-b)/eps2^2 rounding residue when H0 does not
#               read x_add (UnitaryCalculations.jl:87-95), ~N_t*u/eps2^2 <= 1e-5 absolute.
T2, T2_ABS = 1e-6, 1e-7
T3, T3_ABS, T3_XADD_ABS = 1e-5, 1e-7, 1e-5


def close(a, b, tier, atol=0.0):
    a, b = np.asarray(a), np.asarray(b)
    if not b.size:
        return True
    return np.max(np.abs(a - b)) <= tier * np.max(np.abs(b)) + atol


@pytest.fixture(scope="module")
def cref():
    from oracle.cref import build, cref as c
    build.build()
    return c


def test_numpy_oracle_reproduces_c1_golden():
    f = g("c1")
    F, Fdx, _, _ = O.calculate_fidelity_and_derivatives(P.sym_problem(500, t0=P.T0_TO, device=False), f["x"])
    assert F == f["F"] and np.array_equal(Fdx, f["F_dx"])


def test_expm_golden_matches_julia_exp_restatement():
    f = g("expm")
    for i in range(0, len(f["m"]), 5):
        np.testing.assert_array_equal(O.julia_exp(f[f"A{i}"]), f[f"E{i}"])


@pytest.mark.parametrize("name,builder", [
    ("c1", lambda: P.sym_problem(500, t0=P.T0_TO)),
    ("c2", lambda: P.full9_problem(512)),
    ("c1err", lambda: P.sym_problem(500, t0=P.T0_TO, errors=("amp", "freq"))),
    ("d7err", lambda: P.fullblk_problem(500, errors=("amp", "freq"))),
    ("c3n64", lambda: P.full9_problem(64, nerr=4)),
])
def test_cpp_port_matches_golden(cref, name, builder):
    f = g(name)
    fp = builder()
    F, Fdx, d2, d2dx = cref.fidelity_grad(fp, f["x"])
    nmain = len(f["x"]) - fp.unitary_problem.nb_additional_param
    assert abs(F - f["F"]) <= 1e-12
    assert close(Fdx, f["F_dx"], T2, T2_ABS)
    # sensitivities: the operator-basis error is err*H_e, the reference idiom
    # H(err)-H(0) carries fl(1+err)-1 rounding (~1e-8 relative at eps = 1e-8)
    assert close(d2, f["F_d2err"], T3, T3_ABS)
    assert close(d2dx[:nmain], f["F_d2err_dx"][:nmain], T3, T3_ABS)
    assert close(d2dx[nmain:], f["F_d2err_dx"][nmain:], 0.0, T3_XADD_ABS)


def test_cpp_port_unitary_derivatives_match_oracle(cref):
    f = g("unitary_small")
    ref = [f[k] for k in ("U", "U_dx", "U_dx_add", "U_derr", "U_derr_dx", "U_derr_dx_add")]
    got = cref.unitary_derivs(P.sym_problem(8, errors=("amp", "freq")), f["x"])
    tiers = [(1e-13, 0), (T2, T2_ABS), (T2, T2_ABS), (T3, T3_ABS), (T3, T3_ABS), (0, T3_XADD_ABS)]
    for a, b, (t, at) in zip(got, ref, tiers):
        assert a.shape == b.shape
        assert close(a, b, t, at)


def test_cpp_port_same_exp_count_as_reference(cref):
    """N_t * [1 + 2np + 2na + ne(2 + np + na)] exps per evaluation (UnitaryCalculations.jl:45-90)."""
    L = cref.lib()
    before = L.grape_cref_exp_calls()
    cref.fidelity_grad(P.full9_problem(16, nerr=2), P.random_x(16, 3))
    assert L.grape_cref_exp_calls() - before == 16 * (1 + 2 + 2 + 2 * (2 + 1 + 1))
