"""The extended-precision evaluator (oracle/grape_exact.py) against the double oracle and the
reference's known answer (CPU).  grape_exact restates the same formulas as oracle/grape_oracle.py
(UnitaryCalculations.jl:44-151, FidelityCalculations.jl:19-119) in longdouble, so the two agree to
the oracle's own rounding noise: F to 1e-14, the eps forward differences to ~u / eps of their
scale, the eps2 mixed stencils to ~u / eps2^2."""
import numpy as np

from tests import problems as P


def test_exact_matches_oracle_within_its_noise():
    from oracle import grape_exact as E
    from oracle import grape_oracle as O
    for fp, nt in ((P.sym_problem(12), 12), (P.full9_problem(20), 20)):
        x = P.random_x(nt, 31)
        F, g = E.fidelity_and_gradient(fp, x)
        F0, g0 = O.calculate_fidelity_and_derivatives(fp, x)[:2]
        assert abs(F - F0) < 1e-14
        assert np.max(np.abs(g - g0)) < 1e-6 * np.max(np.abs(g0)) + 1e-9
        # the error-free form of the general evaluator: the same computation, products grouped differently
        Fa, ga, d2, d2dx = E.fidelity_and_derivatives(fp, x)
        assert abs(Fa - F) < 1e-16 and np.max(np.abs(ga - g)) < 1e-15 * np.max(np.abs(g)) and d2.shape == (0,)


def test_exact_error_path_matches_oracle_within_its_noise():
    from oracle import grape_exact as E
    from oracle import grape_oracle as O
    fp = P.sym_problem(8, errors=("amp", "freq"))
    x = P.random_x(8, 5)
    ex = E.fidelity_and_derivatives(fp, x)
    ref = O.calculate_fidelity_and_derivatives(fp, x)
    assert abs(ex[0] - ref[0]) < 1e-14
    assert np.max(np.abs(ex[1] - ref[1])) < 1e-6 * np.max(np.abs(ref[1])) + 1e-9
    assert np.max(np.abs(ex[2] - ref[2])) < 1e-6 * np.max(np.abs(ref[2])) + 1e-9
    assert np.max(np.abs(ex[3] - ref[3])) < 1e-4 * np.max(np.abs(ref[3])) + 1e-6


def test_exact_reproduces_the_evered_known_answer():
    """runtests.jl:115-165: F > 0.9999 for the published time-optimal pulse (the restatement value
    0.999996184760959)."""
    from oracle import grape_exact as E
    F, g = E.fidelity_and_gradient(P.sym_problem(1000), P.evered_pulse(1000))
    assert F > 0.9999 and abs(F - 0.999996184760959) < 1e-12


def test_sensitivities_and_xadd_are_the_full_evaluators_rows():
    """grape_exact.sensitivities_and_xadd (only the nominal and eps error propagators) returns
    fidelity_and_derivatives' own F, F_d2err and x_add rows of F_d2err_dx (tests/xadd_pin.py uses it)."""
    import numpy as np
    from oracle import grape_exact as E
    from tests import problems as P
    for fp, x in ((P.sym_problem(7, errors=("amp", "freq")), P.random_x(7, 11)),
                  (P.full9_problem(5, nerr=4), P.random_x(5, 12, small=True))):
        F, _, d2, d2dx = E.fidelity_and_derivatives(fp, x)
        F1, d21, add = E.sensitivities_and_xadd(fp, x)
        assert F1 == F and np.array_equal(d21, d2) and np.array_equal(add, d2dx[len(x) - 1:])
    import pytest
    with pytest.raises(ValueError):
        E.sensitivities_and_xadd(P.xadd_err_problem(5, 3), P.xadd_x(3, 1))
