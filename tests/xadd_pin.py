"""The x_add rows of F_d2err_dx pinned to their exact value.

When H0 and Herror do not read x_add, U_derr_dx_add is exactly zero and those rows are the target's
difference against U_derr (FidelityCalculations.jl:96-113).  The reference nevertheless forms the mixed
eps2 stencil for x_add too (UnitaryCalculations.jl:87-95): ((E(x_add + eps2, err eps2) + E) - E(err eps2)
- E(x_add + eps2)) / eps2^2 with E(x_add + eps2) == E bit for bit, i.e. ((a + b) - a - b) / 1e-8 rounding
residue, summed over the steps -- so the oracle (a faithful restatement) carries up to ~5e-6 absolute
there while the device, which forms no stencil for a parameter H does not read, carries none.  The
device is therefore checked against the exact rows (oracle/grape_exact.sensitivities_and_xadd, longdouble)
at T3 of their scale plus the checker's own measured distance from exact (the double implementations'
u / eps noise of the target difference is of the same size in the device and the checker), and against
the checker within twice that distance.  Both comparisons are logged with the exact rows' scale.
"""
import numpy as np

T3, T3_ABS = 1e-5, 1e-7
XADD_ABS = 1e-5  # problems outside grape_exact (x_add-dependent H): the stencil residue's bound


def exact_rows(fp, x, nparam=1):
    """(na, ne) exact x_add rows of F_d2err_dx, or None when grape_exact does not cover the problem
    (H0 or Herror reading x_add)."""
    from oracle import grape_exact as E
    try:
        return E.sensitivities_and_xadd(fp, x, nparam)[2]
    except ValueError:
        return None


def check_xadd(test, got, ref, nmain, exact, rel=T3, ab=T3_ABS, stencil=False):
    """got / ref: F_d2err_dx (n_x, ne) of the device and of the checker (oracle, golden or another
    device path); exact: (na, ne) exact rows.  Records both comparisons with a non-zero scale.
    stencil: the device path forms the reference's x_add stencil itself (the closure-table path
    tabulates every call site), so it carries a residue of the same kind as the checker's: both bounds
    then take twice the checker's measured distance from exact on top of the tier."""
    from tests.parity_log import record
    ga, ra = np.asarray(got)[nmain:], np.asarray(ref)[nmain:]
    if ga.size == 0:
        return
    if exact is None:  # H0 / Herror read x_add: no exact evaluator, the stencil residue's absolute bound
        ea = float(np.max(np.abs(ga - ra)))
        record(test, "F_d2err_dx_add", ea, float(np.max(np.abs(ra))), XADD_ABS)
        assert ea <= XADD_ABS, (test, "F_d2err_dx_add", ea)
        return
    ex = np.asarray(exact).reshape(ga.shape)
    scale = float(np.max(np.abs(ex)))
    noise = float(np.max(np.abs(ra - ex)))  # the checker's own distance from exact
    e_exact = float(np.max(np.abs(ga - ex)))
    # the device's own u / eps noise (the double difference of the target, U0(x_add + eps) - U0, and of the
    # error propagators) is of the checker's kind: both bounds carry the checker's measured distance from
    # exact, which also holds the checker's stencil residue (T3 |exact| + that distance)
    tol_exact = rel * scale + ab + (2 if stencil else 1) * noise
    record(test + "_vs_exact", "F_d2err_dx_add", e_exact, scale, tol_exact)
    assert e_exact <= tol_exact, (test, "F_d2err_dx_add vs exact", e_exact, scale)
    e_ref = float(np.max(np.abs(ga - ra)))
    tol_ref = rel * scale + ab + (3 if stencil else 2) * noise
    record(test, "F_d2err_dx_add", e_ref, scale, tol_ref)
    assert e_ref <= tol_ref, (test, "F_d2err_dx_add", e_ref, scale, noise)
    return {"vs_exact": e_exact, "vs_ref": e_ref, "ref_noise": noise, "scale": scale}
