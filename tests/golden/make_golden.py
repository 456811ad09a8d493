"""Generate the golden fixtures under tests/golden/ from the CPU oracle.

Run from the repo root:  python tests/golden/make_golden.py
The fixtures are inputs + oracle outputs (data only).  Julia is absent from the
build container, so the outputs come from the numpy
restatement in oracle/grape_oracle.py, which tests/test_oracle_reference_identities.py
pins to the reference's own testsets.

Also produced: two LBFGS-optimised d=5 pulses (1-F < 1e-13) standing in for the
pulses the reference's tests optimise with Optim.jl (runtests.jl:167-290,
:418-619): scipy L-BFGS-B on the oracle's fidelity gradient, started from the
Evered et al. pulse (runtests.jl:127-138) resampled to the time grid.
"""
import os
import sys

import numpy as np
from scipy.optimize import minimize

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import grape_oracle as O  # noqa: E402
from tests import problems as P  # noqa: E402


def optimise(fp, x0, iters=300):
    def f(x):
        F, g, _, _ = O.calculate_fidelity_and_derivatives(fp, x)
        return 1.0 - F, -g
    r = minimize(f, x0, jac=True, method="L-BFGS-B", options=dict(maxiter=iters, ftol=1e-16, gtol=1e-12))
    return r.x


def evered_resampled(n):
    ev = P.evered_pulse(1000)
    ts = np.linspace(0, P.T0_TEST, 1000)
    return np.concatenate([np.interp(np.linspace(0, P.T0_TEST, n), ts, ev[:-1]), ev[-1:]])


def fid(fp, x):
    F, Fdx, d2, d2dx = O.calculate_fidelity_and_derivatives(fp, x)
    return dict(x=x, F=np.float64(F), F_dx=Fdx, F_d2err=d2, F_d2err_dx=d2dx)


def main():
    out = {}
    # optimised pulses (runtests.jl:167-290 uses N=200, t0=2pi*1.22; :418-619 N=500, t0=7.613)
    p200 = optimise(P.sym_problem(200, device=False), evered_resampled(200))
    p500 = optimise(P.sym_problem(500, t0=P.T0_TO, device=False), evered_resampled(500))
    np.save(os.path.join(HERE, "opt_pulse_sym_n200.npy"), p200)
    np.save(os.path.join(HERE, "opt_pulse_sym_n500_t7613.npy"), p500)

    # C1 (examples/time_optimal_cz.jl:13-32): d=5, N=500, t0=7.613, seed 43, small init
    out["c1"] = fid(P.sym_problem(500, t0=P.T0_TO, device=False), P.random_x(500, 43, small=True))
    # C1 + both errors on the optimised pulse (examples/time_optimal_cz.jl:60-71)
    out["c1err"] = fid(P.sym_problem(500, t0=P.T0_TO, errors=("amp", "freq"), device=False), p500)
    # d=7 full blockaded, 2 errors (runtests.jl:474-494)
    out["d7err"] = fid(P.fullblk_problem(500, errors=("amp", "freq"), device=False), p500)
    # C2: d=9, N=512, seed 0, x = 2pi U
    out["c2"] = fid(P.full9_problem(512, device=False), P.random_x(512, 0))
    # C3 reduced and full: d=9, 4 error operators, seed 1
    out["c3n64"] = fid(P.full9_problem(64, nerr=4, device=False), P.random_x(64, 1))
    out["c3"] = fid(P.full9_problem(512, nerr=4, device=False), P.random_x(512, 1))
    # C4 sample: restarts r=1000..1003 of C2 (small init, examples/time_optimal_cz.jl:32)
    out["c4"] = {}
    xs = np.stack([P.random_x(512, 1000 + r, small=True) for r in range(4)])
    res = [fid(P.full9_problem(512, device=False), x) for x in xs]
    out["c4"] = dict(x=xs, F=np.array([r["F"] for r in res]), F_dx=np.stack([r["F_dx"] for r in res]))

    # materialised unitary derivatives, small case with errors (UnitaryCalculations.jl:154)
    fp = P.sym_problem(8, errors=("amp", "freq"), device=False)
    xu = P.random_x(8, 7)
    U, Udx, Udxa, Ue, Uedx, Uedxa = O.calculate_unitary_and_derivatives(fp.unitary_problem, xu)
    out["unitary_small"] = dict(x=xu, U=U, U_dx=Udx, U_dx_add=Udxa, U_derr=Ue, U_derr_dx=Uedx,
                                U_derr_dx_add=Uedxa)

    # expm parity set: skew-Hermitian generators across every Pade degree
    rng = np.random.default_rng(123)
    As, Es, ms = [], [], []
    for d in (5, 7, 9, 12):
        for norm in (0.01, 0.2, 0.6, 1.5, 4.0, 30.0):
            for _ in range(3):
                H = rng.normal(size=(d, d)) + 1j * rng.normal(size=(d, d))
                H = (H + H.conj().T) / 2
                A = -1j * H / np.abs(H).sum(axis=0).max() * norm
                st = {}
                Es.append(O.julia_exp(A, st))
                As.append(A)
                ms.append(list(st)[0][0])
    out["expm"] = dict(A=np.array(As, dtype=object), E=np.array(Es, dtype=object), m=np.array(ms))

    for name, dct in out.items():
        if name == "expm":
            flat = {}
            for i, (A, E) in enumerate(zip(dct["A"], dct["E"])):
                flat[f"A{i}"] = A
                flat[f"E{i}"] = E
            flat["m"] = dct["m"]
            np.savez_compressed(os.path.join(HERE, "expm.npz"), **flat)
        else:
            np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **dct)
        print("wrote", name)


def make_c5():
    """SURVEY.md 8d C5 (d = 64, N_t = 1024, np = 2; robustgrape_amd/synthetic.py), with the
    oracle's (m, s) Pade histogram.  Separate entry point: ~1 min of oracle time."""
    from robustgrape_amd import synthetic as S
    st = {}
    x = S.dense_x()
    F, Fdx, _, _ = O.calculate_fidelity_and_derivatives(S.dense_problem(), x, st)
    hist = np.array([[m, s, n] for (m, s), n in sorted(st.items())], dtype=np.int64)
    np.savez_compressed(os.path.join(HERE, "c5.npz"), x=x, F=np.float64(F), F_dx=Fdx, pade_hist=hist)
    print("wrote c5", F, hist.tolist())


def make_c5_exact(precomputed=None):
    """Add the exact (longdouble) forward difference of the C5 golden input to c5.npz (F_exact,
    F_dx_exact; oracle/grape_exact.py, ~15 min of CPU): the tests read the oracle's own distance
    from it as the checker's noise.  precomputed: an npz of scripts/probes/dense_exact_probe.py for
    the same x."""
    from oracle import grape_exact as E
    from robustgrape_amd import synthetic as S
    path = os.path.join(HERE, "c5.npz")
    g = dict(np.load(path, allow_pickle=False))
    if precomputed:
        pre = dict(np.load(precomputed, allow_pickle=False))
        assert np.array_equal(pre["x"], g["x"])
        F, Fdx = float(pre["F"]), pre["F_dx"]
    else:
        F, Fdx = E.fidelity_and_gradient(S.dense_problem(), g["x"], nparam=2)
    g["F_exact"], g["F_dx_exact"] = np.float64(F), np.asarray(Fdx)
    np.savez_compressed(path, **g)
    print("c5 exact: oracle - exact", float(np.max(np.abs(g["F_dx"] - Fdx))), "of", float(np.max(np.abs(Fdx))))


def make_xadd_err():
    """Error sources with an H0 and an error generator that read x_add (tests/problems.py
    xadd_err_problem: d = 5, N_t = 40, na = 2, 2 errors), closures through the oracle."""
    d, nt = 5, 40
    x = P.xadd_x(nt, 2024)
    dct = fid(P.xadd_err_problem(d, nt, device=False), x)
    np.savez_compressed(os.path.join(HERE, "xadd_err.npz"), d=np.int64(d), ntimes=np.int64(nt), **dct)
    print("wrote xadd_err", dct["F"], dct["F_d2err"])


def make_c5err():
    """C5 with two error sources (robustgrape_amd/synthetic.py dense_error_problem) at N_t = 64:
    the dense engine's error path (~25 s of oracle time)."""
    from robustgrape_amd import synthetic as S
    nt = 64
    x = S.dense_x(nt, seed=167)
    dct = fid(S.dense_error_problem(64, nt), x)
    np.savez_compressed(os.path.join(HERE, "c5err.npz"), ntimes=np.int64(nt), **dct)
    print("wrote c5err", dct["F"], dct["F_d2err"])


if __name__ == "__main__":
    if sys.argv[1:] == ["c5"]:
        make_c5()
    elif sys.argv[1:2] == ["c5_exact"]:
        make_c5_exact(sys.argv[2] if len(sys.argv) > 2 else None)
    elif sys.argv[1:] == ["c5err"]:
        make_c5err()
    elif sys.argv[1:] == ["xadd_err"]:
        make_xadd_err()
    else:
        main()
