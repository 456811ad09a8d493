"""The reference's forward-difference gradient evaluated WITHOUT rounding in the exponentials and
products: a longdouble (64-bit mantissa) evaluation of exactly the quantity
calculate_fidelity_and_derivatives returns (FidelityCalculations.jl:19-119 with
UnitaryCalculations.jl:44-56: F_dx[k] = Re tr(G U C_k^-1 (exp(A(x_k + d_k)) - exp(A(x_k))) / eps C_{k-1}),
d_k = fl(x_k + eps) - x_k the perturbation the reference actually applies, H built in double as the
reference builds it), against which every implementation's rounding noise can be read off:
the numpy oracle (Julia's exp! restated), the C++ port, and -- on a GPU box -- libgrape's default
path (phase-covariant walks) and its per-step exponentials (GRAPE_OPT_NO_GAUGE).

    python scripts/probes/fd_exact_probe.py [--gpu]   -> one JSON line per case
"""
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import grape_oracle as O  # noqa: E402
from tests import problems as P  # noqa: E402

from oracle.grape_exact import fidelity_and_gradient as exact_fd  # noqa: E402


def cases():
    rng = np.random.default_rng(3)
    yield "sym5_nt40_small", P.sym_problem(40), P.random_x(40, 900, small=True)
    yield "sym5_nt40", P.sym_problem(40), P.random_x(40, 901)
    yield "fullblk7_nt40", P.fullblk_problem(40), P.random_x(40, 902, small=True)
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "c2.npz"), allow_pickle=False))
    yield "full9_c2_golden_x", P.full9_problem(512), g["x"]
    yield "full9_nt96_large_phases", P.full9_problem(96), np.concatenate([rng.uniform(-40, 40, 96), [1.1]])


def main():
    gpu = "--gpu" in sys.argv
    try:
        from oracle.cref import cref
        have_c = cref.available()
    except Exception:
        have_c = False
    for name, fp, x in cases():
        F, ex = exact_fd(fp, x)
        scale = float(np.max(np.abs(ex)))
        out = {"case": name, "max_abs_exact": scale, "F_exact": F}
        impls = {"oracle": lambda: O.calculate_fidelity_and_derivatives(fp, x)[:2]}
        if have_c:
            impls["cref"] = lambda: cref.fidelity_grad(fp, x)[:2]
        if gpu:
            from robustgrape_amd.engine import GrapePlan
            from robustgrape_amd.operators import OPT_NO_GAUGE

            def dev(opts):
                def run():
                    pl = GrapePlan(fp, nparam=1, device=0, max_batch=1, options=opts)
                    try:
                        Fg, Gg, _, _ = pl.fidelity_grad(x[None, :])
                    finally:
                        pl.close()
                    return Fg[0], Gg[0]
                return run
            impls["gpu_default"] = dev(0)
            impls["gpu_no_gauge"] = dev(OPT_NO_GAUGE)
        for k, f in impls.items():
            Fi, gi = f()
            e = np.abs(np.asarray(gi) - ex)
            out[k] = {"dF": abs(float(Fi) - F), "max_abs_err_Fdx": float(e.max()), "rel": float(e.max() / scale),
                      "max_abs_err_Fdx_main": float(e[:-1].max())}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
