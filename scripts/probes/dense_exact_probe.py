"""The exact (longdouble) forward-difference gradient of the C5 golden problem (d = 64, N_t = 1024,
oracle/grape_exact.py) against the oracle's golden F_dx and the C++ port: the noise floor of two
correct double-precision implementations at C5.  CPU only, ~15 min.
    python scripts/probes/dense_exact_probe.py OUT.npz [ntimes]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import grape_exact as E  # noqa: E402
from robustgrape_amd import synthetic as S  # noqa: E402

out = sys.argv[1]
nt = int(sys.argv[2]) if len(sys.argv) > 2 else S.C5_NTIMES
if nt == S.C5_NTIMES:
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "c5.npz"), allow_pickle=False))
    fp, x = S.dense_problem(), g["x"]
else:
    fp, x = S.dense_problem(16, nt, rank=13), S.dense_x(nt, seed=300 + nt)
t = time.time()
F, Fdx = E.fidelity_and_gradient(fp, x, nparam=2)
res = {"F": F, "F_dx": Fdx, "x": x, "seconds": time.time() - t}
if nt == S.C5_NTIMES:
    res["oracle_F_dx"] = g["F_dx"]
try:
    from oracle.cref import cref
    res["cref_F_dx"] = cref.fidelity_grad(fp, x)[1]
except Exception as e:  # noqa: BLE001
    print("no cref:", e)
if nt != S.C5_NTIMES:
    from oracle import grape_oracle as O
    res["oracle_F_dx"] = O.calculate_fidelity_and_derivatives(fp, x)[1]
np.savez(out, **res)
m = np.max(np.abs(Fdx))
for k in ("oracle_F_dx", "cref_F_dx"):
    if k in res:
        e = np.max(np.abs(res[k] - Fdx))
        print(f"{k}: max abs err {e:.3e}  rel {e / m:.3e}  (max|F_dx| {m:.3e})", flush=True)
print(f"{res['seconds']:.0f} s")
