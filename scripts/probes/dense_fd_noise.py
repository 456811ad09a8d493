"""Dense-engine F_dx against the oracle at C5 (golden) and d = 16 (live oracle), for the library
named by GRAPE_LIB (A/B of the Gauss-3M and the 4M complex product).
    GRAPE_LIB=robustgrape_amd/libgrape_4m.so python scripts/probes/dense_fd_noise.py TAG
Prints one JSON line: absolute and relative (to max|ref|) errors, and saves F_dx to gpurun_out/."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from robustgrape_amd import _capi, synthetic as S  # noqa: E402
from robustgrape_amd import calculate_fidelity_and_derivatives  # noqa: E402
from oracle import grape_oracle as O  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "lib"
out = {"lib": _capi.LIB_PATH, "build": _capi.build_id()}
g = dict(np.load(os.path.join(ROOT, "tests", "golden", "c5.npz"), allow_pickle=False))
F, Fdx, _, _ = calculate_fidelity_and_derivatives(S.dense_problem(), g["x"])
m = np.max(np.abs(g["F_dx"]))
out["c5"] = {"dF": abs(F - float(g["F"])), "abs": float(np.max(np.abs(Fdx - g["F_dx"]))),
             "rel": float(np.max(np.abs(Fdx - g["F_dx"])) / m), "max_ref": float(m)}
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.save(os.path.join(ROOT, "gpurun_out", f"c5_fdx_{tag}.npy"), Fdx)
for d, nt in ((16, 5), (64, 37)):
    fp = S.dense_problem(d, nt, rank=min(16, d - 3))
    x = S.dense_x(nt, seed=300 + nt)
    F0, g0, _, _ = O.calculate_fidelity_and_derivatives(fp, x)
    F1, g1, _, _ = calculate_fidelity_and_derivatives(fp, x)
    e = float(np.max(np.abs(g1 - g0)))
    out[f"d{d}_nt{nt}"] = {"dF": abs(F1 - F0), "abs": e, "rel": e / float(np.max(np.abs(g0))),
                           "max_ref": float(np.max(np.abs(g0)))}
print(json.dumps(out), flush=True)
