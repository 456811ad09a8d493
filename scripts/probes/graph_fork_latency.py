"""Single-evaluation latency (host arrays, nbatch = 1, the graph path) of C3 and of C2 with
GRAPE_OPT_NO_PAIR, with and without the captured fork (GRAPE_OPT_GRAPH_FORK).
    python scripts/probes/graph_fork_latency.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from robustgrape_amd.engine import GrapePlan  # noqa: E402
from robustgrape_amd.operators import OPT_GRAPH_FORK, OPT_NO_PAIR  # noqa: E402
from tests import problems as P  # noqa: E402

for (case, fp, opts), nofork in [(c, f) for c in (("c3", P.full9_problem(512, nerr=4), 0),
                                                  ("c2-nopair", P.full9_problem(512), OPT_NO_PAIR),
                                                  ("c2", P.full9_problem(512), 0)) for f in (True, False)]:
    plan = GrapePlan(fp, nparam=1, device=0, max_batch=1, options=opts | (0 if nofork else OPT_GRAPH_FORK))
    X = P.random_x(512, 3)[None, :]
    for _ in range(20):
        plan.fidelity_grad(X)
    lat = []
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 2.0:
        t = time.perf_counter()
        plan.fidelity_grad(X)
        lat.append(time.perf_counter() - t)
    plan.close()
    print(f"{case}: graph fork {'off' if nofork else 'on'} median {np.median(lat) * 1e3:.4f} ms "
          f"p10 {np.percentile(lat, 10) * 1e3:.4f} ms ({len(lat)} calls)", flush=True)
