"""Stress of the captured fork/join: small calls whose HIP graphs fork the second
sector class onto the auxiliary stream (plan option GRAPE_OPT_GRAPH_FORK, off by default), mixed
with eager fork/join calls that record and wait on the same plan events, through the graph cache's
eviction (10 batch sizes, 8 cached graphs).  Every output is compared bitwise with a plan that
neither forks nor captures (GRAPE_OPT_NO_FORK | GRAPE_OPT_NO_GRAPH): the fork changes only which
stream a kernel runs on, never its arithmetic.

    python scripts/probes/graph_fork_stress.py c3|c2|xadd ITERATIONS

c3: C3 (two walk classes with error sources); c2: C2 with GRAPE_OPT_NO_PAIR (the two classes as
separate launches, so they fork); xadd: tests/problems.xadd_err_problem(9, 20) (x_add-dependent H0
and errors, three gradient parameters per step), the case that crashed in the GPU suite.  Prints a progress line every 500 iterations and "OK" at the end;
exits 1 at the first mismatch."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from robustgrape_amd.engine import GrapePlan  # noqa: E402
from robustgrape_amd.operators import OPT_GRAPH_FORK, OPT_NO_FORK, OPT_NO_GRAPH, OPT_NO_PAIR  # noqa: E402
from tests import problems as P  # noqa: E402


def main(case, iters):
    if case == "xadd":
        fp, opts = P.xadd_err_problem(9, 20), 0
        X = np.stack([P.xadd_x(20, 500 + s) for s in range(128)])
    else:
        fp = P.full9_problem(512, nerr=4) if case == "c3" else P.full9_problem(512)
        opts = 0 if case == "c3" else OPT_NO_PAIR
        X = np.stack([P.random_x(512, 500 + s) for s in range(128)])
    plan = GrapePlan(fp, nparam=1, device=0, max_batch=128, options=opts | OPT_GRAPH_FORK)
    ref = GrapePlan(fp, nparam=1, device=0, max_batch=128, options=opts | OPT_NO_FORK | OPT_NO_GRAPH)
    assert plan.sectors() == ref.sectors() and len(plan.sectors()) == 2, plan.sectors()
    t0 = time.time()
    try:
        for it in range(iters):
            calls = [(1 + it % 10, (7 * it) % 118)]
            if it % 3 == 1:
                calls.append((100, it % 28))  # an eager fork/join call with the same events
            for nb, b0 in calls:
                rows = X[b0:b0 + nb]
                got, want = plan.fidelity_grad(rows), ref.fidelity_grad(rows)
                for g, w in zip(got, want):
                    if not np.array_equal(g, w):
                        print(f"MISMATCH at iteration {it}, nb {nb}: max |diff| {np.max(np.abs(g - w))}", flush=True)
                        return 1
            if it % 500 == 499:
                print(f"{case}: {it + 1} iterations, {time.time() - t0:.1f} s", flush=True)
    finally:
        plan.close()
        ref.close()
    print(f"{case}: OK, {iters} iterations, graph fork on", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], int(sys.argv[2])))
