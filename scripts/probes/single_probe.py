"""Probe: per-kernel durations of nbatch = 1 host-array calls (C2), for rocprofv3 --kernel-trace --stats."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from robustgrape_amd.engine import GrapePlan  # noqa: E402

plan = GrapePlan(bench.problem(), nparam=1, device=0, max_batch=1)
X = bench.restart_inputs(0, 1)
for _ in range(20):
    plan.fidelity_grad(X)
n = int(os.environ.get("CALLS", "500"))
t = time.perf_counter()
for _ in range(n):
    plan.fidelity_grad(X)
dt = time.perf_counter() - t
print(f"{n / dt:.0f} single evals/s, {dt / n * 1e3:.4f} ms per call")
plan.close()
