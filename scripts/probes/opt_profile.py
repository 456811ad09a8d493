"""Where does a batched L-BFGS iteration spend its time? (torch profiler, one GPU)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from robustgrape_amd import optimize as OPT  # noqa: E402
from robustgrape_amd import regularization as REG  # noqa: E402
from robustgrape_amd.types import FidelityRobustGRAPEParameters  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
fp = bench.problem()
X0 = bench.restart_inputs(0, B)
params = FidelityRobustGRAPEParameters(x_initial=X0[0], regularization_functions=[REG.regularization_cost_phase],
                                       regularization_coeff1=[1e-7], regularization_coeff2=[1e-7],
                                       error_source_coeff=[], iterations=10 ** 9)
cost = OPT.RobustCost(fp, params, nparam=1, max_batch=B, device=0)
dev = torch.device("cuda", 0)
X = torch.as_tensor(X0, device=dev)
calls = [0, 0.0]
per_call = []


def timed(Xs, rows=None):
    torch.cuda.synchronize()
    t = time.perf_counter()
    r = cost(Xs, rows)
    torch.cuda.synchronize()
    calls[0] += 1
    calls[1] += time.perf_counter() - t
    per_call.append((Xs.shape[0], time.perf_counter() - t))
    return r


res = OPT.lbfgs_batched(timed, X, iterations=3, g_tol=0.0)
calls[:] = [0, 0.0]
torch.cuda.synchronize()
t0 = time.perf_counter()
res = OPT.lbfgs_batched(timed, res.minimizer, iterations=10, g_tol=0.0)
torch.cuda.synchronize()
tot = time.perf_counter() - t0
print(f"B={B}: 10 iterations {tot * 1e3:.1f} ms, {calls[0]} cost calls taking {calls[1] * 1e3:.1f} ms "
      f"(evals {int(res.f_calls.sum())})", flush=True)
print("per call (rows, ms):", [(n, round(dt * 1e3, 3)) for n, dt in per_call[-40:]], flush=True)
with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
    OPT.lbfgs_batched(cost, res.minimizer, iterations=3, g_tol=0.0)
print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=25))
cost.close()
