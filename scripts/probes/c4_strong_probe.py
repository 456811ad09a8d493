"""Probe: bench.py's C4 strong leg on its own (one rank), eval1 on and off, and c4_points' loop for
comparison -- where does the per-round time of the sweep go?"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from robustgrape_amd.engine import GrapePlan  # noqa: E402
from robustgrape_amd.operators import OPT_NO_EVAL1  # noqa: E402

dev = torch.device("cuda:0")
fp = bench.problem()
stream = torch.cuda.Stream(device=dev)
for opts in (0, OPT_NO_EVAL1):
    def make_step(f, c, opts=opts):
        p = GrapePlan(fp, nparam=1, device=0, max_batch=max(1, c), options=opts)
        p.set_stream(stream.cuda_stream)
        Xs = torch.from_numpy(bench.restart_inputs(f, c)).to(dev)
        Fs = torch.empty(c, dtype=torch.float64, device=dev)
        Gs = torch.empty(c, Xs.shape[1], dtype=torch.float64, device=dev)
        return ((lambda: p.fidelity_grad_device_async(Xs.data_ptr(), Fs.data_ptr(), Gs.data_ptr(), c, 0, 0)),
                Fs, Xs, torch.arange(f, f + c, device=dev), p.close)
    for rep in range(2):
        r = bench.c4_strong(make_step, 1, 0, False, torch.cuda.synchronize, total=256)
        print(f"opts {opts}: c4_strong {r['ms_per_eval_round']:.4f} ms per round (run {rep})", flush=True)
    from robustgrape_amd.sweep import gather_best_local
    step, F, X, ids, close = make_step(0, 256)
    for _ in range(300):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(100):
        step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    gather_best_local(F, ids, X)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"opts {opts}: steps {(t1 - t) * 1e3:.3f} ms, gather {(t2 - t1) * 1e3:.3f} ms", flush=True)
    close()
    step, F, X, ids, close = make_step(0, 256)
    for _ in range(100):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(100):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"opts {opts}: 100 steps enqueue {(t1 - t) * 1e3:.3f} ms, until done {(t2 - t) * 1e3:.3f} ms", flush=True)
    close()
