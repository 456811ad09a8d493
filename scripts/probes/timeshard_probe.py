"""Probe: latency of ONE C5 evaluation (d = 64, N_t = 1 024) whole vs time-sharded.

Prints the whole-evaluation call, the sliced evaluation run as virtual ranks on this one GPU
(slices one after another: what R GPUs would do in parallel, in sequence), and per slice the
forward and gradient calls -- the critical path of an R-GPU run is one slice's forward, the
exchange, and one slice's gradient.  Under torchrun (WORLD_SIZE > 1, nccl) it times the real
sharded call instead."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from robustgrape_amd.engine import GrapePlan  # noqa: E402
from robustgrape_amd.synthetic import dense_problem, dense_x  # noqa: E402
from robustgrape_amd import timeshard as TS  # noqa: E402


def best(fn, n=5):
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return min(ts) * 1e3


fp, x = dense_problem(), dense_x()
world = int(os.environ.get("WORLD_SIZE", "1"))
if world > 1:
    import torch
    import torch.distributed as dist
    rank = int(os.environ["RANK"])
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group("nccl")
    TS.time_sharded_fidelity_grad(fp, x, nparam=2, device=torch.cuda.current_device())
    ms = best(lambda: TS.time_sharded_fidelity_grad(fp, x, nparam=2, device=torch.cuda.current_device()))
    if rank == 0:
        print(f"C5 time-sharded over {world} ranks: {ms:.2f} ms per evaluation")
    dist.destroy_process_group()
    sys.exit(0)
pl = GrapePlan(fp, 2, max_batch=1)
pl.fidelity_grad(x[None, :])
whole = best(lambda: pl.fidelity_grad(x[None, :]))
print(f"C5 whole evaluation: {whole:.2f} ms")
for R in (2, 4, 8):
    TS.time_sharded_fidelity_grad(fp, x, nparam=2, nslices=R)
    seq = best(lambda: TS.time_sharded_fidelity_grad(fp, x, nparam=2, nslices=R))
    a, b = TS.slice_bounds(fp.unitary_problem.ntimes, R)[0]
    sp = TS._slice_plan(fp, 2, a, b, 0)
    fwd = best(lambda: sp.forward(x[2 * a:2 * b]))
    M = np.eye(fp.unitary_problem.ndim, dtype=np.complex128)
    grad = best(lambda: sp.gradient(M))
    print(f"  {R} slices: sequential on one GPU {seq:.2f} ms; one slice forward {fwd:.2f} ms + gradient "
          f"{grad:.2f} ms (the {R}-GPU critical path without the exchange: {fwd + grad:.2f} ms)")
    # device exchange: totals, head, M' and F_dx stay device tensors (grape_slice_*_device)
    import torch
    TS.time_sharded_fidelity_grad(fp, x, nparam=2, nslices=R, device_exchange=True)
    seqd = best(lambda: TS.time_sharded_fidelity_grad(fp, x, nparam=2, nslices=R, device_exchange=True))
    xt = torch.as_tensor(x[2 * a:2 * b], device="cuda:0")
    Mt = torch.eye(fp.unitary_problem.ndim, dtype=torch.complex128, device="cuda:0")

    def one_slice():
        sp.forward_device(xt)
        sp.gradient_device(Mt)
        torch.cuda.synchronize()
    one_slice()
    fg = best(one_slice)
    print(f"  {R} slices, device exchange: sequential on one GPU {seqd:.2f} ms; one slice forward + "
          f"gradient on device buffers {fg:.2f} ms")
pl.close()
