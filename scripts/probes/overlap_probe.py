"""Probe: do two workspaces on two streams overlap one pass's HBM-bound scan with another
pass's VALU-bound exponentials?  C2 (d = 9, N_t = 512), 65 536 evaluations per step in
passes of 16 384: (a) one plan, one stream; (b) two plans, passes alternating between two
streams.  Prints evals/s for each.  Run on the GPU box:  python scripts/probes/overlap_probe.py"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from robustgrape_amd.engine import GrapePlan  # noqa: E402

B, CH, STEPS = 65536, 16384, int(os.environ.get("STEPS", "15"))
dev = torch.device("cuda", 0)
fp = bench.problem()
X = torch.from_numpy(bench.restart_inputs(0, B)).to(dev)
F = torch.empty(B, dtype=torch.float64, device=dev)
Fdx = torch.empty(B, X.shape[1], dtype=torch.float64, device=dev)


def run(nlanes):
    plans = [GrapePlan(fp, nparam=1, device=0, max_batch=CH) for _ in range(nlanes)]
    streams = [torch.cuda.Stream(device=dev) for _ in range(nlanes)]
    for p, s in zip(plans, streams):
        p.set_stream(s.cuda_stream)

    def step():
        for i in range(B // CH):
            j = i % nlanes
            o = i * CH
            plans[j].fidelity_grad_device_async(X[o:].data_ptr(), F[o:].data_ptr(), Fdx[o:].data_ptr(), CH, 0, 0)

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(STEPS):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    for p in plans:
        p.synchronize()
        p.close()
    return STEPS * B / dt


for n in (1, 2, 1, 2):
    print(f"lanes={n}: {run(n):.0f} evals/s", flush=True)
