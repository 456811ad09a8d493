"""A/B of the C2 device step: chunk walks (default) vs the round-2 stored-intermediate sector
kernels (GRAPE_OPT_NO_WALK), same inputs, same stream discipline as bench.py.

    python scripts/probes/walk_ab.py [--batch 262144] [--chunk 32768] [--steps 10] [--opts 0,8]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def run(opts, args, X, F, Fdx, fp):
    import torch
    from robustgrape_amd.engine import GrapePlan
    plan = GrapePlan(fp, nparam=1, device=0, max_batch=min(args.chunk, args.batch), options=opts)
    stream = torch.cuda.Stream()
    plan.set_stream(stream.cuda_stream)
    n = X.shape[0]
    step = lambda: plan.fidelity_grad_device_async(X.data_ptr(), F.data_ptr(), Fdx.data_ptr(), n)  # noqa: E731
    for _ in range(2):
        step()
    plan.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    plan.synchronize()
    dt = time.perf_counter() - t0
    plan.kernel_times(reset=True)
    plan.set_profiling(True)
    for _ in range(2):
        step()
    plan.synchronize()
    kt = {k: round(v[0] / 2, 3) for k, v in plan.kernel_times().items() if v[1]}
    plan.close()
    return {"options": opts, "evals_per_s": args.steps * n / dt, "ms_per_step": dt / args.steps * 1e3,
            "kernel_ms_per_step": kt, "F0": float(F[0]), "Fdx0": float(Fdx[0, 7])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--chunk", type=int, default=32768)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--opts", default="0,8")
    args = ap.parse_args()
    import torch
    import bench
    fp = bench.problem()
    X = torch.from_numpy(bench.restart_inputs(0, args.batch)).cuda()
    F = torch.empty(args.batch, dtype=torch.float64, device="cuda")
    Fdx = torch.empty(args.batch, X.shape[1], dtype=torch.float64, device="cuda")
    for o in args.opts.split(","):
        print(json.dumps(run(int(o), args, X, F, Fdx, fp)), flush=True)


if __name__ == "__main__":
    main()
