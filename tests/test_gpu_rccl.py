"""The sweep's exchange over RCCL on a real device: one rank, "nccl"
process group, device tensors straight from the engine's HBM-resident outputs.

The multi-rank partition and tie rules are covered on CPU with gloo (test_sweep_cpu.py);
this test is the hardware half: the RCCL process group binds to the device, all_gather and
broadcast run on the tensors the engine wrote, and the answer equals the single-process
rule (gather_best_local)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    try:
        from robustgrape_amd.engine import GrapePlan
        from robustgrape_amd.sweep import gather_best, gather_best_local
        from tests import problems as P
        dev = torch.device("cuda", 0)
        fp = P.full9_problem(64, nerr=0)
        n = 40
        X = torch.as_tensor(np.stack([P.random_x(64, 300 + s) for s in range(n)]), device=dev)
        F = torch.empty(n, dtype=torch.float64, device=dev)
        Fdx = torch.empty_like(X)
        plan = GrapePlan(fp, nparam=1, device=0, max_batch=n)
        try:
            plan.set_stream(torch.cuda.current_stream().cuda_stream)
            plan.fidelity_grad_device_async(X.data_ptr(), F.data_ptr(), Fdx.data_ptr(), n, 0, 0)
            plan.synchronize()
        finally:
            plan.close()
        ids = torch.arange(100, 100 + n, device=dev)
        fb, rid, owner, xb = gather_best(F, ids, X)
        fl, ridl, _, xl = gather_best_local(F, ids, X)
        t = torch.tensor([1.5], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)   # bench.py's max-over-ranks timing
        dist.barrier()
        q.put((fb, rid, owner, fl, ridl, bool(torch.equal(xb, xl)), xb.device.type, float(t.item()),
               float(F.max().item())))
    finally:
        dist.destroy_process_group()


def test_gather_best_over_rccl():
    import torch
    import torch.multiprocessing as mp
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    try:
        fb, rid, owner, fl, ridl, same_x, xdev, t, fmax = q.get(timeout=240)
    finally:
        p.join(timeout=60)
    assert p.exitcode == 0
    assert fb == fl == fmax and rid == ridl and owner == 0
    assert same_x and xdev == "cuda"
    assert t == 1.5
