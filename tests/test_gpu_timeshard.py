"""Time-sharded single evaluations on the MI355X (robustgrape_amd/timeshard.py,
grape_slice_forward / grape_slice_gradient of include/grape.h).

Slices run one after another on the one device ("virtual ranks"; the exchange over ranks is the
gloo-tested code of tests/test_timeshard_cpu.py): F and F_dx of the sliced evaluation against the
oracle (UnitaryCalculations.jl:20-155, FidelityCalculations.jl:19-119) and against a
whole-evaluation call of the dense engine -- the same algebra with the chain products associated
slice by slice, so F within T1 and F_dx within the FD tier: against the oracle T2 (1e-6 max|ref|)
+ 1e-9 + the oracle's own distance from the exact forward difference (oracle/grape_exact.py; at
d = 16 the oracle sits ~5.8e-7 of max|F_dx| from it, tests/test_gpu_dense.py), against a whole
call of the same engine 1e-6 max|ref| + 1e-9."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
T1 = 1e-12
T2, T2_ABS = 1e-6, 1e-9


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _check(test, F, Fdx, F0, g0, t2=T2, t2a=T2_ABS):
    from tests.parity_log import record
    ef = abs(float(F) - float(F0))
    record(test, "F", ef, 1.0, T1)
    assert ef <= T1, (test, F, F0)
    err, scale = float(np.max(np.abs(Fdx - g0))), float(np.max(np.abs(g0)))
    record(test, "F_dx", err, scale, t2 * scale + t2a)
    print(f"{test}: |dF| {ef:.2e}  max|dF_dx| {err:.2e} (scale {scale:.2e})")
    assert err <= t2 * scale + t2a, (test, err, scale)


@pytest.mark.parametrize("nslices", [1, 2, 3, 4])
def test_sliced_evaluation_matches_oracle_and_whole_call(nslices):
    from oracle import grape_oracle as O
    from robustgrape_amd.engine import GrapePlan
    from robustgrape_amd.synthetic import dense_problem, dense_x
    from robustgrape_amd.timeshard import time_sharded_fidelity_grad
    fp = dense_problem(d=16, ntimes=48, dt=0.3, rank=6)
    x = dense_x(ntimes=48, seed=5)
    from oracle import grape_exact as E
    F, Fdx = time_sharded_fidelity_grad(fp, x, nparam=2, nslices=nslices)
    F0, g0 = O.calculate_fidelity_and_derivatives(fp, x)[:2]
    Fe, ge = E.fidelity_and_gradient(fp, x, nparam=2)
    _check(f"timeshard_d16_s{nslices}_exact", F, Fdx, Fe, ge)
    _check(f"timeshard_d16_s{nslices}_oracle", F, Fdx, F0, np.asarray(g0),
           t2a=T2_ABS + float(np.max(np.abs(np.asarray(g0) - ge))))
    pl = GrapePlan(fp, 2, max_batch=1)
    try:
        Fw, gw = pl.fidelity_grad(x[None, :])[:2]
    finally:
        pl.close()
    _check(f"timeshard_d16_s{nslices}_whole", F, Fdx, Fw[0], gw[0])


def test_c5_sliced_eight_ways_matches_whole_call():
    """C5 itself (d = 64, N_t = 1 024, np = 2) in 8 slices of 128 steps -- the 8-GPU layout --
    against one whole-evaluation call and the committed C5 golden."""
    import os
    from robustgrape_amd.engine import GrapePlan
    from robustgrape_amd.synthetic import dense_problem
    from robustgrape_amd.timeshard import time_sharded_fidelity_grad
    g = dict(np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c5.npz"),
                     allow_pickle=False))
    fp = dense_problem()
    x = g["x"]
    F, Fdx = time_sharded_fidelity_grad(fp, x, nparam=2, nslices=8)
    noise = 0.0
    if "F_dx_exact" in g:  # the golden's distance from the exact forward difference (make_golden.py)
        _check("timeshard_c5_exact", F, Fdx, float(g["F_exact"]), g["F_dx_exact"])
        noise = float(np.max(np.abs(g["F_dx"] - g["F_dx_exact"])))
    _check("timeshard_c5_golden", F, Fdx, float(g["F"]), g["F_dx"], t2a=T2_ABS + noise)
    pl = GrapePlan(fp, 2, max_batch=1)
    try:
        Fw, gw = pl.fidelity_grad(x[None, :])[:2]
    finally:
        pl.close()
    _check("timeshard_c5_whole", F, Fdx, Fw[0], gw[0])


def test_slices_refuse_unsupported_plans():
    """Slice calls need the dense engine (12 < d <= 64) without x_add / error sources."""
    from robustgrape_amd._capi import GrapeError
    from robustgrape_amd.synthetic import dense_problem
    from robustgrape_amd.timeshard import SlicePlan
    sp = SlicePlan(dense_problem(d=8, ntimes=8, dt=0.3, rank=4), 2, 0, 8)  # d <= 12: the small engine
    try:
        with pytest.raises(GrapeError):
            sp.forward(np.zeros(16))
    finally:
        sp.close()


@pytest.mark.parametrize("nslices", [1, 3, 8])
def test_device_exchange_matches_host_exchange(nslices):
    """grape_slice_forward_device / grape_slice_gradient_device with the chain, head and M' as
    device tensors (the nccl path of time_sharded_fidelity_grad, here with the slices in order):
    the same F and F_dx as the host-staged exchange (rocBLAS products instead of numpy's: 1e-14)
    and as the oracle."""
    from oracle import grape_oracle as O
    from robustgrape_amd.synthetic import dense_problem, dense_x
    from robustgrape_amd.timeshard import time_sharded_fidelity_grad
    fp = dense_problem(d=24, ntimes=40, dt=0.3, rank=8)
    x = dense_x(ntimes=40, seed=9)
    Fh, gh = time_sharded_fidelity_grad(fp, x, nparam=2, nslices=nslices)
    Fd, gd = time_sharded_fidelity_grad(fp, x, nparam=2, nslices=nslices, device_exchange=True)
    assert abs(Fd - Fh) <= 1e-14
    assert np.max(np.abs(gd - gh)) <= 1e-14 * max(1.0, float(np.max(np.abs(gh))))
    from oracle import grape_exact as E
    F0, g0 = O.calculate_fidelity_and_derivatives(fp, x)[:2]
    Fe, ge = E.fidelity_and_gradient(fp, x, nparam=2)
    _check(f"timeshard_device_s{nslices}_exact", Fd, gd, Fe, ge)
    _check(f"timeshard_device_s{nslices}_oracle", Fd, gd, F0, np.asarray(g0),
           t2a=T2_ABS + float(np.max(np.abs(np.asarray(g0) - ge))))


def _device_exchange_worker(rank, world, port, q):
    import os
    import torch
    import torch.distributed as dist
    from robustgrape_amd.synthetic import dense_problem, dense_x
    from robustgrape_amd.timeshard import time_sharded_fidelity_grad
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fp = dense_problem(d=24, ntimes=41, dt=0.3, rank=8)
        F, Fdx = time_sharded_fidelity_grad(fp, dense_x(ntimes=41, seed=9), nparam=2, device_exchange=True)
        q.put((rank, F, Fdx.tolist()))
    finally:
        dist.destroy_process_group()


def test_ranks_exchange_device_buffers():
    """The rank path of the device exchange (all_gathers of device tensors; gloo's CUDA all_gather
    here, RCCL on a multi-GPU node), two ranks sharing this GPU, ragged slices (21 + 20 steps: the
    padded F_dx all_gather): every rank returns the oracle's F and F_dx."""
    import socket
    import torch.multiprocessing as mp
    from oracle import grape_oracle as O
    from robustgrape_amd.synthetic import dense_problem, dense_x
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_device_exchange_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=100) for _ in range(2)]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    from oracle import grape_exact as E
    fp = dense_problem(d=24, ntimes=41, dt=0.3, rank=8)
    F0, g0 = O.calculate_fidelity_and_derivatives(fp, dense_x(ntimes=41, seed=9))[:2]
    Fe, ge = E.fidelity_and_gradient(fp, dense_x(ntimes=41, seed=9), nparam=2)
    for r, F, Fdx in out:
        _check(f"timeshard_device_rank{r}_exact", F, np.asarray(Fdx), Fe, ge)
        _check(f"timeshard_device_rank{r}_oracle", F, np.asarray(Fdx), F0, np.asarray(g0),
               t2a=T2_ABS + float(np.max(np.abs(np.asarray(g0) - ge))))


def test_rank_path_plan_follows_the_current_device():
    """on the rank path the slice plan is built on the current torch device (the rank's
    GPU under torchrun), where the slice tensors and the side stream live; an explicit `device`
    other than the current one is refused with the device exchange."""
    import os
    import socket
    import torch
    import torch.distributed as dist
    from robustgrape_amd import timeshard as TS
    from robustgrape_amd.synthetic import dense_problem, dense_x
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    own = not dist.is_initialized()
    if own:
        dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        fp = dense_problem(d=16, ntimes=6, dt=0.3, rank=8)
        x = dense_x(ntimes=6, seed=3)
        seen = []
        real = TS._slice_plan
        TS._slice_plan = lambda fp_, nparam, k0, k1, device, keep=0: seen.append(device) or real(
            fp_, nparam, k0, k1, device, keep)
        try:
            F, _ = TS.time_sharded_fidelity_grad(fp, x, nparam=2, device_exchange=True)
        finally:
            TS._slice_plan = real
        assert seen == [torch.cuda.current_device()] and np.isfinite(F)
        with pytest.raises(ValueError):
            TS.time_sharded_fidelity_grad(fp, x, nparam=2, device_exchange=True,
                                          device=torch.cuda.current_device() + 1)
    finally:
        if own:
            dist.destroy_process_group()
