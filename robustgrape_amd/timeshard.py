"""Time sharding of ONE evaluation (the optional C5 mode).

The restart sweep (sweep.py) shards independent evaluations; a single large evaluation (C5:
d = 64, N_t = 1024) can instead split its time steps.  Slice r of R owns the contiguous steps
[k_r, k_{r+1}) and runs them as a problem of its own on its device (a slice plan: the same H0,
N_t = the slice's steps, the same dt):

1. forward (grape_slice_forward): the slice's propagators and chunk prefixes stay on the device;
   its total S_r = E_{k_{r+1}-1} ... E_{k_r} comes back (d x d);
2. one exchange: all_gather of the R totals (R d^2 complex: 512 KB at d = 64, R = 8);
3. every rank forms U = S_{R-1} ... S_0, the fidelity and M = G U from the reference's
   expressions (FidelityCalculations.jl:47-63, here on the host: d x d work), and its carry
   B_r = S_{r-1} ... S_0;
4. gradient (grape_slice_gradient): F_dx[p, k] = Re tr(G U_dx[p, k]) with
   U_dx[p, k] = U C_k^-1 dE C_{k-1} and C_k = Q_k B_r (Q_k the slice-local prefix) is
   Re tr(M' Q_k^dag dE Q_{k-1}) with M' = B_r M B_r^dag -- the slice plan's own gradient
   pipeline with M' in place of its M;
5. all_gather of the F_dx slices.

Same algebra as the engine's chunked scan (the slices are chunks one level up), so F and F_dx
agree with a whole-evaluation call to rounding (the products associate differently):
tests/test_gpu_timeshard.py.  Multi-rank exchanges go through torch.distributed (RCCL over xGMI
on GPUs, gloo for the CPU tests of the exchange logic); without a process group the slices run
one after another on one device ("virtual ranks")."""
from __future__ import annotations

import ctypes
from collections import OrderedDict

import numpy as np

from . import _capi
from .types import FidelityRobustGRAPEProblem

__all__ = ["slice_bounds", "slice_problem", "SlicePlan", "fidelity_head", "time_sharded_fidelity_grad"]


def slice_bounds(ntimes: int, nslices: int):
    """Contiguous step ranges [(k_0, k_1), ...] of nearly equal length (the first ones longer)."""
    if nslices < 1 or nslices > ntimes:
        raise ValueError("need 1 <= nslices <= ntimes")
    q, r = divmod(ntimes, nslices)
    out, k = [], 0
    for s in range(nslices):
        n = q + (1 if s < r else 0)
        out.append((k, k + n))
        k += n
    return out


def slice_problem(fp: FidelityRobustGRAPEProblem, k0: int, k1: int) -> FidelityRobustGRAPEProblem:
    """The steps [k0, k1) of fp as a problem of their own: same H0, dt, projector and target."""
    up = fp.unitary_problem
    if up.nb_additional_param or up.error_sources:
        raise ValueError("time slices: problems without x_add and error sources (the C5 family)")
    dt = up.t0 / up.ntimes
    return fp.replace(unitary_problem=up.replace(t0=dt * (k1 - k0), ntimes=k1 - k0))


class SlicePlan:
    """A device plan of one time slice (grape_slice_forward / grape_slice_gradient)."""

    def __init__(self, fp: FidelityRobustGRAPEProblem, nparam: int, k0: int, k1: int, device: int = 0):
        from .engine import GrapePlan
        self.k0, self.k1, self.nparam = int(k0), int(k1), int(nparam)
        self.source = fp  # the problem the plan was built for (kept alive: _slice_plan's key is its id)
        self.d = fp.unitary_problem.ndim
        self.plan = GrapePlan(slice_problem(fp, k0, k1), nparam, device=device, max_batch=1)

    def forward(self, x_slice) -> np.ndarray:
        """The slice's total propagator (d x d complex); keeps its propagators on the device."""
        x = np.ascontiguousarray(x_slice, dtype=np.float64)
        if x.shape != (self.nparam * (self.k1 - self.k0),):
            raise AssertionError("slice controls: nparam * steps values")
        U = np.empty((self.d, self.d), dtype=np.complex128, order="F")
        _capi.check(_capi.lib().grape_slice_forward(self.plan.handle, _capi.dptr(x),
                                                    U.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
        return np.ascontiguousarray(U)

    def gradient(self, M_prime) -> np.ndarray:
        """The slice's F_dx entries (nparam * steps) for M' = B M B^dag."""
        Mp = np.asfortranarray(M_prime, dtype=np.complex128)
        g = np.empty(self.nparam * (self.k1 - self.k0))
        _capi.check(_capi.lib().grape_slice_gradient(self.plan.handle,
                                                     Mp.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                                     _capi.dptr(g)))
        return g

    # device buffers (grape_slice_*_device).  The plan runs on a side stream ordered after the
    # caller's current torch stream and joined back into it (a null current stream cannot be handed
    # to grape_plan_set_stream, which takes 0 for the plan's own, non-blocking stream).
    def _enqueue(self, dev, call):
        import torch
        cur = torch.cuda.current_stream(dev)
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(device=dev)
        self._side.wait_stream(cur)
        self.plan.set_stream(self._side.cuda_stream)
        call()
        cur.wait_stream(self._side)

    def forward_device(self, x_t):
        """forward() on a device tensor; returns the total as a (d, d) complex128 device tensor."""
        import torch
        if tuple(x_t.shape) != (self.nparam * (self.k1 - self.k0),) or x_t.dtype != torch.float64:
            raise AssertionError("slice controls: nparam * steps float64 values")
        x_t = x_t.contiguous()
        Ut = torch.empty(self.d, self.d, dtype=torch.complex128, device=x_t.device)  # column-major U = Ut^T
        self._enqueue(x_t.device, lambda: _capi.check(_capi.lib().grape_slice_forward_device(
            self.plan.handle, ctypes.c_void_p(x_t.data_ptr()), ctypes.c_void_p(Ut.data_ptr()))))
        return Ut.transpose(0, 1)

    def gradient_device(self, M_prime_t):
        """gradient() for a (d, d) complex128 device tensor M'; returns a float64 device tensor
        (synchronise with plan.synchronize() before trusting it: it reports a singular Pade)."""
        import torch
        Mc = M_prime_t.transpose(0, 1).contiguous()  # column-major storage of M'
        g = torch.empty(self.nparam * (self.k1 - self.k0), dtype=torch.float64, device=Mc.device)
        self._enqueue(Mc.device, lambda: _capi.check(_capi.lib().grape_slice_gradient_device(
            self.plan.handle, ctypes.c_void_p(Mc.data_ptr()), ctypes.c_void_p(g.data_ptr()))))
        return g

    def close(self):
        self.plan.close()


def fidelity_head(fp: FidelityRobustGRAPEProblem, U: np.ndarray, x_add=()):
    """F and M = G U of the whole evaluation from its U (FidelityCalculations.jl:47-63):
    P0 = projector, P = (P0 != 0), D = Re tr(P0), K = U0^dag U, tau = tr(P0 P K),
    F = [Re tr(P0 P K P K^dag) + |tau|^2] / (D (D + 1)),
    M = [(P K^dag P0 P + P^T K^dag (P0 P)^dag) K + 2 conj(tau) P0 P K] / (D (D + 1))
    (dF = Re tr(G dU), the engine's general-projector head, grape_projector.hip)."""
    P0 = np.asarray(fp.projector, dtype=np.float64)
    P = (P0 != 0).astype(np.float64)
    D = float(np.trace(P0).real)
    DD = D * (D + 1.0)
    U0 = np.asarray(fp.target_unitary(np.asarray(x_add, dtype=np.float64)), dtype=np.complex128)
    K = U0.conj().T @ U
    A, B = P0 @ P, P
    tau = np.trace(A @ K)
    F = (np.trace(A @ K @ B @ K.conj().T).real + abs(tau) ** 2) / DD
    M = ((B @ K.conj().T @ A + B.T @ K.conj().T @ A.conj().T) @ K + 2.0 * np.conj(tau) * (A @ K)) / DD
    return float(F), M


def fidelity_head_torch(fp: FidelityRobustGRAPEProblem, U):
    """fidelity_head on a device tensor U (the same expressions in torch): (F as a 0-d tensor, M)."""
    import torch
    dev = U.device
    P0 = torch.as_tensor(np.asarray(fp.projector, dtype=np.float64), device=dev).to(torch.complex128)
    P = (P0 != 0).to(torch.complex128)
    D = float(np.trace(np.asarray(fp.projector, dtype=np.float64)))
    DD = D * (D + 1.0)
    U0 = torch.as_tensor(np.asarray(fp.target_unitary(np.zeros(0)), dtype=np.complex128), device=dev)
    K = U0.conj().T @ U
    A, B = P0 @ P, P
    tau = torch.trace(A @ K)
    F = (torch.trace(A @ K @ B @ K.conj().T).real + torch.abs(tau) ** 2) / DD
    M = ((B @ K.conj().T @ A + B.T @ K.conj().T @ A.conj().T) @ K + 2.0 * torch.conj(tau) * (A @ K)) / DD
    return F, M


def _chain_torch(mats, d, dev):
    import torch
    out = torch.eye(d, dtype=torch.complex128, device=dev)
    for S in mats:
        out = S @ out
    return out


_plans: "OrderedDict[tuple, SlicePlan]" = OrderedDict()
_KEEP = 16


def _slice_plan(fp, nparam, k0, k1, device, keep=_KEEP):
    """The cached slice plan of (fp, nparam, [k0, k1), device).  The key holds id(fp); the plan
    holds fp itself (`source`), so the id cannot be recycled while the entry lives, and an entry
    whose source is not fp (or whose plan was closed) is rebuilt -- as engine.get_plan guards
    with `ent.fp is fp`.  `keep`: entries the caller needs alive at once (a call over nslices
    plans on one device), so the LRU never closes a plan of the call in progress."""
    key = (id(fp), nparam, k0, k1, device)
    sp = _plans.pop(key, None)
    if sp is not None and (sp.source is not fp or sp.plan.handle is None):
        sp.close()
        sp = None
    if sp is None:
        sp = SlicePlan(fp, nparam, k0, k1, device)
    _plans[key] = sp
    while len(_plans) > max(_KEEP, keep):
        _plans.popitem(last=False)[1].close()
    return sp


def clear_slice_plans():
    while _plans:
        _plans.popitem()[1].close()


def _chain(mats, d):
    """mats[-1] ... mats[0] (later slices act on the left: C_k = E_k C_{k-1}); I for none."""
    out = np.eye(d, dtype=np.complex128)
    for S in mats:
        out = S @ out
    return out


def time_sharded_fidelity_grad(fp: FidelityRobustGRAPEProblem, x, nparam: int, nslices: int | None = None,
                               group=None, device: int | None = None, device_exchange: bool | None = None):
    """(F, F_dx) of ONE evaluation with its time steps split into slices.

    group: a torch.distributed process group (or the default group when torch.distributed is
    initialised and group is None and nslices is None): one slice per rank, two all_gathers.
    Otherwise `nslices` slices run one after another on `device`.  Every rank returns the full
    (F, F_dx).  device_exchange (default: with the nccl backend; optional for the in-order slices):
    slice totals, the chain, the head, M' and the F_dx slices stay device tensors
    (grape_slice_*_device, RCCL all_gathers of device buffers); only F and F_dx come back.
    device: the GPU of the slice plan(s); default: the current torch device on the rank path (under
    torchrun with torch.cuda.set_device(local_rank): the rank's own GPU), 0 for the in-order slices.
    On the rank path the plan, the slice tensors and the side stream are all on that device; a
    `device` other than the current one with the device exchange is refused (ValueError)."""
    up = fp.unitary_problem
    x = np.ascontiguousarray(x, dtype=np.float64)
    if x.shape != (nparam * up.ntimes,):
        raise AssertionError("Control parameter size must be a multiple of time steps")
    dist = None
    if nslices is None:
        import torch.distributed as dist
        if not dist.is_initialized():
            raise ValueError("nslices is required without a torch.distributed process group")
        nslices = dist.get_world_size(group)
        rank = dist.get_rank(group)
    bounds = slice_bounds(up.ntimes, nslices)
    if dist is None and device is None:
        device = 0
    if dist is None and device_exchange:  # virtual ranks, device buffers throughout
        import torch
        dev = torch.device("cuda", device)
        xt = torch.as_tensor(x, device=dev)
        plans = [_slice_plan(fp, nparam, a, b, device, keep=nslices) for a, b in bounds]
        totals = [sp.forward_device(xt[a * nparam:b * nparam]) for sp, (a, b) in zip(plans, bounds)]
        F, M = fidelity_head_torch(fp, _chain_torch(totals, up.ndim, dev))
        grads = []
        for r, sp in enumerate(plans):
            B = _chain_torch(totals[:r], up.ndim, dev)
            grads.append(sp.gradient_device(B @ M @ B.conj().T))
        Fdx = torch.cat(grads)
        for sp in plans:
            sp.plan.synchronize()
        return float(F.item()), Fdx.cpu().numpy()
    if dist is None:  # virtual ranks: every slice here, in order
        plans = [_slice_plan(fp, nparam, a, b, device, keep=nslices) for a, b in bounds]
        totals = [sp.forward(x[a * nparam:b * nparam]) for sp, (a, b) in zip(plans, bounds)]
        F, M = fidelity_head(fp, _chain(totals, up.ndim))
        grads = []
        for r, sp in enumerate(plans):
            B = _chain(totals[:r], up.ndim)
            grads.append(sp.gradient(B @ M @ B.conj().T))
        return F, np.concatenate(grads)
    import torch
    a, b = bounds[rank]
    backend = dist.get_backend(group)
    if device_exchange is None:
        device_exchange = backend == "nccl"
    if device is None:
        device = torch.cuda.current_device() if (device_exchange or backend == "nccl") else 0
    elif device_exchange and device != torch.cuda.current_device():
        raise ValueError(f"device={device} but the current torch device is {torch.cuda.current_device()}: the "
                         "device exchange keeps the slice tensors on the current device")
    sp = _slice_plan(fp, nparam, a, b, device)
    if device_exchange:  # device buffers throughout: two RCCL all_gathers, no host staging
        dev = torch.device("cuda", device)
        d = up.ndim
        S = torch.view_as_real(sp.forward_device(torch.as_tensor(x[a * nparam:b * nparam], device=dev)).contiguous())
        got = [torch.empty_like(S) for _ in range(nslices)]
        dist.all_gather(got, S, group=group)  # the one exchange of slice totals (as real pairs)
        got = [torch.view_as_complex(t) for t in got]
        F, M = fidelity_head_torch(fp, _chain_torch(got, d, dev))
        B = _chain_torch(got[:rank], d, dev)
        g = sp.gradient_device(B @ M @ B.conj().T)
        width = max(nb - na for na, nb in bounds) * nparam
        pad = torch.zeros(width, dtype=torch.float64, device=dev)
        pad[:g.numel()] = g
        parts = [torch.empty_like(pad) for _ in range(nslices)]
        dist.all_gather(parts, pad, group=group)  # the F_dx slices
        Fdx = torch.cat([parts[r][:(nb - na) * nparam] for r, (na, nb) in enumerate(bounds)])
        sp.plan.synchronize()
        return float(F.item()), Fdx.cpu().numpy()
    S = sp.forward(x[a * nparam:b * nparam])
    dev = torch.device("cuda", device) if backend == "nccl" else torch.device("cpu")
    d = up.ndim
    mine = torch.from_numpy(np.ascontiguousarray(S).view(np.float64).reshape(d, d, 2)).to(dev)
    got = [torch.empty_like(mine) for _ in range(nslices)]
    dist.all_gather(got, mine, group=group)  # the one exchange of slice totals
    totals = [g.cpu().numpy().reshape(d, 2 * d).view(np.complex128).reshape(d, d) for g in got]
    F, M = fidelity_head(fp, _chain(totals, up.ndim))
    B = _chain(totals[:rank], up.ndim)
    g = sp.gradient(B @ M @ B.conj().T)
    width = max(nb - na for na, nb in bounds) * nparam
    pad = torch.zeros(width, dtype=torch.float64, device=dev)
    pad[:g.size] = torch.from_numpy(g).to(dev)
    parts = [torch.empty_like(pad) for _ in range(nslices)]
    dist.all_gather(parts, pad, group=group)  # the F_dx slices
    Fdx = np.concatenate([parts[r].cpu().numpy()[:(nb - na) * nparam] for r, (na, nb) in enumerate(bounds)])
    return F, Fdx
