"""Host side of the GPU path: plans over libgrape.so and the reference's functions.

``calculate_fidelity_and_derivatives`` mirrors src/FidelityCalculations.jl:19-119
(same arguments, same return tuple, AssertionError on a bad x shape as
src/UnitaryCalculations.jl:22) and additionally accepts a 2-D ``x`` of shape
(nbatch, n_x) to evaluate a batch of control vectors in one device pass.
"""
from __future__ import annotations

import contextlib
import ctypes
import threading
from collections import OrderedDict

import numpy as np

from . import _capi
from .operators import OPT_GENERAL_H0, DescriptorBuffers, TableDescriptor, has_operator_basis
from .tables import SharedTables, get_workers, host_tables, is_hermitian_h0, table_batch_cap, table_shapes
from .types import FidelityRobustGRAPEProblem, split_x


class GrapePlan:
    """One device plan for one problem (grape_plan_create / grape_plan_destroy)."""

    def __init__(self, fp: FidelityRobustGRAPEProblem, nparam: int, device: int = 0, max_batch: int = 256,
                 options: int = 0, scan_waves: int = 0):
        """options: GRAPE_OPT_* flags (operators.OPT_*), scan_waves: k_scan width override --
        plan-creation choices between implementations of the same outputs (include/grape.h)."""
        L = _capi.lib()
        self.fp = fp
        self.up = fp.unitary_problem
        self.nparam = int(nparam)
        self.device = int(device)
        self.nx = self.nparam * self.up.ntimes + self.up.nb_additional_param
        self.nerr = len(self.up.error_sources)
        self.max_batch = int(max_batch)
        self.requested_batch = self.max_batch  # before the closure-table byte cap (get_plan's key)
        self.options = int(options)
        self.lock = threading.Lock()  # one evaluation at a time (the plan's buffers are shared)
        self._shared = None  # closure fallback: double-buffered shared-memory tables
        # operator bases -> the fused device path; plain closures -> the host-table fallback
        self.tables = not has_operator_basis(fp)
        if self.tables:
            # closure tables (device d_Htab and the two shared-memory buffers) hold nv d x d
            # matrices per step per evaluation: bound the evaluations per pass by bytes
            self.max_batch = max(1, min(self.max_batch, table_batch_cap(fp, self.nparam)))
            self._bufs = TableDescriptor(fp, self.nparam, self.max_batch, options, scan_waves)
        else:
            self._bufs = DescriptorBuffers(fp, self.nparam, self.max_batch, options, scan_waves)
        h = ctypes.c_void_p()
        _capi.check(L.grape_plan_create(ctypes.byref(self._bufs.desc), self.device, ctypes.byref(h)))
        self.handle = h
        self._stream_ptr = None

    def general_h0_for(self, H0s, Hall=None):
        """Closure plans: the host sees H0 only as tables; a non-Hermitian nominal H0 (e.g. a
        -i Gamma/2 decay term) recreates the plan on the general-H0 path (GRAPE_OPT_GENERAL_H0,
        the reference's LU-inverted chain, UnitaryCalculations.jl:47) before the device call.
        Above 12 levels every tabulated generator Hall (default H0s) goes through the dense
        engine's interchange-free solve, which needs it Hermitian: anything else is refused.
        H0s / Hall: matrices (any leading shape, either storage order)."""
        if not self.tables:
            return
        if self.up.ndim > 12:
            if not is_hermitian_h0(H0s if Hall is None else Hall):
                raise ValueError("closure problems above 12 levels need Hermitian H0 / H0 + Herror tables "
                                 "(the dense engine's exponential); non-Hermitian generators are served up to 12 levels")
            return
        if (self.options & OPT_GENERAL_H0) or is_hermitian_h0(H0s):
            return
        self.options |= OPT_GENERAL_H0
        self._bufs.desc.reserved[1] = self.options
        h = ctypes.c_void_p()
        _capi.check(_capi.lib().grape_plan_create(ctypes.byref(self._bufs.desc), self.device, ctypes.byref(h)))
        _capi.lib().grape_plan_destroy(self.handle)
        self.handle = h
        if self._stream_ptr:
            self.set_stream(self._stream_ptr)

    def close(self):
        if getattr(self, "handle", None) is not None and self.handle.value:
            _capi.lib().grape_plan_destroy(self.handle)
            self.handle = None
        for tabs in getattr(self, "_shared", None) or ():
            try:
                self._workers.release(tabs)
            except Exception:
                pass
            tabs.close()
        self._shared = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self) -> int:
        return _capi.lib().grape_plan_stream(self.handle)

    def set_stream(self, stream_ptr: int | None):
        """Enqueue on the caller's hipStream_t (e.g. a torch.cuda.Stream's cuda_stream);
        None / 0 selects the plan's own stream -- so torch's default (null) stream cannot be
        joined this way: use a side stream and wait_stream (optimize.RobustCost does)."""
        _capi.check(_capi.lib().grape_plan_set_stream(self.handle, ctypes.c_void_p(stream_ptr or None)))
        self._stream_ptr = stream_ptr

    def fidelity_grad(self, X):
        """Host arrays in/out. X: (nbatch, n_x). Returns F (nb,), F_dx (nb, n_x),
        F_d2err (nb, nerr), F_d2err_dx (nb, n_x, nerr)."""
        X = np.ascontiguousarray(X, dtype=np.float64)
        if X.ndim != 2 or X.shape[1] != self.nx:
            raise AssertionError("Control parameter size must be a multiple of time steps")
        nb = X.shape[0]
        F = np.empty(nb)
        Fdx = np.empty((nb, self.nx))
        Fd2 = np.empty((nb, self.nerr)) if self.nerr else None
        Fd2dx = np.empty((nb, self.nerr, self.nx)) if self.nerr else None
        if self.tables:  # closures evaluated here, everything else on the device
            self._fidelity_grad_tables(X, F, Fdx, Fd2, Fd2dx)
        else:
            _capi.check(_capi.lib().grape_fidelity_grad(self.handle, nb, _capi.dptr(X), _capi.dptr(F),
                                                         _capi.dptr(Fdx), _capi.dptr(Fd2), _capi.dptr(Fd2dx)))
        if not self.nerr:
            Fd2 = np.zeros((nb, 0))
            Fd2dx = np.zeros((nb, self.nx, 0))
        else:
            Fd2dx = Fd2dx.transpose(0, 2, 1)
        return F, Fdx, Fd2, Fd2dx

    def _fidelity_grad_tables(self, X, F, Fdx, Fd2, Fd2dx):
        """Closure fallback: the closure tables are built by the worker pool (tables.py) into
        shared memory, chunk by chunk of max_batch evaluations, double-buffered: the workers
        fill chunk j + 1 while the device evaluates chunk j."""
        L = _capi.lib()
        nb = X.shape[0]
        C = self.max_batch
        chunks = [(b0, min(C, nb - b0)) for b0 in range(0, nb, C)]
        sl = lambda a, b0, n: None if a is None else a[b0:b0 + n]
        W = get_workers(self.fp)
        shipped = W.prepare(self.fp) if W is not None else None  # the closures' current state
        if shipped is not None and self._shared is None:
            sh, su = table_shapes(self.fp, C, self.nparam)
            try:
                self._shared = [SharedTables(sh, su)]
                self._shared.append(SharedTables(sh, su))
                self._workers = W
            except MemoryError:  # /dev/shm too small for two chunks: evaluate the closures here
                for t in self._shared or ():
                    t.close()
                self._shared = None
        if shipped is None or self._shared is None:  # serial, chunk by chunk
            for b0, n in chunks:
                H, U0 = host_tables(self.fp, X[b0:b0 + n], self.nparam)
                self.general_h0_for(H[:, :, 0], H)
                _capi.check(L.grape_fidelity_grad_tables(
                    self.handle, n, _capi.dptr(X[b0:b0 + n]), _capi.dptr(H), _capi.dptr(U0),
                    _capi.dptr(F[b0:b0 + n]), _capi.dptr(Fdx[b0:b0 + n]), _capi.dptr(sl(Fd2, b0, n)),
                    _capi.dptr(sl(Fd2dx, b0, n))))
            return
        pending = {}
        try:
            pending[0] = W.submit(shipped, self.nparam, self._shared[0], X, range(chunks[0][0], sum(chunks[0])))
            for j, (b0, n) in enumerate(chunks):
                if j + 1 < len(chunks):  # the other buffer's chunk (j - 1) is done on the device
                    c0, cn = chunks[j + 1]
                    pending[j + 1] = W.submit(shipped, self.nparam, self._shared[(j + 1) % 2], X,
                                              range(c0, c0 + cn))
                for r in pending[j]:
                    r.get()
                del pending[j]  # kept until every task of the chunk is done: drained below on error
                tabs = self._shared[j % 2]
                self.general_h0_for(tabs.H[:n, :, 0], tabs.H[:n])
                _capi.check(L.grape_fidelity_grad_tables(
                    self.handle, n, _capi.dptr(X[b0:b0 + n]), _capi.dptr(tabs.H), _capi.dptr(tabs.U0),
                    _capi.dptr(F[b0:b0 + n]), _capi.dptr(Fdx[b0:b0 + n]), _capi.dptr(sl(Fd2, b0, n)),
                    _capi.dptr(sl(Fd2dx, b0, n))))
        except BaseException:
            # a worker or the device call failed: every task still writing into the two shared
            # buffers must finish before the next call may refill them
            for rs in pending.values():
                for r in rs:
                    try:
                        r.wait()
                    except BaseException:
                        pass
            raise

    def fidelity_grad_device_async(self, x_ptr: int, F_ptr: int, Fdx_ptr: int, nbatch: int,
                                   Fd2_ptr: int = 0, Fd2dx_ptr: int = 0):
        """Device pointers (e.g. torch CUDA tensors' data_ptr()), enqueued on the plan stream."""
        _capi.check(_capi.lib().grape_fidelity_grad_device_async(
            self.handle, int(nbatch), ctypes.c_void_p(x_ptr), ctypes.c_void_p(F_ptr),
            ctypes.c_void_p(Fdx_ptr), ctypes.c_void_p(Fd2_ptr or None), ctypes.c_void_p(Fd2dx_ptr or None)))

    def unitary_derivs(self, x):
        """grape_unitary_derivs: the 6-tuple of src/UnitaryCalculations.jl:154 for ONE x, as
        complex arrays in the reference's shapes (column-major, like Julia)."""
        up = self.up
        x = np.ascontiguousarray(x, dtype=np.float64)
        if x.ndim != 1 or x.shape[0] != self.nx:
            raise AssertionError("Control parameter size must be a multiple of time steps")
        d, nt, npar, na, ne = up.ndim, up.ntimes, self.nparam, up.nb_additional_param, self.nerr
        shapes = [(d, d), (d, d, npar, nt), (d, d, na), (d, d, ne), (d, d, npar, nt, ne), (d, d, na, ne)]
        outs = [np.zeros(sh, dtype=np.complex128, order="F") for sh in shapes]
        ptr = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)) if a.size else None
        if self.tables:  # closure problem: every closure call site evaluated here
            H, _ = host_tables(self.fp, x[None, :], self.nparam)
            self.general_h0_for(H[:, :, 0], H)
            _capi.check(_capi.lib().grape_unitary_derivs_tables(self.handle, _capi.dptr(x), _capi.dptr(H),
                                                                *[ptr(a) for a in outs]))
        else:
            _capi.check(_capi.lib().grape_unitary_derivs(self.handle, _capi.dptr(x), *[ptr(a) for a in outs]))
        return tuple(outs)

    def set_profiling(self, enable: bool):
        _capi.check(_capi.lib().grape_plan_set_profiling(self.handle, int(bool(enable))))

    def kernel_times(self, reset: bool = False):
        """{kernel name: (total ms, launches)} accumulated while profiling was on."""
        nk = len(_capi.KERNEL_NAMES)
        ms = (ctypes.c_double * nk)()
        n = (ctypes.c_longlong * nk)()
        _capi.check(_capi.lib().grape_plan_kernel_times(self.handle, ms, n, int(reset)))
        return {name: (ms[k], n[k]) for k, name in enumerate(_capi.KERNEL_NAMES)}

    def synchronize(self):
        _capi.check(_capi.lib().grape_plan_synchronize(self.handle))

    def sectors(self) -> tuple:
        """((sector size, sectors per evaluation), ...) per sector class of the fidelity path;
        ((ndim, 1),) = whole matrices (include/grape.h grape_plan_sectors)."""
        S, n = (ctypes.c_int * 2)(), (ctypes.c_int * 2)()
        k = _capi.lib().grape_plan_sectors(self.handle, S, n, 2)
        _capi.check(min(k, 0))
        return tuple((S[c], n[c]) for c in range(k))

    def sector_info(self) -> dict:
        """{"twin": (per class: its two sectors share one exponential per step), "symmetric":
        the sectors are the symmetry-adapted ones} (include/grape.h grape_plan_sector_info)."""
        t, sym = (ctypes.c_int * 2)(), ctypes.c_int(0)
        k = _capi.lib().grape_plan_sector_info(self.handle, t, ctypes.byref(sym), 2)
        _capi.check(min(k, 0))
        g = (ctypes.c_int * 2)()
        kg = _capi.lib().grape_plan_gauge_info(self.handle, g, 2)
        _capi.check(min(kg, 0))
        e1 = _capi.lib().grape_plan_eval1(self.handle)
        _capi.check(min(e1, 0))
        return {"twin": tuple(bool(t[c]) for c in range(k)), "symmetric": bool(sym.value),
                "gauge": tuple(bool(g[c]) for c in range(kg)), "ladder": tuple(g[c] == 2 for c in range(kg)),
                "eval1": bool(e1)}


# Plan cache of the reference-shaped entry points (one plan per problem object, nparam and
# device).  A plan owns HBM workspace for `max_batch` evaluations; larger batches are
# chunked by the C side, so one plan serves every batch size: it is recreated larger only
# up to PLAN_BATCH_CAP.  At most MAX_CACHED_PLANS plans live at once (least recently used
# evicted and destroyed).  Evaluations on one plan are serialised by its lock, so cached
# plans may be shared by threads (locked_plan: fetch and lock in one step).
PLAN_BATCH_CAP = 256
MAX_CACHED_PLANS = 8
_cache_lock = threading.Lock()
_plan_cache: "OrderedDict" = OrderedDict()


def get_plan(fp: FidelityRobustGRAPEProblem, nparam: int, device: int = 0, max_batch: int = 1) -> GrapePlan:
    """The cached plan of (problem object, nparam, device) holding at least
    min(max_batch, PLAN_BATCH_CAP) evaluations of workspace."""
    want = max(1, min(int(max_batch), PLAN_BATCH_CAP))
    key = (id(fp), int(nparam), int(device))
    with _cache_lock:
        ent = _plan_cache.get(key)
        if ent is not None and ent.fp is fp and ent.requested_batch >= want:
            _plan_cache.move_to_end(key)
            return ent
        if ent is not None:
            del _plan_cache[key]
            with ent.lock:
                ent.close()
            if ent.fp is fp:
                want = max(want, ent.requested_batch)
        plan = GrapePlan(fp, nparam, device, want)
        _plan_cache[key] = plan
        while len(_plan_cache) > MAX_CACHED_PLANS:
            _, old = _plan_cache.popitem(last=False)
            with old.lock:
                old.close()
        return plan


@contextlib.contextmanager
def locked_plan(fp: FidelityRobustGRAPEProblem, nparam: int, device: int = 0, max_batch: int = 1):
    """get_plan, with the plan's lock held for the block: a plan another thread evicted or
    regrew between get_plan and the lock (it is closed then) is fetched again."""
    while True:
        plan = get_plan(fp, nparam, device, max_batch)
        with plan.lock:
            if plan.handle is not None:
                yield plan
                return


def cached_plan_count() -> int:
    with _cache_lock:
        return len(_plan_cache)


def clear_plans():
    with _cache_lock:
        for p in _plan_cache.values():
            with p.lock:
                p.close()
        _plan_cache.clear()
        _wrapped.clear()
    from .timeshard import clear_slice_plans
    clear_slice_plans()


# UnitaryRobustGRAPEProblem -> a FidelityRobustGRAPEProblem around it (the descriptor needs
# a projector and a target; neither enters the unitary-level outputs).  Small LRU.
_wrapped: "OrderedDict" = OrderedDict()


def fidelity_wrapper(unitary_problem) -> FidelityRobustGRAPEProblem:
    from .operators import OperatorBasisTarget, Term, has_operator_basis_h
    key = id(unitary_problem)
    with _cache_lock:
        fp = _wrapped.get(key)
        if fp is not None and fp.unitary_problem is unitary_problem:
            _wrapped.move_to_end(key)
            return fp
        eye = np.eye(unitary_problem.ndim, dtype=np.complex128)
        target = OperatorBasisTarget([Term(eye)]) if has_operator_basis_h(unitary_problem) else (lambda xa: eye)
        fp = FidelityRobustGRAPEProblem(unitary_problem, np.eye(unitary_problem.ndim), target)
        _wrapped[key] = fp
        while len(_wrapped) > MAX_CACHED_PLANS:
            _wrapped.popitem(last=False)
        return fp


def calculate_fidelity_and_derivatives(fidelity_problem: FidelityRobustGRAPEProblem, x, device: int = 0):
    """GPU restatement of src/FidelityCalculations.jl:19-119.

    Returns (F, F_dx_tot, F_d2err, F_d2err_dx_tot) with the reference's shapes:
    F scalar, F_dx_tot (n_x,), F_d2err (nerr,), F_d2err_dx_tot (n_x, nerr).
    A 2-D x of shape (nbatch, n_x) returns the same quantities with a leading
    batch axis.
    """
    x = np.asarray(x, dtype=np.float64)
    batched = x.ndim == 2
    X = x if batched else x[None, :]
    _, _, nparam = split_x(fidelity_problem.unitary_problem, X[0])
    with locked_plan(fidelity_problem, nparam, device, max_batch=X.shape[0]) as plan:
        F, Fdx, Fd2, Fd2dx = plan.fidelity_grad(X)
    if batched:
        return F, Fdx, Fd2, Fd2dx
    return float(F[0]), Fdx[0], Fd2[0], Fd2dx[0]


def calculate_unitary_and_derivatives(unitary_problem, x, device: int = 0):
    """GPU restatement of src/UnitaryCalculations.jl:20-155 (through grape_unitary_derivs).

    Returns (U, U_dx, U_dx_add, U_derr, U_derr_dx, U_derr_dx_add) with the reference's shapes
    (d,d), (d,d,np,N_t), (d,d,na), (d,d,ne), (d,d,np,N_t,ne), (d,d,na,ne)."""
    x = np.asarray(x, dtype=np.float64)
    _, _, nparam = split_x(unitary_problem, x)
    with locked_plan(fidelity_wrapper(unitary_problem), nparam, device, max_batch=1) as plan:
        return plan.unitary_derivs(x)
