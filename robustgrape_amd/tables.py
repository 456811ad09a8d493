"""Closure fallback, host side: the reference's closure calls tabulated for the device.

A problem whose ``H0`` / ``Herror`` / ``target_unitary`` are plain callables (the
reference's idiom, src/Types.jl:10,25,50) cannot be evaluated on the GPU.  The host
calls them at exactly the reference's call sites (src/UnitaryCalculations.jl:45-95,
src/FidelityCalculations.jl:32-38) and hands the tables to
``grape_fidelity_grad_tables``; everything else runs on the device.

The closure calls are the reference's own cost (one Python call per call site), so
this module spreads them over worker processes: ``TableWorkers`` spawns a pool once
(the workers never touch the GPU), ships them the problem by value with every call, splits a batch by
evaluations -- or a single evaluation by time steps -- and the workers write straight
into shared-memory tables that the device call then copies to HBM.  While the device
evaluates one chunk of a batch, the workers fill the next (``GrapePlan.fidelity_grad``).

Worker count: ``GRAPE_TABLE_WORKERS`` (0 or 1 = serial in the calling process; default
min(8, cpu_count)).
"""
from __future__ import annotations

import atexit
import contextlib
import multiprocessing as mp
import multiprocessing.pool
import os
import sys
import threading
import time
from multiprocessing import shared_memory

import numpy as np

from .types import split_x


def table_variants(nparam: int, nadd: int, nerr: int) -> int:
    """Variants per step of the grape_fidelity_grad_tables H table (include/grape.h):
    n = nparam + nadd gradient parameters; 1 + n without error sources, else
    1 + 2n + nerr (2 + n)."""
    n = nparam + nadd
    return 1 + n if nerr == 0 else 1 + 2 * n + nerr * (2 + n)


def fill_tables(fp, X, nparam: int, H, U0, rows, k0: int, k1: int, target: bool = True):
    """Fill H[r, k0:k1] (and U0[r] when `target`) for the evaluations r in `rows` with the
    closure values of X[r], column-major matrices (the C-order image of M^T), in the
    variant order of include/grape.h:
      0: H0(nt, x[:,nt], x_add) (:45) | 1 + u: parameter u + eps (:48-51, :57-59) |
      ne > 0: 1 + n + u: parameter u + eps2 (:53-54, :61-62) | per error e, base 1 + 2n + e(2 + n):
      base: Herror_e(.., eps) + H0 (:67) | base + 1: Herror_e(.., eps2) + H0 (:71) |
      base + 2 + u: Herror_e(u + eps2, .., eps2) + H0(u + eps2) (:77-78, :89-90)
    with u < nparam a control x[u, nt] and u >= nparam the additional parameter
    x_add[u - nparam]; U0: target(x_add), target(x_add + eps e_q) (FidelityCalculations.jl:32-38).
    Every call gets fresh argument arrays, as Julia's slicing does."""
    up = fp.unitary_problem
    na = up.nb_additional_param
    eps, eps2 = float(up.eps), float(up.eps2)
    errs = up.error_sources
    ne = len(errs)
    n = nparam + na
    H0f, tgt = up.H0, fp.target_unitary
    asc = np.asarray
    for b in rows:
        x_main, x_add, _ = split_x(up, X[b])
        for k in range(k0, k1):
            nt1 = k + 1
            xk = x_main[:, k]
            Hb = H[b, k]

            def at(u, delta):  # (x_k, x_add) with gradient parameter u moved by delta
                xp, xa = xk.copy(), x_add.copy()
                if u < nparam:
                    xp[u] = xk[u] + delta
                else:
                    xa[u - nparam] = x_add[u - nparam] + delta
                return xp, xa

            H0k = asc(H0f(nt1, xk.copy(), x_add.copy()), np.complex128)
            Hb[0] = H0k.T
            for u in range(n):
                Hb[1 + u] = asc(H0f(nt1, *at(u, eps))).T
            if ne == 0:
                continue
            Hx2 = []
            for u in range(n):  # H0 at u + eps2 also feeds the mixed stencils below (same call)
                h = asc(H0f(nt1, *at(u, eps2)), np.complex128)
                Hx2.append(h)
                Hb[1 + n + u] = h.T
            for e, es in enumerate(errs):
                base = 1 + 2 * n + e * (2 + n)
                Hb[base] = (asc(es.Herror(nt1, xk.copy(), x_add.copy(), eps), np.complex128) + H0k).T
                Hb[base + 1] = (asc(es.Herror(nt1, xk.copy(), x_add.copy(), eps2), np.complex128) + H0k).T
                for u in range(n):
                    Hb[base + 2 + u] = (asc(es.Herror(nt1, *at(u, eps2), eps2), np.complex128) + Hx2[u]).T
        if target:
            U0[b, 0] = asc(tgt(x_add.copy())).T
            for q in range(na):
                xa = x_add.copy()
                xa[q] += eps
                U0[b, 1 + q] = asc(tgt(xa)).T


def is_hermitian_h0(H0s, rtol=1e-12) -> bool:
    """Whether the tabulated nominal H0(nt, x, x_add) matrices are Hermitian.  The fused device
    path chains the nominal propagators with C_k^-1 = C_k^dagger; a non-Hermitian H0 -- e.g. a
    -i Gamma/2 decay term -- moves the plan to the general-H0 path (GRAPE_OPT_GENERAL_H0: the LU
    inverse of UnitaryCalculations.jl:47).  Error generators need no such property: their
    propagators only enter through differences the nominal chain transports."""
    H0s = np.asarray(H0s)
    if H0s.size == 0:
        return True
    dev = np.max(np.abs(H0s - np.conj(np.swapaxes(H0s, -1, -2))))
    return bool(dev <= rtol * max(np.max(np.abs(H0s)), 1e-300))


def table_shapes(fp, nb: int, nparam: int):
    up = fp.unitary_problem
    d, na = up.ndim, up.nb_additional_param
    nv = table_variants(nparam, na, len(up.error_sources))
    return (nb, up.ntimes, nv, d, d), (nb, 1 + na, d, d)


TABLE_CHUNK_BYTES = 256 << 20  # per table buffer (GRAPE_TABLE_CHUNK_MB overrides)


def table_batch_cap(fp, nparam: int) -> int:
    """Evaluations per closure-table chunk: one chunk's H + U0 tables within TABLE_CHUNK_BYTES
    (the plan holds one chunk on the device and two in /dev/shm; e.g. d = 9, N_t = 100 with
    4 error sources is ~2.7 MB per evaluation -> 94 evaluations)."""
    sh, su = table_shapes(fp, 1, nparam)
    per = (int(np.prod(sh)) + int(np.prod(su))) * 16
    env = os.environ.get("GRAPE_TABLE_CHUNK_MB")
    budget = int(float(env) * (1 << 20)) if env else TABLE_CHUNK_BYTES
    return max(1, budget // per)


def host_tables(fp, X, nparam: int):
    """The closure tables of a batch, serially in this process: H (nb, N_t, nv, d, d) and
    U0 (nb, 1 + na, d, d), column-major matrices (see fill_tables)."""
    X = np.asarray(X, np.float64)
    sh, su = table_shapes(fp, X.shape[0], nparam)
    H, U0 = np.empty(sh, np.complex128), np.empty(su, np.complex128)
    fill_tables(fp, X, nparam, H, U0, range(X.shape[0]), 0, fp.unitary_problem.ntimes)
    return H, U0


# ---------------------------------------------------------------------------
# worker pool
# ---------------------------------------------------------------------------
# Workers receive the problem by value (cloudpickle) with every call and cache it under the
# digest of those bytes: a closure whose captured state changed between calls pickles to new
# bytes, so a worker can never evaluate a stale copy (the serial path and the reference call the
# live closure).  Functions of importable modules travel by reference, as pickle does: a worker
# sees such a module as imported, so closures that read MUTABLE module globals must run serially
# (GRAPE_TABLE_WORKERS=0).
_problems = {}   # worker side: digest -> problem (small LRU)
_shm_cache = {}  # worker side: attachments
_KEEP_PROBLEMS = 8


def _attach(name):
    shm = _shm_cache.get(name)
    if shm is None:
        # attaching registers the name with the resource tracker the spawned workers share with
        # the creating process (a set: no second entry); the creator's unlink unregisters it
        shm = shared_memory.SharedMemory(name=name)
        _shm_cache[name] = shm
    return shm


def _worker_fill(task):
    token, blob, nparam, hname, uname, sh, su, X, rows, k0, k1, target = task
    fp = _problems.pop(token, None)
    if fp is None:
        import cloudpickle
        fp = cloudpickle.loads(blob)
    _problems[token] = fp  # most recent last
    while len(_problems) > _KEEP_PROBLEMS:
        _problems.pop(next(iter(_problems)))
    # keep the most recently named attachments only (a plan's two double buffers, a few plans):
    # a closed or regrown plan's segments are unmapped here, so their tmpfs pages can be freed
    for n in (hname, uname):
        if n in _shm_cache:
            _shm_cache[n] = _shm_cache.pop(n)  # most recent last
    while len(_shm_cache) > 4 * _KEEP_PROBLEMS:
        _shm_cache.pop(next(iter(_shm_cache))).close()
    H = np.ndarray(sh, np.complex128, buffer=_attach(hname).buf)
    U0 = np.ndarray(su, np.complex128, buffer=_attach(uname).buf)
    t = time.perf_counter()
    fill_tables(fp, X, nparam, H, U0, rows, k0, k1, target)
    return time.perf_counter() - t


def _worker_release(names):
    for n in names:
        shm = _shm_cache.pop(n, None)
        if shm is not None:
            shm.close()
    return 0


class SharedTables:
    """H / U0 tables in POSIX shared memory (readable by the device copy, writable by workers)."""

    def __init__(self, sh, su):
        nbytes = lambda s: int(np.prod(s)) * 16
        need = nbytes(sh) + nbytes(su)
        free = shm_free_bytes()  # tmpfs accepts an oversized ftruncate and SIGBUSes the writer later
        if free is not None and need > free:
            raise MemoryError(f"closure tables need {need / 2**20:.1f} MiB of /dev/shm, {free / 2**20:.1f} MiB free")
        self.shm_h = shared_memory.SharedMemory(create=True, size=max(16, nbytes(sh)))
        self.shm_u = shared_memory.SharedMemory(create=True, size=max(16, nbytes(su)))
        self.sh, self.su = sh, su
        self.H = np.ndarray(sh, np.complex128, buffer=self.shm_h.buf)
        self.U0 = np.ndarray(su, np.complex128, buffer=self.shm_u.buf)

    def close(self):
        self.H = self.U0 = None
        for s in (self.shm_h, self.shm_u):
            s.close()
            s.unlink()


def shm_free_bytes():
    try:
        st = os.statvfs("/dev/shm")
        return st.f_bavail * st.f_frsize
    except OSError:
        return None


@contextlib.contextmanager
def _main_hidden():
    """Hide the parent's __main__ from spawned children while a pool starts.  A spawned child
    re-imports the parent's main script (multiprocessing.spawn get_preparation_data: __spec__.name
    or __file__) and runs its top-level code; a user script without an
    `if __name__ == "__main__"` guard (the reference's example style) would then build GRAPE
    plans -- initialising HIP in a worker -- and start a nested pool in every worker.  The workers
    need only this module and the problem, which cloudpickle ships by value (__main__ closures
    included), so they start without the main module."""
    main = sys.modules.get("__main__")
    if main is None:
        yield
        return
    saved = {k: main.__dict__[k] for k in ("__file__", "__spec__") if k in main.__dict__}
    main.__dict__.pop("__file__", None)
    main.__dict__["__spec__"] = None
    try:
        yield
    finally:
        main.__dict__.pop("__spec__", None)
        main.__dict__.update(saved)


_SPAWN = mp.get_context("spawn")


class _NoMainProcess(_SPAWN.Process):
    """A spawned worker started with the parent's __main__ hidden (_main_hidden) -- every start,
    including the replacements Pool._repopulate_pool makes when a worker dies.  The
    hiding is a short process-wide change around the start; a thread of the parent that reads
    __main__.__file__ at that instant would see it unset."""

    def start(self):
        with _main_hidden():
            super().start()


class _NoMainContext(type(_SPAWN)):
    Process = _NoMainProcess


class TableWorkers:
    """A process pool that fills closure tables in shared memory.  Spawned, not forked: the pool
    may first be needed after this process has initialised HIP, and a fork would copy that
    state into the workers (they never touch the GPU).  The workers start without the parent's
    main module (_NoMainProcess: also the pool's replacement workers)."""

    def __init__(self, nworkers: int):
        self.n = nworkers
        self.pool = multiprocessing.pool.Pool(nworkers, context=_NoMainContext())
        self.lock = threading.Lock()

    @staticmethod
    def prepare(fp):
        """(token, bytes) of the problem as the workers will evaluate it, or None when cloudpickle
        cannot serialise its closures (then the caller evaluates them serially).  Called once per
        evaluation call, so the workers always see the closures' current state."""
        try:
            import cloudpickle
            import hashlib
            blob = cloudpickle.dumps(fp)
        except Exception:
            return None
        return hashlib.blake2b(blob, digest_size=16).hexdigest(), blob

    def submit(self, shipped, nparam, tabs: SharedTables, X, rows_of_chunk):
        """Asynchronously fill the tables for the evaluations `rows_of_chunk` (indices into X and
        into the tables' first axis) of the problem `shipped` (from prepare); returns an
        AsyncResult list."""
        token, blob = shipped
        nt = tabs.sh[1]
        X = np.asarray(X, np.float64)
        nb = len(rows_of_chunk)
        tasks = []
        if nb >= self.n:  # split by evaluations
            for part in np.array_split(np.arange(nb), self.n):
                if len(part):
                    tasks.append((part, 0, nt, True))
        else:  # few evaluations: split each by time steps
            per = max(1, -(-self.n // max(1, nb)))
            for r in range(nb):
                bounds = np.linspace(0, nt, min(per, nt) + 1).astype(int)
                for j in range(len(bounds) - 1):
                    tasks.append((np.array([r]), int(bounds[j]), int(bounds[j + 1]), j == 0))
        sub = X[np.asarray(rows_of_chunk)]
        return [self.pool.apply_async(_worker_fill, ((token, blob, nparam, tabs.shm_h.name, tabs.shm_u.name,
                                                      tabs.sh, tabs.su, sub, rows, k0, k1, tg),))
                for rows, k0, k1, tg in tasks]

    def release(self, tabs: SharedTables):
        """Best effort: workers that run one of these calls drop their mappings now; the others
        drop them at their next fill (_worker_fill keeps only recently named segments)."""
        names = [tabs.shm_h.name, tabs.shm_u.name]
        rs = [self.pool.apply_async(_worker_release, (names,)) for _ in range(self.n)]
        for r in rs:
            try:
                r.get(timeout=10)
            except Exception:
                pass

    def close(self):
        self.pool.terminate()
        self.pool.join()


_workers = None
_workers_lock = threading.Lock()


def default_workers() -> int:
    env = os.environ.get("GRAPE_TABLE_WORKERS")
    if env is not None:
        return max(0, int(env))
    return min(8, os.cpu_count() or 1)


def get_workers(fp=None):
    """The process-wide pool (None when the fallback runs serially)."""
    global _workers
    n = default_workers()
    if n <= 1:
        return None
    with _workers_lock:
        if _workers is None:
            try:
                _workers = TableWorkers(n)
            except Exception as e:  # no pool (e.g. a process limit): the tables fill serially
                import warnings
                warnings.warn(f"closure-table worker pool unavailable ({e!r}); filling tables serially")
                return None
            atexit.register(_shutdown)
        return _workers


def _shutdown():
    global _workers
    if _workers is not None:
        _workers.close()
        _workers = None
