"""Time sharding of one evaluation (robustgrape_amd/timeshard.py) on CPU.

The device slice plans (grape_slice_forward / grape_slice_gradient) are replaced by a numpy
model of the same two calls (scipy's expm; the slice total, then Re tr(M' Q_k^dag dE Q_{k-1})
per step and control); what is under test is the slicing, the chaining of the slice totals,
the fidelity head, the M' = B M B^dag transform, the assembly of F_dx and the two all_gathers
(gloo, world_size 2 and 3) -- against the oracle's whole evaluation
(UnitaryCalculations.jl:20-155, FidelityCalculations.jl:19-119).  The device calls themselves are
checked in tests/test_gpu_timeshard.py."""
import os
import socket

import numpy as np
import pytest
import scipy.linalg as sla

from robustgrape_amd import timeshard as TS

T1 = 1e-12
T2, T2_ABS = 1e-6, 1e-7


def _problem(d=6, ntimes=12, dt=0.3):
    from robustgrape_amd.synthetic import dense_problem
    return dense_problem(d=d, ntimes=ntimes, dt=dt, rank=3)


class NumpySlice:
    """The two device calls of a slice plan, in numpy (test model)."""

    def __init__(self, fp, nparam, k0, k1, device=0):
        self.fp, self.nparam, self.k0, self.k1 = fp, nparam, k0, k1
        up = fp.unitary_problem
        self.dt, self.eps = up.t0 / up.ntimes, up.eps
        self.plan = self  # (the cache checks plan.handle)
        self.handle = 1

    def _E(self, k, xk):
        H = np.asarray(self.fp.unitary_problem.H0(k + 1, xk, np.zeros(0)), dtype=np.complex128)
        return sla.expm(-1j * self.dt * H)

    def forward(self, xs):
        self.xs = np.asarray(xs).reshape(self.k1 - self.k0, self.nparam)
        self.E = [self._E(self.k0 + j, self.xs[j]) for j in range(len(self.xs))]
        S = np.eye(self.E[0].shape[0], dtype=np.complex128)
        self.Q = []
        for E in self.E:
            S = E @ S
            self.Q.append(S)
        return S

    def gradient(self, Mp):
        d = self.E[0].shape[0]
        g = np.empty((len(self.E), self.nparam))
        for j, E in enumerate(self.E):
            Qm = self.Q[j - 1] if j else np.eye(d)
            for p in range(self.nparam):
                xp = self.xs[j].copy()
                xp[p] += self.eps
                dE = (self._E(self.k0 + j, xp) - E) / self.eps
                g[j, p] = np.trace(Mp @ self.Q[j].conj().T @ dE @ Qm).real
        return g.reshape(-1)

    def close(self):
        pass


@pytest.fixture
def numpy_slices(monkeypatch):
    monkeypatch.setattr(TS, "_slice_plan", lambda fp, nparam, k0, k1, device, keep=0: NumpySlice(fp, nparam, k0, k1))
    TS._plans.clear()


def _check(F, Fdx, F0, g0):
    assert abs(F - F0) <= T1, (F, F0)
    err, scale = float(np.max(np.abs(Fdx - g0))), float(np.max(np.abs(g0)))
    assert err <= T2 * scale + T2_ABS, (err, scale)


def test_slice_bounds_cover_every_step_once():
    for nt, ns in [(1024, 8), (13, 4), (5, 5), (7, 1)]:
        b = TS.slice_bounds(nt, ns)
        assert b[0][0] == 0 and b[-1][1] == nt and all(b[i][1] == b[i + 1][0] for i in range(ns - 1))
        assert max(y - x for x, y in b) - min(y - x for x, y in b) <= 1
    with pytest.raises(ValueError):
        TS.slice_bounds(4, 5)


def test_slice_problem_keeps_dt_and_refuses_x_add():
    fp = _problem()
    sp = TS.slice_problem(fp, 3, 7)
    up = sp.unitary_problem
    assert up.ntimes == 4 and abs(up.t0 / up.ntimes - 0.3) < 1e-15
    with pytest.raises(ValueError):
        TS.slice_problem(fp.replace(unitary_problem=fp.unitary_problem.replace(nb_additional_param=1)), 0, 4)


def test_fidelity_head_matches_oracle_fidelity():
    from oracle import grape_oracle as O
    fp = _problem()
    x = np.random.default_rng(3).uniform(-1, 1, size=24)
    U = O.calculate_unitary_and_derivatives(fp.unitary_problem, x)[0]
    F, _ = TS.fidelity_head(fp, np.asarray(U, dtype=np.complex128))
    F0 = O.calculate_fidelity_and_derivatives(fp, x)[0]
    assert abs(F - F0) <= T1


@pytest.mark.parametrize("nslices", [1, 2, 3, 5])
def test_virtual_slices_match_oracle(numpy_slices, nslices):
    from oracle import grape_oracle as O
    fp = _problem()
    x = np.random.default_rng(7).uniform(-1, 1, size=24)
    F, Fdx = TS.time_sharded_fidelity_grad(fp, x, nparam=2, nslices=nslices)
    F0, g0 = O.calculate_fidelity_and_derivatives(fp, x)[:2]
    _check(F, Fdx, F0, np.asarray(g0))


class CachedNumpySlice(NumpySlice):
    """NumpySlice as the plan cache sees a SlicePlan: `source`, `plan.handle`, close()."""

    def __init__(self, fp, nparam, k0, k1, device=0):
        super().__init__(fp, nparam, k0, k1, device)
        self.source = fp

    def forward(self, xs):
        assert self.handle is not None, "forward on a closed slice plan"
        return super().forward(xs)

    def close(self):
        self.handle = None


def test_slice_plan_cache_keeps_the_calls_plans_and_checks_the_problem(monkeypatch):
    """More slices than the LRU keeps (robustgrape_amd/timeshard.py _KEEP = 16) on one device: no
    plan of the call is closed before its forward; a cached entry whose problem is not the
    caller's (a recycled id) is rebuilt."""
    from oracle import grape_oracle as O
    monkeypatch.setattr(TS, "SlicePlan", CachedNumpySlice)
    TS._plans.clear()
    fp = _problem(ntimes=20)
    x = np.random.default_rng(11).uniform(-1, 1, size=40)
    F, Fdx = TS.time_sharded_fidelity_grad(fp, x, nparam=2, nslices=20)
    F0, g0 = O.calculate_fidelity_and_derivatives(fp, x)[:2]
    _check(F, Fdx, F0, np.asarray(g0))
    assert len(TS._plans) == 20
    # an entry under fp2's id built for another problem (what a recycled id would leave behind)
    fp2 = _problem(ntimes=20, dt=0.2)
    other = CachedNumpySlice(fp, 2, 0, 1)
    TS._plans[(id(fp2), 2, 0, 1, 0)] = other
    sp = TS._slice_plan(fp2, 2, 0, 1, 0)
    assert sp is not other and sp.source is fp2 and other.handle is None
    TS.clear_slice_plans()
    assert not TS._plans


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        TS._slice_plan = lambda fp, nparam, k0, k1, device, keep=0: NumpySlice(fp, nparam, k0, k1)
        fp = _problem()
        x = np.random.default_rng(7).uniform(-1, 1, size=24)
        F, Fdx = TS.time_sharded_fidelity_grad(fp, x, nparam=2)
        q.put((rank, F, Fdx.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_ranks_exchange_slices(world):
    """One slice per gloo rank, two all_gathers: every rank returns the oracle's F and F_dx."""
    import torch.multiprocessing as mp
    from oracle import grape_oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    fp = _problem()
    x = np.random.default_rng(7).uniform(-1, 1, size=24)
    F0, g0 = O.calculate_fidelity_and_derivatives(fp, x)[:2]
    for _, F, Fdx in out:
        _check(F, np.asarray(Fdx), F0, np.asarray(g0))
