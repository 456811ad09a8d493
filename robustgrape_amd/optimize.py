"""The optimiser around the hot path: src/FidelityCalculations.jl:161-218
(``optimize_fidelity_and_error_sources``), run as a BATCHED L-BFGS over
random restarts with every evaluation on the GPU.

Reference behaviour kept:
  * the cost and gradient of ``calculate_common!`` (:172-196):
      cost = 1 - F + sum_e c_e F_d2err_e^2 + sum_p (c1_p r1_p + c2_p r2_p)
      grad = -F_dx + 2 sum_e c_e F_d2err_e F_d2err_dx[:, e] + regulariser gradients
    (nparam > 1: each control's regulariser gradient lands on its own entries;
    the reference's ``sum(reg_costs_grad, dims=1)`` at :195 only has matching
    shapes for nparam == 1 and throws DimensionMismatch otherwise);
  * the shape assertions (:162-170) -> AssertionError;
  * Optim.jl's stopping rules for ``iterations``, ``time_limit`` and the
    ``additional_parameters`` g_tol (|g|_inf), f_abstol, f_reltol, x_abstol.
Optim.jl (the reference's solver, a third-party dependency absent here) is
replaced by an L-BFGS (memory 10, initial inverse-Hessian scaling s.y/y.y, as
Optim's LBFGS) with a strong-Wolfe line search (Nocedal & Wright alg. 3.5/3.6,
c1 = 1e-4, c2 = 0.9) in place of Optim's default Hager-Zhang: iterates are
not bit-identical to Optim's, the minimisation problem is.

MI355X design: all restarts of a sweep advance together.  Their control
vectors, gradients and L-BFGS histories live in HBM as (restarts, n_x)
tensors; each line-search round evaluates the still-active restarts in ONE
batched device pass (``GrapePlan.fidelity_grad_device_async``) and the
two-loop recursion is a handful of batched reductions.  Nothing leaves the
GPU inside the loop except the per-round active count.
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass, field
from typing import Callable, Optional

import numpy as np
import torch

from .types import FidelityRobustGRAPEParameters, FidelityRobustGRAPEProblem

C1, C2 = 1e-4, 0.9
MAX_LS_ROUNDS = 30
_ASYNC_ROWS_DEFAULT = True  # device optimiser: rows advance asynchronously unless a callback is given
MAX_PLAN_BATCH = 4096


@dataclass
class OptimizationResult:
    """What callers read from Optim's result (Optim.minimizer / minimum / iterations ...)."""
    minimizer: np.ndarray
    minimum: float
    iterations: int
    f_calls: int
    converged: bool
    g_converged: bool
    f_converged: bool
    x_converged: bool
    time_run: float
    stop_reason: str = ""
    trace: list = field(default_factory=list)  # Optim's store_trace: (iteration, value, g_norm, time)


@dataclass
class BatchResult:
    """Per-restart results of a batched run (rows follow the input order)."""
    minimizer: torch.Tensor          # (R, n)
    minimum: torch.Tensor            # (R,)
    gradient: torch.Tensor           # (R, n)
    iterations: torch.Tensor         # (R,) int64
    f_calls: torch.Tensor            # (R,) int64
    g_converged: torch.Tensor        # (R,) bool
    f_converged: torch.Tensor
    x_converged: torch.Tensor
    ls_failed: torch.Tensor
    time_run: float
    extra: dict = field(default_factory=dict)

    def result(self, r: int) -> OptimizationResult:
        conv = bool(self.g_converged[r] or self.f_converged[r] or self.x_converged[r])
        reason = "converged" if conv else ("line search failed" if bool(self.ls_failed[r]) else "iterations/time")
        return OptimizationResult(self.minimizer[r].detach().cpu().numpy(), float(self.minimum[r]),
                                  int(self.iterations[r]), int(self.f_calls[r]), conv,
                                  bool(self.g_converged[r]), bool(self.f_converged[r]),
                                  bool(self.x_converged[r]), self.time_run, reason,
                                  list(self.extra.get("trace", [])) if r == 0 else [])


def minimizer(res):
    """Optim.minimizer"""
    return res.minimizer


def minimum(res):
    """Optim.minimum"""
    return res.minimum


# ---------------------------------------------------------------------------
# batched L-BFGS with a strong-Wolfe line search (device agnostic)
# ---------------------------------------------------------------------------
def _rowdot(a, b):
    return torch.sum(a * b, dim=1)


def _cubic_min(a0, f0, g0, a1, f1, g1):
    """Minimiser of the cubic interpolating (a0, f0, g0), (a1, f1, g1), safeguarded into
    the middle 80 % of the interval; bisection where the cubic is not usable."""
    d1 = g0 + g1 - 3 * (f0 - f1) / (a0 - a1)
    disc = d1 * d1 - g0 * g1
    d2 = torch.sign(a1 - a0) * torch.sqrt(torch.clamp(disc, min=0.0))
    den = g1 - g0 + 2 * d2
    a = a1 - (a1 - a0) * (g1 + d2 - d1) / den
    lo = torch.minimum(a0, a1)
    hi = torch.maximum(a0, a1)
    w = hi - lo
    ok = (disc >= 0) & torch.isfinite(a) & (den != 0)
    a = torch.where(ok, a, 0.5 * (a0 + a1))
    return torch.clamp(a, lo + 0.1 * w, hi - 0.1 * w)


_TORCH_TWO_LOOP = bool(os.environ.get("GRAPE_TORCH_TWO_LOOP"))  # A/B switch for measurements


def _torch_direction(S, Y, rho, head, hist, gamma, g):
    """-H g for every row with batched torch ops (host tensors; the device path's checker)."""
    m, R, _ = S.shape
    all_rows = torch.arange(R, device=g.device)
    q = -g.clone()
    alpha = torch.zeros(m, R, dtype=g.dtype, device=g.device)
    for j in range(m):
        slot = (head - 1 - j) % m
        use = (j < hist)
        s_j = S[slot, all_rows]
        y_j = Y[slot, all_rows]
        r_j = rho[slot, all_rows]
        a_j = torch.where(use, r_j * _rowdot(s_j, q), torch.zeros_like(r_j))
        alpha[j] = a_j
        q = q - a_j[:, None] * y_j
    q = q * gamma[:, None]
    for j in reversed(range(m)):
        slot = (head - 1 - j) % m
        use = (j < hist)
        s_j = S[slot, all_rows]
        y_j = Y[slot, all_rows]
        r_j = rho[slot, all_rows]
        b_j = r_j * _rowdot(y_j, q)
        q = q + torch.where(use, alpha[j] - b_j, torch.zeros_like(b_j))[:, None] * s_j
    return q


def _device_direction(S, Y, rho, head, hist, gamma, g):
    """-H g for every row: grape_lbfgs_direction (csrc/grape_lbfgs.hip), enqueued on torch's
    current stream so it stays ordered with the surrounding torch ops."""
    import ctypes

    from . import _capi
    m, R, n = S.shape
    D = torch.empty_like(g)
    ptrs = [ctypes.c_void_p(t.data_ptr()) for t in (S, Y, rho, head, hist, gamma, g, D)]
    assert all(t.is_contiguous() for t in (S, Y, rho, head, hist, gamma, g))
    assert head.dtype == hist.dtype == torch.int64
    stream = ctypes.c_void_p(torch.cuda.current_stream(g.device).cuda_stream)
    _capi.check(_capi.lib().grape_lbfgs_direction(R, n, m, *ptrs, stream))
    return D


_TORCH_LS = bool(os.environ.get("GRAPE_TORCH_LS"))  # A/B switch: the torch line search on the GPU too


class _CLbfgsState:  # filled lazily (ctypes import only with a GPU run)
    cls = None

    @classmethod
    def get(cls):
        if cls.cls is None:
            import ctypes
            vp = ctypes.c_void_p
            fields = [("R", ctypes.c_int), ("n", ctypes.c_int), ("m", ctypes.c_int), ("reserved0", ctypes.c_int)]
            fields += [(nm, vp) for nm in _LS_F64 + _LS_I64 + _LS_I32]
            fields += [(nm, ctypes.c_double) for nm in ("f_abstol", "f_reltol", "x_abstol", "x_reltol")]
            fields += [("iterations", ctypes.c_int64), ("f_calls_limit", ctypes.c_int64)]
            cls.cls = type("grape_lbfgs_state", (ctypes.Structure,), {"_fields_": fields})
        return cls.cls


# include/grape.h grape_lbfgs_state, pointer fields in declaration order
_LS_F64 = ("X", "f", "g", "D", "Xn", "fn", "gn", "Xt", "f0", "dphi0", "a_cur", "a_prev", "f_prev", "dp_prev",
           "a_lo", "f_lo", "dp_lo", "a_hi", "f_hi", "dp_hi", "S", "Y", "rho", "gamma", "g_thr")
_LS_I64 = ("f_calls", "iters", "hist", "head", "rows")
_LS_I32 = ("phase", "first", "accepted", "gconv", "fconv", "xconv", "lsfail", "active", "count")


def _lbfgs_device(fun, X0, m, iterations, g_tol, f_abstol, f_reltol, x_abstol, time_limit, x_reltol, g_reltol,
                  f_calls_limit, callback, steepest=False, asynchronous=None) -> BatchResult:
    """lbfgs_batched on the GPU: the same algorithm with its per-round state machine, the descent
    check and the L-BFGS update as HIP kernels (csrc/grape_lbfgs.hip, include/grape.h
    grape_lbfgs_state), one host sync per line-search round (the count of searching rows).

    asynchronous (default when there is no callback): rows do not wait for each other at iteration
    boundaries -- every round evaluates every searching row whatever its iteration
    (grape_lbfgs_async_advance), so the few-row tail rounds of each iteration disappear; each row's
    trajectory is bitwise the synchronous one.  The callback (Optim's, per iteration of all rows)
    needs the synchronous loop."""
    import ctypes

    from . import _capi
    L = _capi.lib()
    t_start = time.perf_counter()
    X = X0.clone().contiguous()
    R, n = X.shape
    dev, dt = X.device, torch.float64
    t = {}
    t["X"] = X
    f, g = fun(X, torch.arange(R, device=dev))
    t["f"], t["g"] = f.to(dt).contiguous().clone(), g.to(dt).contiguous().clone()
    for nm in ("D", "Xn", "gn", "Xt"):
        t[nm] = torch.zeros(R, n, dtype=dt, device=dev)
    for nm in ("fn", "f0", "dphi0", "a_cur", "a_prev", "f_prev", "dp_prev", "a_lo", "f_lo", "dp_lo", "a_hi", "f_hi",
               "dp_hi"):
        t[nm] = torch.zeros(R, dtype=dt, device=dev)
    t["S"] = torch.zeros(m, R, n, dtype=dt, device=dev)
    t["Y"] = torch.zeros(m, R, n, dtype=dt, device=dev)
    t["rho"] = torch.zeros(m, R, dtype=dt, device=dev)
    t["gamma"] = torch.ones(R, dtype=dt, device=dev)
    gabs = torch.amax(torch.abs(t["g"]), dim=1)
    t["g_thr"] = torch.clamp(g_reltol * gabs, min=g_tol)
    for nm in _LS_I64:
        t[nm] = torch.zeros(R, dtype=torch.int64, device=dev)
    t["f_calls"] += 1
    for nm in _LS_I32:
        t[nm] = torch.zeros(max(R, 1), dtype=torch.int32, device=dev)
    t["gconv"] = (gabs <= t["g_thr"]).to(torch.int32)
    st = _CLbfgsState.get()()
    st.R, st.n, st.m = R, n, m
    for nm in _LS_F64 + _LS_I64 + _LS_I32:
        setattr(st, nm, t[nm].data_ptr())
    st.f_abstol, st.f_reltol, st.x_abstol, st.x_reltol = f_abstol, f_reltol, x_abstol, x_reltol
    st.iterations = int(min(iterations, 2 ** 62))
    st.f_calls_limit = int(f_calls_limit)
    sp = ctypes.byref(st)
    stream = lambda: ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)  # noqa: E731
    timed_out = False
    stopped = callback is not None and bool(callback(t["X"], t["f"], t["g"], t["iters"]))
    if asynchronous is None:
        asynchronous = _ASYNC_ROWS_DEFAULT and callback is None
    if asynchronous and not stopped:
        rounds = torch.zeros(max(R, 1), dtype=torch.int32, device=dev)
        t["phase"].fill_(3)  # no row has started its first iteration
        while True:
            if not math.isnan(time_limit) and time.perf_counter() - t_start > time_limit:
                timed_out = True  # (one more advance: rows whose search ended take their step)
                _capi.check(L.grape_lbfgs_async_advance(sp, int(bool(steepest)), MAX_LS_ROUNDS,
                                                        ctypes.c_void_p(rounds.data_ptr()), stream()))
                break
            _capi.check(L.grape_lbfgs_async_advance(sp, int(bool(steepest)), MAX_LS_ROUNDS,
                                                    ctypes.c_void_p(rounds.data_ptr()), stream()))
            _capi.check(L.grape_lbfgs_ls_begin(sp, stream()))
            cnt = int(t["count"][0].item())  # the round's one host sync
            if cnt == 0:
                break
            ft, gt = fun(t["Xt"][:cnt], t["rows"][:cnt])
            ft, gt = ft.to(dt).contiguous(), gt.to(dt).contiguous()
            _capi.check(L.grape_lbfgs_ls_end(sp, cnt, ctypes.c_void_p(ft.data_ptr()), ctypes.c_void_p(gt.data_ptr()),
                                             stream()))
        stopped = True
    while not stopped:
        if not math.isnan(time_limit) and time.perf_counter() - t_start > time_limit:
            timed_out = True
            break
        _capi.check(L.grape_lbfgs_direction(R, n, m, *[ctypes.c_void_p(t[k].data_ptr()) for k in
                                                          ("S", "Y", "rho", "head", "hist", "gamma", "g", "D")],
                                             stream()))
        _capi.check(L.grape_lbfgs_ls_init(sp, stream()))
        cnt = 0
        for rnd in range(MAX_LS_ROUNDS):
            _capi.check(L.grape_lbfgs_ls_begin(sp, stream()))
            cnt = int(t["count"][0].item())  # the round's one host sync
            if cnt == 0:
                break
            ft, gt = fun(t["Xt"][:cnt], t["rows"][:cnt])
            ft, gt = ft.to(dt).contiguous(), gt.to(dt).contiguous()
            _capi.check(L.grape_lbfgs_ls_end(sp, cnt, ctypes.c_void_p(ft.data_ptr()), ctypes.c_void_p(gt.data_ptr()),
                                             stream()))
        if rnd == 0 and cnt == 0:  # no row searches any more
            break
        _capi.check(L.grape_lbfgs_step(sp, stream()))
        if steepest:  # GradientDescent: drop the pair just stored (stream-ordered torch ops)
            t["hist"].zero_()
            t["gamma"].fill_(1.0)
        if callback is not None and bool(callback(t["X"], t["f"], t["g"], t["iters"])):
            break
    if hasattr(fun, "check"):  # deferred device status of the last evaluation (RobustCost)
        fun.check()
    b = lambda k: t[k][:R].bool()  # noqa: E731
    return BatchResult(t["X"], t["f"], t["g"], t["iters"], t["f_calls"], b("gconv"), b("fconv"), b("xconv"),
                       b("lsfail"), time.perf_counter() - t_start, {"timed_out": timed_out, "device_ls": True})


def lbfgs_batched(fun: Callable[[torch.Tensor, torch.Tensor], tuple], X0: torch.Tensor, *, m: int = 10,
                  iterations: int = 1000, g_tol: float = 1e-8, f_abstol: float = 0.0, f_reltol: float = 0.0,
                  x_abstol: float = 0.0, time_limit: float = float("nan"), x_reltol: float = 0.0,
                  g_reltol: float = 0.0, f_calls_limit: int = 0,
                  callback: Optional[Callable] = None, steepest: bool = False,
                  asynchronous: Optional[bool] = None) -> BatchResult:
    """Minimise fun row-wise from every row of X0.

    fun(X, rows) -> (f (r,), g (r, n)) evaluates the rows `rows` (int64 indices into the
    batch) at control vectors X (r, n).  Rows stop independently (Optim's rules: |g|_inf <=
    max(g_tol, g_reltol |g_0|_inf), |df| <= f_abstol or f_reltol |f|, |dx|_inf <= x_abstol or
    x_reltol |x|_inf, f_calls_limit (0: none)).  callback(X, f, g, iters) runs after the initial
    evaluation and after every iteration; a True return stops every row (Optim's callback).
    steepest: gradient descent (GradientDescent): the history is cleared after every step, so the
    two-loop recursion returns D = -g (gamma = 1) and the same line search runs along it.
    asynchronous (device path): rows advance without waiting for each other (default without a
    callback; same per-row trajectories, _lbfgs_device)."""
    if X0.is_cuda and not _TORCH_LS and not _TORCH_TWO_LOOP and X0.dtype == torch.float64 and m <= 64:
        return _lbfgs_device(fun, X0, m, iterations, g_tol, f_abstol, f_reltol, x_abstol, time_limit, x_reltol,
                             g_reltol, f_calls_limit, callback, steepest, asynchronous)
    t_start = time.perf_counter()
    X = X0.clone()
    R, n = X.shape
    dev, dt = X.device, X.dtype
    all_rows = torch.arange(R, device=dev)
    f, g = fun(X, all_rows)
    f_calls = torch.ones(R, dtype=torch.int64, device=dev)
    iters = torch.zeros(R, dtype=torch.int64, device=dev)
    S = torch.zeros(m, R, n, dtype=dt, device=dev)
    Y = torch.zeros(m, R, n, dtype=dt, device=dev)
    rho = torch.zeros(m, R, dtype=dt, device=dev)
    hist = torch.zeros(R, dtype=torch.int64, device=dev)     # stored pairs (<= m)
    head = torch.zeros(R, dtype=torch.int64, device=dev)     # next slot (ring buffer)
    g_thr = torch.clamp(g_reltol * torch.amax(torch.abs(g), dim=1), min=g_tol)
    gconv = torch.amax(torch.abs(g), dim=1) <= g_thr
    fconv = torch.zeros(R, dtype=torch.bool, device=dev)
    xconv = torch.zeros(R, dtype=torch.bool, device=dev)
    lsfail = torch.zeros(R, dtype=torch.bool, device=dev)
    gamma = torch.ones(R, dtype=dt, device=dev)
    timed_out = False
    stopped = callback is not None and bool(callback(X, f, g, iters))
    while not stopped:
        active = ~(gconv | fconv | xconv | lsfail) & (iters < iterations)
        if f_calls_limit > 0:
            active = active & (f_calls < f_calls_limit)
        if not math.isnan(time_limit) and time.perf_counter() - t_start > time_limit:
            timed_out = True
            break
        if not bool(active.any()):
            break
        # ---- two-loop recursion (ring buffer, newest first), batched over rows
        if X.is_cuda and not _TORCH_TWO_LOOP:  # one launch: csrc/grape_lbfgs.hip
            D = _device_direction(S, Y, rho, head, hist, gamma, g)
        else:
            D = _torch_direction(S, Y, rho, head, hist, gamma, g)
        dphi0 = _rowdot(g, D)
        # not a descent direction: restart from -g (masked, so no host sync)
        bad = ~(dphi0 < 0) & active
        D = torch.where(bad[:, None], -g, D)
        dphi0 = torch.where(bad, _rowdot(g, D), dphi0)
        hist = torch.where(bad, torch.zeros_like(hist), hist)
        gamma = torch.where(bad, torch.ones_like(gamma), gamma)
        # ---- strong-Wolfe line search, all active rows in lock step
        f0 = f.clone()
        phase = torch.where(active, torch.zeros_like(iters), torch.full_like(iters, 2))  # 0 bracket 1 zoom 2 done
        a_cur = torch.ones(R, dtype=dt, device=dev)
        a_prev = torch.zeros(R, dtype=dt, device=dev)
        f_prev, dp_prev = f0.clone(), dphi0.clone()
        a_lo, f_lo, dp_lo = a_prev.clone(), f0.clone(), dphi0.clone()
        a_hi, f_hi, dp_hi = a_prev.clone(), f0.clone(), dphi0.clone()
        Xn, fn, gn = X.clone(), f.clone(), g.clone()
        accepted = torch.zeros(R, dtype=torch.bool, device=dev)
        first = torch.ones(R, dtype=torch.bool, device=dev)
        for _ in range(MAX_LS_ROUNDS):
            rows = torch.nonzero(phase < 2).flatten()  # the round's one host sync
            if rows.numel() == 0:
                break
            a = a_cur[rows]
            Xt = X[rows] + a[:, None] * D[rows]
            ft, gt = fun(Xt, rows)
            f_calls[rows] += 1
            dpt = _rowdot(gt, D[rows])
            f0r, d0r = f0[rows], dphi0[rows]
            armijo = ft <= f0r + C1 * a * d0r
            curv = torch.abs(dpt) <= -C2 * d0r
            ph = phase[rows]
            newph = ph.clone()
            # bracketing phase (alg. 3.5)
            br = ph == 0
            to_zoom_a = br & (~armijo | (~first[rows] & (ft >= f_prev[rows])))
            acc_b = br & ~to_zoom_a & curv
            to_zoom_b = br & ~to_zoom_a & ~acc_b & (dpt >= 0)
            expand = br & ~to_zoom_a & ~acc_b & ~to_zoom_b
            # zoom phase (alg. 3.6)
            zm = ph == 1
            z_hi = zm & (~armijo | (ft >= f_lo[rows]))
            z_acc = zm & ~z_hi & curv
            z_flip = zm & ~z_hi & ~z_acc & (dpt * (a_hi[rows] - a_lo[rows]) >= 0)
            z_lo = zm & ~z_hi & ~z_acc
            acc = acc_b | z_acc
            # bookkeeping on the row subset
            A_lo, F_lo, P_lo = a_lo[rows], f_lo[rows], dp_lo[rows]
            A_hi, F_hi, P_hi = a_hi[rows], f_hi[rows], dp_hi[rows]
            Ap, Fp, Pp = a_prev[rows], f_prev[rows], dp_prev[rows]
            # bracket (a): zoom(a_prev, a)
            A_lo = torch.where(to_zoom_a, Ap, A_lo)
            F_lo = torch.where(to_zoom_a, Fp, F_lo)
            P_lo = torch.where(to_zoom_a, Pp, P_lo)
            A_hi = torch.where(to_zoom_a, a, A_hi)
            F_hi = torch.where(to_zoom_a, ft, F_hi)
            P_hi = torch.where(to_zoom_a, dpt, P_hi)
            # bracket (b): zoom(a, a_prev)
            A_lo = torch.where(to_zoom_b, a, A_lo)
            F_lo = torch.where(to_zoom_b, ft, F_lo)
            P_lo = torch.where(to_zoom_b, dpt, P_lo)
            A_hi = torch.where(to_zoom_b, Ap, A_hi)
            F_hi = torch.where(to_zoom_b, Fp, F_hi)
            P_hi = torch.where(to_zoom_b, Pp, P_hi)
            # zoom: new hi
            A_hi = torch.where(z_hi, a, A_hi)
            F_hi = torch.where(z_hi, ft, F_hi)
            P_hi = torch.where(z_hi, dpt, P_hi)
            # zoom: flip (hi <- lo) then lo <- a
            A_hi = torch.where(z_flip, a_lo[rows], A_hi)
            F_hi = torch.where(z_flip, f_lo[rows], F_hi)
            P_hi = torch.where(z_flip, dp_lo[rows], P_hi)
            A_lo = torch.where(z_lo, a, A_lo)
            F_lo = torch.where(z_lo, ft, F_lo)
            P_lo = torch.where(z_lo, dpt, P_lo)
            newph = torch.where(to_zoom_a | to_zoom_b, torch.ones_like(newph), newph)
            newph = torch.where(acc, torch.full_like(newph, 2), newph)
            # the best Armijo point so far is kept as a fallback
            better = armijo & (ft < fn[rows])
            keep = acc | better
            Xn[rows] = torch.where(keep[:, None], Xt, Xn[rows])
            fn[rows] = torch.where(keep, ft, fn[rows])
            gn[rows] = torch.where(keep[:, None], gt, gn[rows])
            accepted[rows[acc]] = True
            # next trial step
            zoom_now = newph == 1
            a_zoom = _cubic_min(A_lo, F_lo, P_lo, A_hi, F_hi, P_hi)
            a_next = torch.where(expand, 4.0 * a, a)
            a_next = torch.where(zoom_now, a_zoom, a_next)
            # a collapsed bracket ends the search (keep the best Armijo point if any)
            tiny = zoom_now & (torch.abs(A_hi - A_lo) <= 1e-12 * torch.maximum(torch.abs(A_lo), torch.ones_like(A_lo)))
            newph = torch.where(tiny, torch.full_like(newph, 2), newph)
            a_prev[rows] = torch.where(expand, a, Ap)
            f_prev[rows] = torch.where(expand, ft, Fp)
            dp_prev[rows] = torch.where(expand, dpt, Pp)
            a_lo[rows], f_lo[rows], dp_lo[rows] = A_lo, F_lo, P_lo
            a_hi[rows], f_hi[rows], dp_hi[rows] = A_hi, F_hi, P_hi
            a_cur[rows] = a_next
            phase[rows] = newph
            first[rows] = False
        moved = active & (fn < f0)
        lsfail = lsfail | (active & ~moved & ~accepted)
        step = active & (accepted | moved)
        # ---- L-BFGS update and convergence (Optim's rules)
        s = Xn - X
        y = gn - g
        sy = _rowdot(s, y)
        upd = step & (sy > 0)
        # masked ring-buffer update of every row (no host sync; rows without an update keep theirs)
        slot = head
        S[slot, all_rows] = torch.where(upd[:, None], s, S[slot, all_rows])
        Y[slot, all_rows] = torch.where(upd[:, None], y, Y[slot, all_rows])
        rho[slot, all_rows] = torch.where(upd, 1.0 / sy, rho[slot, all_rows])
        head = torch.where(upd, (head + 1) % m, head)
        hist = torch.where(upd, torch.clamp(hist + 1, max=m), hist)
        gamma = torch.where(upd, sy / _rowdot(y, y), gamma)
        if steepest:  # GradientDescent: no curvature pairs, D = -g next iteration
            hist = torch.zeros_like(hist)
            gamma = torch.ones_like(gamma)
        fold = f.clone()
        X = torch.where(step[:, None], Xn, X)
        f = torch.where(step, fn, f)
        g = torch.where(step[:, None], gn, g)
        iters = iters + step.to(iters.dtype)
        gconv = gconv | (step & (torch.amax(torch.abs(g), dim=1) <= g_thr))
        df = torch.abs(f - fold)
        fconv = fconv | (step & ((df <= f_abstol) | (df <= f_reltol * torch.abs(f))))
        dx = torch.amax(torch.abs(s), dim=1)
        xconv = xconv | (step & ((dx <= x_abstol) | (dx <= x_reltol * torch.amax(torch.abs(X), dim=1))))
        if callback is not None and bool(callback(X, f, g, iters)):
            break
    if hasattr(fun, "check"):  # deferred device status of the last evaluation (RobustCost)
        fun.check()
    return BatchResult(X, f, g, iters, f_calls, gconv, fconv, xconv, lsfail,
                       time.perf_counter() - t_start, {"timed_out": timed_out})


# ---------------------------------------------------------------------------
# the reference's cost (calculate_common!) on the GPU
# ---------------------------------------------------------------------------
class RobustCost:
    """cost(X) and its gradient for a batch of control vectors, FidelityCalculations.jl:172-196.

    The fidelity terms come from the GPU engine in one batched pass; the error-source and
    regulariser terms are assembled with torch on the same device."""

    def __init__(self, fp: FidelityRobustGRAPEProblem, params: FidelityRobustGRAPEParameters, nparam: int,
                 max_batch: int, device: int = 0, evaluate: Optional[Callable] = None,
                 scan_waves: Optional[int] = None, options: int = 0):
        up = fp.unitary_problem
        self.fp, self.up, self.nparam = fp, up, nparam
        self.ntimes, self.na = up.ntimes, up.nb_additional_param
        self.nx = nparam * up.ntimes + up.nb_additional_param
        self.nerr = len(up.error_sources)
        self.params = params
        self.c1 = [float(c) for c in params.regularization_coeff1]
        self.c2 = [float(c) for c in params.regularization_coeff2]
        self.ce = [float(c) for c in params.error_source_coeff]
        self.regs = list(params.regularization_functions)
        self._evaluate = evaluate
        self._unchecked = False
        self._stream = None
        self.plan = None
        self._fused = None
        if evaluate is None:
            from .engine import GrapePlan
            # Line-search rounds are latency-bound (most rounds evaluate a few rows): the widest scan
            # (most chunks: the shortest chunk walks) unless the caller chooses; c4opt at B = 1 024:
            # 0.93 -> 1.04 M evals/s (profiles/r03/c4opt)
            if scan_waves is None:
                scan_waves = 8 if max_batch <= 4096 else 0
            self.plan = GrapePlan(fp, nparam, device=device, max_batch=max_batch, scan_waves=scan_waves,
                                  options=options)
            self.device = torch.device("cuda", device)
            # the reference's own regularisers (no user transform) and an operator-basis plan:
            # the whole cost in one launch (grape_robust_cost); anything else stays in torch
            from . import regularization as REG
            kinds = [2 if fn is REG.regularization_cost_phase else 1 if fn is REG.regularization_cost else -1
                     for fn in self.regs]
            # (grape_robust_cost reads one regulariser kind per control parameter)
            if (not self.plan.tables and len(kinds) == nparam and all(k > 0 for k in kinds)
                    and 4 <= self.ntimes <= 4096):
                dev = self.device
                self._fused = {"kind": torch.tensor(kinds, dtype=torch.int32, device=dev),
                               "c1": torch.tensor(self.c1, dtype=torch.float64, device=dev),
                               "c2": torch.tensor(self.c2, dtype=torch.float64, device=dev),
                               "ce": torch.tensor(self.ce + [0.0], dtype=torch.float64, device=dev)}
        else:
            self.device = torch.device("cpu")

    def check(self):
        """Raise the device error of the last evaluation, if any (synchronises the plan's stream)."""
        if self._unchecked and self.plan is not None:
            self._unchecked = False
            self.plan.synchronize()

    def close(self):
        if self.plan is not None:
            self.check()
            self.plan.close()
            self.plan = None

    def fidelity_terms(self, X: torch.Tensor, raw: bool = False):
        """(F (r,), F_dx (r,nx), F_d2err (r,ne), F_d2err_dx (r,nx,ne)) for the rows of X
        (raw: F_d2err_dx in the engine's (r, ne, nx) layout, F_d2err (r, max(ne, 1)))."""
        if self._evaluate is not None:
            return self._evaluate(X)
        X = X.contiguous()
        r = X.shape[0]
        if self.plan.tables:
            # closure problem: the host evaluates the closures into tables, the device does
            # the rest (grape_fidelity_grad_tables; host arrays in and out)
            F, Fdx, Fd2, Fd2dx = (torch.as_tensor(a, device=X.device)
                                  for a in self.plan.fidelity_grad(X.detach().cpu().numpy()))
            return F, Fdx, Fd2, Fd2dx
        F = torch.empty(r, dtype=torch.float64, device=X.device)
        Fdx = torch.empty(r, self.nx, dtype=torch.float64, device=X.device)
        Fd2 = torch.empty(r, max(1, self.nerr), dtype=torch.float64, device=X.device)
        Fd2dx = torch.empty(r, max(1, self.nerr), self.nx, dtype=torch.float64, device=X.device)
        # The plan runs on its own torch stream, ordered after the producer of X and before
        # every consumer of the outputs by stream waits (torch's default stream is the null
        # stream, which grape_plan_set_stream cannot name: NULL selects the plan's stream).
        cur = torch.cuda.current_stream(X.device)
        if self._stream is None:
            self._stream = torch.cuda.Stream(X.device)
            self.plan.set_stream(self._stream.cuda_stream)
        self._stream.wait_stream(cur)
        self.plan.fidelity_grad_device_async(X.data_ptr(), F.data_ptr(), Fdx.data_ptr(), r,
                                             Fd2.data_ptr() if self.nerr else 0,
                                             Fd2dx.data_ptr() if self.nerr else 0)
        cur.wait_stream(self._stream)
        # raises on a singular Pade denominator (a deferred check measured slower: 99k vs 118k)
        self._unchecked = True
        self.check()
        if raw:
            return F, Fdx, Fd2, Fd2dx
        if not self.nerr:
            return F, Fdx, Fd2[:, :0], Fd2dx[:, :0, :].transpose(1, 2)
        return F, Fdx, Fd2, Fd2dx.transpose(1, 2)

    def __call__(self, X: torch.Tensor, rows=None):
        if self._fused is not None and X.is_cuda:
            return self._fused_cost(X)
        F, Fdx, Fd2, Fd2dx = self.fidelity_terms(X)
        cost = 1.0 - F
        grad = -Fdx
        if self.nerr:
            ce = torch.tensor(self.ce, dtype=X.dtype, device=X.device)
            cost = cost + torch.sum(ce[None, :] * Fd2 ** 2, dim=1)
            grad = grad + 2.0 * torch.sum((ce[None, :] * Fd2)[:, None, :] * Fd2dx, dim=2)
        nm = self.nparam * self.ntimes
        xm = X[:, :nm].reshape(X.shape[0], self.ntimes, self.nparam)
        reg_cost = torch.zeros_like(cost)
        reg_grad = torch.zeros(X.shape[0], self.ntimes, self.nparam, dtype=X.dtype, device=X.device)
        for p, fn in enumerate(self.regs):
            r1, j1, r2, j2 = _call_reg(fn, xm[:, :, p])
            reg_cost = reg_cost + (self.c1[p] * r1 + self.c2[p] * r2)
            reg_grad[:, :, p] = self.c1[p] * j1 + self.c2[p] * j2
        cost = cost + reg_cost
        grad = grad.clone()
        grad[:, :nm] += reg_grad.reshape(X.shape[0], nm)
        return cost, grad

    def _fused_cost(self, X):
        """cost and gradient of the rows of X with one launch after the engine (grape_robust_cost)."""
        import ctypes

        from . import _capi
        X = X.contiguous()
        F, Fdx, Fd2, Fd2dx = self.fidelity_terms(X, raw=True)
        r = X.shape[0]
        cost = torch.empty(r, dtype=torch.float64, device=X.device)
        grad = torch.empty(r, self.nx, dtype=torch.float64, device=X.device)
        fz = self._fused
        p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        _capi.check(_capi.lib().grape_robust_cost(
            r, self.nparam, self.ntimes, self.na, self.nerr, p(X), p(F), p(Fdx), p(Fd2), p(Fd2dx), p(fz["ce"]),
            p(fz["c1"]), p(fz["c2"]), p(fz["kind"]), p(cost), p(grad),
            ctypes.c_void_p(torch.cuda.current_stream(X.device).cuda_stream)))
        return cost, grad


def _call_reg(fn, xp: torch.Tensor):
    """Batched call when the function supports it, else the reference's 1-D signature per row."""
    if getattr(fn, "batched", False):
        return fn(xp)
    outs = [fn(row.detach().cpu().numpy()) for row in xp]
    t = lambda v: torch.as_tensor(np.asarray(v, dtype=np.float64), device=xp.device)
    return (t([o[0] for o in outs]), torch.stack([t(o[1]) for o in outs]),
            t([o[2] for o in outs]), torch.stack([t(o[3]) for o in outs]))


@dataclass(frozen=True)
class LBFGS:
    """Optim.LBFGS(; m = 10) (the reference's default solver_algorithm, Types.jl:82): limited-memory
    BFGS with m correction pairs and the s.y/y.y initial inverse-Hessian scaling."""
    m: int = 10


@dataclass(frozen=True)
class GradientDescent:
    """Optim.GradientDescent(): steepest descent, direction -g (no preconditioner), with this
    module's strong-Wolfe line search in place of Optim's Hager-Zhang."""


_SOLVER_NAMES = {"LBFGS": LBFGS, "GradientDescent": GradientDescent}


def solver_config(algorithm):
    """(history m, steepest) for FidelityRobustGRAPEParameters.solver_algorithm (Types.jl:82, used
    at FidelityCalculations.jl:211-213).  Accepts LBFGS(m=...) / GradientDescent() instances, the
    classes, or their names ("LBFGS", "LBFGS()", "GradientDescent", "GradientDescent()").  Any
    other Optim.FirstOrderOptimizer (BFGS, ConjugateGradient, Momentum, ...) is not implemented
    here and raises TypeError rather than silently running L-BFGS."""
    alg = algorithm
    if isinstance(alg, str):
        name = alg.strip()
        name = name[:-2] if name.endswith("()") else name
        if name not in _SOLVER_NAMES:
            raise TypeError(f"unsupported solver_algorithm {algorithm!r}: LBFGS(m=...) or GradientDescent()")
        alg = _SOLVER_NAMES[name]
    if isinstance(alg, type) and alg in (LBFGS, GradientDescent):
        alg = alg()
    if isinstance(alg, LBFGS):
        if not (isinstance(alg.m, (int, np.integer)) and alg.m >= 1):
            raise ValueError("LBFGS memory m must be a positive integer")
        return int(alg.m), False
    if isinstance(alg, GradientDescent):
        return 1, True
    raise TypeError(f"unsupported solver_algorithm {algorithm!r}: LBFGS(m=...) or GradientDescent()")


def _checks(fp, params, nx):
    up = fp.unitary_problem
    nerr = len(up.error_sources)
    if len(params.error_source_coeff) != nerr:
        raise AssertionError("error_source_coeff must have one entry per error source")
    nparam = (nx - up.nb_additional_param) // up.ntimes
    if not (len(params.regularization_coeff1) == len(params.regularization_coeff2)
            == len(params.regularization_functions) == nparam):
        raise AssertionError("regularization functions / coefficients must have one entry per control")
    return nparam


# Optim.Options keywords the reference forwards from fidelity_parameters.additional_parameters
# (FidelityCalculations.jl:211-216; Optim.jl is third party, absent here).  Accepted without
# effect: the options of Optim features this solver does not have (f increases are never
# accepted by the strong-Wolfe search; no Hessian; one outer loop).
_OPTIM_STOP = ("g_tol", "g_abstol", "g_reltol", "f_abstol", "f_reltol", "f_tol", "x_abstol", "x_reltol", "x_tol",
               "f_calls_limit", "g_calls_limit")
_OPTIM_TRACE = ("show_trace", "show_every", "store_trace", "extended_trace", "callback")
_OPTIM_NOOP = ("allow_f_increases", "allow_outer_f_increases", "successive_f_tol", "show_warnings",
               "h_calls_limit", "outer_iterations", "outer_x_abstol", "outer_x_reltol", "outer_f_abstol",
               "outer_f_reltol", "outer_g_abstol", "outer_g_reltol", "trace_simplex")


class _OptimTrace:
    """Optim's show_trace / show_every / extended_trace printout and store_trace record for
    restart 0 (the single optimisation of optimize_fidelity_and_error_sources), plus the
    user's callback (Optim passes the trace state; returning true stops the run)."""

    def __init__(self, show, every, store, extended, user_cb, t0):
        self.show, self.every, self.store, self.extended = show, max(1, int(every)), store, extended
        self.user_cb, self.t0, self.trace = user_cb, t0, []
        self.last = -1

    def __call__(self, X, f, g, iters):
        it = int(iters[0])
        if it == self.last:  # restart 0 did not move this round
            return False
        self.last = it
        state = {"iteration": it, "value": float(f[0]), "g_norm": float(torch.amax(torch.abs(g[0]))),
                 "time": time.perf_counter() - self.t0}
        if self.extended:
            state["x"] = X[0].detach().cpu().numpy().copy()
            state["g(x)"] = g[0].detach().cpu().numpy().copy()
        if self.store:
            self.trace.append(state)
        if self.show and it % self.every == 0:
            if it == 0:
                print("Iter     Function value   Gradient norm ")
            print(f"{it:6d}   {state['value']:14e}   {state['g_norm']:14e}")
            print(f" * time: {state['time']}")
            if self.extended:
                print(f" * x: {state['x']}")
                print(f" * g(x): {state['g(x)']}")
        return bool(self.user_cb(state)) if self.user_cb is not None else False


def _solver_options(params):
    """lbfgs_batched keywords from FidelityRobustGRAPEParameters (iterations, time_limit and the
    Optim.Options pass-through); an unknown keyword raises like Julia's keyword MethodError."""
    ap = {str(k).lstrip(":"): v for k, v in dict(params.additional_parameters).items()}
    unknown = sorted(set(ap) - set(_OPTIM_STOP + _OPTIM_TRACE + _OPTIM_NOOP))
    if unknown:
        raise TypeError(f"unsupported Optim option(s): {', '.join(unknown)}")
    opts = dict(iterations=int(params.iterations), time_limit=float(params.time_limit),
                g_tol=float(ap.get("g_tol", ap.get("g_abstol", 1e-8))), g_reltol=float(ap.get("g_reltol", 0.0)),
                f_abstol=float(ap.get("f_abstol", 0.0)), f_reltol=float(ap.get("f_reltol", ap.get("f_tol", 0.0))),
                x_abstol=float(ap.get("x_abstol", ap.get("x_tol", 0.0))), x_reltol=float(ap.get("x_reltol", 0.0)),
                f_calls_limit=int(max(ap.get("f_calls_limit", 0), ap.get("g_calls_limit", 0))))
    if any(ap.get(k) for k in ("show_trace", "store_trace", "extended_trace", "callback")):
        opts["callback"] = _OptimTrace(bool(ap.get("show_trace", False)), ap.get("show_every", 1),
                                       bool(ap.get("store_trace", False)), bool(ap.get("extended_trace", False)),
                                       ap.get("callback"), time.perf_counter())
    return opts


def optimize_restarts(fidelity_problem: FidelityRobustGRAPEProblem, fidelity_parameters: FidelityRobustGRAPEParameters,
                      X0, device: int = 0, evaluate: Optional[Callable] = None, m: Optional[int] = None) -> BatchResult:
    """Batched restarts: every row of X0 (R, n_x) is one optimisation of the reference's
    problem; all of them advance together on the GPU (see the module docstring).  The solver is
    fidelity_parameters.solver_algorithm (solver_config); `m` overrides its L-BFGS memory."""
    X0 = torch.as_tensor(np.asarray(X0, dtype=np.float64) if not isinstance(X0, torch.Tensor) else X0,
                         dtype=torch.float64)
    if X0.dim() != 2:
        raise AssertionError("X0 must be (restarts, n_x)")
    nparam = _checks(fidelity_problem, fidelity_parameters, X0.shape[1])
    m_alg, steepest = solver_config(fidelity_parameters.solver_algorithm)
    m = m_alg if m is None else int(m)
    opts = _solver_options(fidelity_parameters)  # (raises on unknown options before any device work)
    # workspace for at most MAX_PLAN_BATCH restarts per device pass: larger sweeps are
    # chunked by the C side instead of failing to allocate
    cost = RobustCost(fidelity_problem, fidelity_parameters, nparam, max_batch=min(X0.shape[0], MAX_PLAN_BATCH),
                      device=device, evaluate=evaluate)
    try:
        res = lbfgs_batched(cost, X0.to(cost.device), m=m, steepest=steepest, **opts)
    finally:
        cost.close()
    if isinstance(opts.get("callback"), _OptimTrace):
        res.extra["trace"] = opts["callback"].trace
    return res


def optimize_fidelity_and_error_sources(fidelity_problem: FidelityRobustGRAPEProblem,
                                        fidelity_parameters: FidelityRobustGRAPEParameters,
                                        device: int = 0, evaluate: Optional[Callable] = None) -> OptimizationResult:
    """FidelityCalculations.jl:161-218: one optimisation from fidelity_parameters.x_initial."""
    x0 = np.asarray(fidelity_parameters.x_initial, dtype=np.float64)
    res = optimize_restarts(fidelity_problem, fidelity_parameters, x0[None, :], device=device, evaluate=evaluate)
    return res.result(0)
