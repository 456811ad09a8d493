"""Pulse regularisers, src/Regularization.jl:26-115, batched over restarts.

Each function keeps the reference signature -- one control's time series
``x`` (length ntimes) in, ``(reg1, jac1, reg2, jac2)`` out -- and also accepts a
2-D torch tensor (restarts, ntimes) on any device, returning per-row costs
(restarts,) and gradients (restarts, ntimes).  The optimiser
(:mod:`robustgrape_amd.optimize`) calls them on the GPU-resident batch.

The arithmetic follows the reference's own stencils and evaluation order
(jac2's explicit end rows, Regularization.jl:39-45) so results match the CPU
restatement in oracle/grape_oracle.py to rounding.
"""
from __future__ import annotations

import numpy as np
import torch


def _as_batch(x):
    if isinstance(x, torch.Tensor):
        return x if x.dim() == 2 else x[None, :], x.dim() == 1, True
    t = torch.as_tensor(np.asarray(x, dtype=np.float64))
    return t[None, :], True, False


def _unbatch(res, single, is_torch):
    r1, j1, r2, j2 = res
    if single:
        r1, j1, r2, j2 = r1[0], j1[0], r2[0], j2[0]
        if not is_torch:
            return float(r1), j1.numpy(), float(r2), j2.numpy()
    return r1, j1, r2, j2


def _reg(x: torch.Tensor):
    """Regularization.jl:26-48 on rows of x (n >= 4)."""
    n = x.shape[1]
    if n < 4:
        raise ValueError("regularization_cost needs at least 4 time steps (Regularization.jl:39-45)")
    d = x[:, 1:] - x[:, :-1]
    dd = d[:, 1:] - d[:, :-1]
    reg1 = torch.sum(d * d, dim=1)
    reg2 = torch.sum(dd * dd, dim=1)
    jac1 = torch.zeros_like(x)
    jac1[:, 1:n - 1] = -2.0 * dd
    jac1[:, 0] += -2.0 * d[:, 0]
    jac1[:, n - 1] += 2.0 * d[:, n - 2]
    jac2 = torch.empty_like(x)
    jac2[:, 0] = 2 * (x[:, 2] - 2 * x[:, 1] + x[:, 0])
    jac2[:, 1] = 2 * (x[:, 3] - 4 * x[:, 2] + 5 * x[:, 1] - 2 * x[:, 0])
    i = slice(2, n - 2)
    jac2[:, i] = 2 * (x[:, 4:] - 4 * x[:, 3:n - 1] + 6 * x[:, i] - 4 * x[:, 1:n - 3] + x[:, 0:n - 4])
    jac2[:, n - 2] = 2 * (x[:, n - 4] - 4 * x[:, n - 3] + 5 * x[:, n - 2] - 2 * x[:, n - 1])
    jac2[:, n - 1] = 2 * (x[:, n - 3] - 2 * x[:, n - 2] + x[:, n - 1])
    return reg1, jac1, reg2, jac2


def regularization_cost(x, f=None, df=None):
    """Regularization.jl:26 (x only) and :76 (transform f with derivative df,
    both elementwise torch functions, e.g. torch.sin / torch.cos)."""
    xb, single, is_torch = _as_batch(x)
    if f is None:
        return _unbatch(_reg(xb), single, is_torch)
    r1, j1, r2, j2 = _reg(f(xb))
    dfx = df(xb)
    return _unbatch((r1, dfx * j1, r2, dfx * j2), single, is_torch)


def regularization_cost_phase(phis):
    """Regularization.jl:111-115: regularise cos(phi) and sin(phi), summed."""
    xb, single, is_torch = _as_batch(phis)
    a = _reg(torch.cos(xb))
    b = _reg(torch.sin(xb))
    c, s = torch.cos(xb), torch.sin(xb)
    res = (a[0] + b[0], -s * a[1] + c * b[1], a[2] + b[2], -s * a[3] + c * b[3])
    return _unbatch(res, single, is_torch)


# marks the functions that accept a (restarts, ntimes) batch (see optimize.py)
for _f in (regularization_cost, regularization_cost_phase):
    _f.batched = True
