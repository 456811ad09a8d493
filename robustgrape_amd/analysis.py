"""Error-analysis entry points of the reference on the GPU.

* ``calculate_interaction_error_operators`` -- src/UnitaryCalculations.jl:180-204,
  HIP kernels behind ``grape_interaction_error_operators`` (nominal propagators
  from the engine's k_expm, the chain C_k, then C_{k-1}^dagger Herror C_{k-1}).
* ``calculate_expectation_values`` -- src/FidelityCalculations.jl:368-390,
  ``grape_expectation_values``.
* ``calculate_fidelity_response`` (:246-280) and ``calculate_fidelity_response_fft``
  (:306-343): the interaction operators stay on the device and the frequency sums,
  FFTs (rocFFT through torch.fft) and trace contractions run there as batched
  tensor ops; only the (nfreq, nerr) result comes back.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch

from . import _capi
from .engine import fidelity_wrapper, locked_plan
from .operators import host_interaction_tables
from .types import FidelityRobustGRAPEProblem, split_x

def _problem(fp_or_up, x):
    """(fidelity problem, nparam): a UnitaryRobustGRAPEProblem is wrapped (the descriptor needs a
    projector and a target, unused here)."""
    fp = fp_or_up if isinstance(fp_or_up, FidelityRobustGRAPEProblem) else fidelity_wrapper(fp_or_up)
    _, _, nparam = split_x(fp.unitary_problem, x)
    return fp, nparam


def calculate_interaction_error_operators(unitary_problem, x, device: int = 0) -> np.ndarray:
    """(ndim, ndim, ntimes, nerr) complex, like the reference's permuted tensor."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    fp, nparam = _problem(unitary_problem, x)
    up = fp.unitary_problem
    O = np.zeros((up.ndim, up.ndim, up.ntimes, len(up.error_sources)), dtype=np.complex128, order="F")
    if O.size:
        with locked_plan(fp, nparam, device) as plan:
            if plan.tables:  # closure problem: H0 / Herror evaluated here (the reference's calls)
                H0, Oerr = host_interaction_tables(up, x, plan.nparam)
                plan.general_h0_for(H0)
                _capi.check(_capi.lib().grape_interaction_error_operators_tables(
                    plan.handle, _capi.dptr(x), _capi.dptr(H0), _capi.dptr(Oerr), O.ctypes.data, 0))
            else:
                _capi.check(_capi.lib().grape_interaction_error_operators(plan.handle, _capi.dptr(x),
                                                                           _capi.dptr(O)))
    return O


def calculate_expectation_values(fidelity_problem: FidelityRobustGRAPEProblem, x, device: int = 0) -> np.ndarray:
    """(ntimes, nerr) real."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    fp, nparam = _problem(fidelity_problem, x)
    up = fp.unitary_problem
    ev = np.zeros((up.ntimes, len(up.error_sources)), dtype=np.float64, order="F")
    if ev.size:
        with locked_plan(fp, nparam, device) as plan:
            if plan.tables:
                H0, Oerr = host_interaction_tables(up, x, plan.nparam)
                plan.general_h0_for(H0)
                _capi.check(_capi.lib().grape_expectation_values_tables(
                    plan.handle, _capi.dptr(x), _capi.dptr(H0), _capi.dptr(Oerr), _capi.dptr(ev)))
            else:
                _capi.check(_capi.lib().grape_expectation_values(plan.handle, _capi.dptr(x), _capi.dptr(ev)))
    return ev


def _device_operators(fp, x, device):
    """Interaction operators as a (nerr, ntimes, d, d) complex128 tensor, written by the HIP
    kernels straight into device memory (grape_interaction_error_operators_device): they never
    visit the host."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    fp, nparam = _problem(fp, x)
    up = fp.unitary_problem
    d, nt, ne = up.ndim, up.ntimes, len(up.error_sources)
    # the reference's column-major (d, d, nt, ne) tensor is the C-order (ne, nt, d_col, d_row) one
    O = torch.empty(ne, nt, d, d, dtype=torch.complex128, device=torch.device("cuda", device))
    torch.cuda.synchronize(O.device)
    with locked_plan(fp, nparam, device) as plan:
        if plan.tables:
            H0, Oerr = host_interaction_tables(up, x, plan.nparam)
            plan.general_h0_for(H0)
            _capi.check(_capi.lib().grape_interaction_error_operators_tables(
                plan.handle, _capi.dptr(x), _capi.dptr(H0), _capi.dptr(Oerr), O.data_ptr(), 1))
        else:
            _capi.check(_capi.lib().grape_interaction_error_operators_device(
                plan.handle, _capi.dptr(x), ctypes.c_void_p(O.data_ptr())))
    return O.transpose(-1, -2)


def _projector_parts(fp, dev):
    """FidelityCalculations.jl:256-260: P0 = projector (any real matrix), P = P0 with every nonzero
    entry set to 1, D = Re tr(P0); tr_mod(X) = tr(P0 X)."""
    P0n = np.asarray(fp.projector, dtype=np.float64)
    P0 = torch.as_tensor(P0n.astype(np.complex128), device=dev)
    P = torch.as_tensor((P0n != 0).astype(np.complex128), device=dev)
    return P0, P, float(np.trace(P0n))


def _response_terms(A, B, P0, P, D):
    """Re of the three trace terms of :268-272 / :333-337 for matching stacks A, B (..., d, d):
    1/D tr_mod(A B P) - 1/(D(D+1)) tr_mod(A P B P) - 1/(D(D+1)) tr_mod(A P) tr_mod(B P), before Re,
    with tr_mod(X) = tr(P0 X) = sum_ij P0_ij X_ji."""
    def trm(X):
        return torch.einsum("ij,...ji->...", P0, X)
    AP, BP = A @ P, B @ P
    t1 = trm(A @ BP)
    t2 = trm(AP @ BP)
    t3 = trm(AP) * trm(BP)
    return t1 / D - t2 / (D * (D + 1)) - t3 / (D * (D + 1))


def calculate_fidelity_response(fidelity_problem: FidelityRobustGRAPEProblem, x, normalized_frequencies,
                                device: int = 0) -> np.ndarray:
    """src/FidelityCalculations.jl:246-280 -> (nfreq, nerr)."""
    up = fidelity_problem.unitary_problem
    nt, dt = up.ntimes, up.t0 / up.ntimes
    w = torch.as_tensor(np.asarray(normalized_frequencies, dtype=np.float64))
    nerr = len(up.error_sources)
    if nerr == 0 or w.numel() == 0:
        return np.zeros((w.numel(), nerr))
    O = _device_operators(fidelity_problem, x, device)                # (ne, nt, d, d)
    dev = O.device
    P0, P, D = _projector_parts(fidelity_problem, dev)
    w = w.to(dev)
    k0 = torch.arange(nt, dtype=torch.float64, device=dev)            # time_indices (0-based, :262)
    k1 = k0 + 1.0                                                     # k = 1..ntimes (:266)
    out = torch.empty(w.numel(), nerr, dtype=torch.float64, device=dev)
    for e in range(nerr):
        ph0 = torch.exp(-1j * w[:, None] * dt * k0[None, :])            # (nf, nt)
        S = torch.einsum("ft,tij->fij", ph0, O[e])                    # sum_error_freq per frequency
        ph1 = torch.exp(1j * w[:, None] * dt * k1[None, :])             # (nf, nt)
        terms = _response_terms(O[e][None, :, :, :], S[:, None, :, :], P0, P, D)  # (nf, nt)
        out[:, e] = dt ** 2 * torch.sum(torch.real(ph1 * terms), dim=1)
    return out.cpu().numpy()


def calculate_fidelity_response_fft(fidelity_problem: FidelityRobustGRAPEProblem, x, oversampling: int = 1,
                                    device: int = 0):
    """src/FidelityCalculations.jl:306-343 -> (response (ntimes*oversampling, nerr), norm_frequencies)."""
    if oversampling < 1:
        raise AssertionError("oversampling >= 1")
    up = fidelity_problem.unitary_problem
    nt, dt = up.ntimes, up.t0 / up.ntimes
    N = nt * oversampling
    nerr = len(up.error_sources)
    freqs = (2 * math.pi / (N * dt)) * np.arange(N, dtype=np.float64)
    if nerr == 0:
        return np.zeros((N, 0)), freqs
    O = _device_operators(fidelity_problem, x, device)
    dev = O.device
    P0, P, D = _projector_parts(fidelity_problem, dev)
    out = torch.empty(N, nerr, dtype=torch.float64, device=dev)
    for e in range(nerr):
        Oe = torch.zeros(N, up.ndim, up.ndim, dtype=torch.complex128, device=dev)
        Oe[:nt] = O[e]
        Ff = torch.fft.fft(Oe, dim=0)
        Fi = N * torch.fft.ifft(Oe, dim=0)
        out[:, e] = dt ** 2 * torch.real(_response_terms(Fi, Ff, P0, P, D))
    return out.cpu().numpy(), freqs
