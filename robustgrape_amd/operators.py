"""Operator-basis descriptors: the device-side stand-in for the reference's closures.

The reference passes Julia closures ``H0(nt, x, x_add)``,
``Herror(nt, x, x_add, err)`` and ``target_unitary(x_add)`` (src/Types.jl:10,25,50).
A closure cannot run on the GPU, so the device path takes each of them as a
sum of fixed operators times scalar coefficients (see ``include/grape.h``):

    H(nt, x, x_add) = sum_t scale_t * f_t(a_t * v_t + b_t) * OP_t

Each descriptor is ALSO a callable with the reference signature, so it can be
handed to anything that expects the closure (including the CPU oracle).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Sequence, Tuple

import numpy as np

# grape_var / grape_func (include/grape.h)
VAR_ONE, VAR_X, VAR_XADD, VAR_TSTEP = 0, 1, 2, 3
FN_ONE, FN_LINEAR, FN_COS, FN_SIN, FN_CIS = 0, 1, 2, 3, 4


@dataclass(frozen=True)
class Term:
    """One coefficient * operator term (grape_term)."""
    op: np.ndarray          # (d, d) complex
    var: int = VAR_ONE
    index: int = 0
    func: int = FN_ONE
    a: float = 1.0
    b: float = 0.0
    scale: complex = 1.0

    def coefficient(self, nt, x, x_add):
        if self.var == VAR_ONE:
            v = 1.0
        elif self.var == VAR_X:
            v = float(x[self.index])
        elif self.var == VAR_XADD:
            v = float(x_add[self.index])
        elif self.var == VAR_TSTEP:
            v = float(nt)
        else:
            raise ValueError(f"bad var {self.var}")
        t = self.a * v + self.b
        if self.func == FN_ONE:
            f = 1.0
        elif self.func == FN_LINEAR:
            f = t
        elif self.func == FN_COS:
            f = np.cos(t)
        elif self.func == FN_SIN:
            f = np.sin(t)
        elif self.func == FN_CIS:
            f = complex(np.cos(t), np.sin(t))
        else:
            raise ValueError(f"bad func {self.func}")
        s = complex(self.scale)
        if isinstance(f, complex) or s.imag != 0.0:
            return s * f
        return s.real * f  # real coefficient times complex operator, like the closures


def _accumulate(terms: Sequence[Term], nt, x, x_add, ndim):
    H = np.zeros((ndim, ndim), np.complex128)
    for t in terms:
        H = H + t.coefficient(nt, x, x_add) * t.op
    return H


class OperatorBasisHamiltonian:
    """H0(nt, x, x_add) = sum_t c_t * OP_t  (a device-buildable H0 closure)."""

    def __init__(self, terms: Sequence[Term]):
        self.terms: Tuple[Term, ...] = tuple(terms)
        if not self.terms:
            raise ValueError("need at least one term")
        self.ndim = self.terms[0].op.shape[0]
        for t in self.terms:
            if t.op.shape != (self.ndim, self.ndim):
                raise ValueError("all operators must share one shape")
            if t.func == FN_CIS:
                raise ValueError("cis coefficients are only allowed in target terms")

    def __call__(self, nt, x, x_add):
        return _accumulate(self.terms, nt, x, x_add, self.ndim)

    def depends_on_xadd(self) -> bool:
        return any(t.var == VAR_XADD for t in self.terms)


class OperatorBasisError:
    """Herror(nt, x, x_add, err) = err * sum_t c_t * OP_t (linear in err)."""

    def __init__(self, terms: Sequence[Term]):
        self.terms: Tuple[Term, ...] = tuple(terms)
        if not self.terms:
            raise ValueError("need at least one term")
        self.ndim = self.terms[0].op.shape[0]
        for t in self.terms:
            if t.func == FN_CIS:
                raise ValueError("cis coefficients are only allowed in target terms")

    def __call__(self, nt, x, x_add, err):
        return err * _accumulate(self.terms, nt, x, x_add, self.ndim)


class OperatorBasisTarget:
    """target_unitary(x_add) = sum_t c_t(x_add) * OP_t."""

    def __init__(self, terms: Sequence[Term]):
        self.terms: Tuple[Term, ...] = tuple(terms)
        self.ndim = self.terms[0].op.shape[0]
        for t in self.terms:
            if t.var in (VAR_X, VAR_TSTEP):
                raise ValueError("target terms may only depend on x_add")

    def __call__(self, x_add):
        return _accumulate(self.terms, 1, (), x_add, self.ndim)


# ---------------------------------------------------------------------------
# ctypes mirror of grape_term / grape_desc (include/grape.h)
# ---------------------------------------------------------------------------
class CTerm(ctypes.Structure):
    _fields_ = [("op", ctypes.c_int32), ("var", ctypes.c_int32), ("index", ctypes.c_int32),
                ("func", ctypes.c_int32), ("a", ctypes.c_double), ("b", ctypes.c_double),
                ("scale_re", ctypes.c_double), ("scale_im", ctypes.c_double)]


class CDesc(ctypes.Structure):
    _fields_ = [("ndim", ctypes.c_int32), ("ntimes", ctypes.c_int32), ("nparam", ctypes.c_int32),
                ("nadd", ctypes.c_int32), ("nerr", ctypes.c_int32), ("n_ops", ctypes.c_int32),
                ("t0", ctypes.c_double), ("eps", ctypes.c_double), ("eps2", ctypes.c_double),
                ("projector_diag", ctypes.POINTER(ctypes.c_double)),
                ("ops", ctypes.POINTER(ctypes.c_double)),
                ("n_h0_terms", ctypes.c_int32), ("h0_terms", ctypes.POINTER(CTerm)),
                ("err_term_offsets", ctypes.POINTER(ctypes.c_int32)),
                ("err_terms", ctypes.POINTER(CTerm)),
                ("n_target_terms", ctypes.c_int32), ("target_terms", ctypes.POINTER(CTerm)),
                ("max_batch", ctypes.c_int32), ("reserved", ctypes.c_int32 * 5),
                ("projector", ctypes.POINTER(ctypes.c_double))]


def projector_arrays(fp):
    """(diagonal, full) host arrays of FidelityRobustGRAPEProblem.projector for grape_desc:
    the diagonal always; the full matrix (complex, column-major, interleaved) only when P0 is
    not diagonal -- then the engines run the general-projector heads (FidelityCalculations.jl:47-51)."""
    P = np.asarray(fp.projector, np.float64)
    pdiag = np.ascontiguousarray(np.diag(P).astype(np.float64))
    if not np.count_nonzero(P - np.diag(np.diag(P))):
        return pdiag, None
    full = np.empty(2 * P.size, np.float64)
    full[0::2] = P.reshape(-1, order="F")
    full[1::2] = 0.0
    return pdiag, full


# grape_desc.reserved[1] engine options (include/grape.h GRAPE_OPT_*): implementations of the
# same outputs, fixed at plan creation (A/B measurements and cross-path tests)
OPT_NO_SECTORS, OPT_NO_LANE, OPT_NO_CHAIN, OPT_NO_WALK, OPT_NO_GRAPH = 1, 2, 4, 8, 16
OPT_WALK_RECOMPUTE = 32
OPT_GENERAL_H0 = 64  # non-Hermitian H0: LU-inverted chain, fidelity from the materialised derivatives
OPT_NO_FORK = 128  # every call on the plan's one stream (no auxiliary stream for the second sector class)
OPT_GENERAL_HEAD = 256  # the general sector head even for a diagonal projector and target
OPT_NO_PAIR = 512  # latency-bound calls: one launch per sector class (not both classes per launch)
OPT_NO_SYMMETRY = 1024  # permutation sectors only (no symmetry-adapted basis, grape_symmetry.hpp)
OPT_NO_TWIN = 2048  # every walk sector computes its own exponentials (no twin sharing, grape_walk.hpp)
OPT_GRAPH_FORK = 4096  # accepted and ignored since round 5 (the captured fork was removed)
OPT_NO_GAUGE = 8192  # per-step exponentials even for phase-covariant walk classes (grape_walk.hpp GAUGE)
OPT_NO_EVAL1 = 16384  # latency-bound calls through the pair-kernel pipeline, not one workgroup per evaluation
OPT_NO_MERGE = 32768  # throughput passes: one walk kernel per sector class instead of merged lanes


def _reserved(flags: int = 0, options: int = 0, scan_waves: int = 0):
    if scan_waves not in (0, 1, 4, 8, 16):
        raise ValueError("scan_waves must be 0 (by batch size), 1, 4, 8 or 16 (chunk-walk classes only)")
    return (ctypes.c_int32 * 5)(int(flags), int(options), int(scan_waves), 0, 0)


class DescriptorBuffers:
    """Owns the host arrays a CDesc points into (keep alive while the C call runs)."""

    def __init__(self, fp, nparam: int, max_batch: int = 256, options: int = 0, scan_waves: int = 0):
        up = fp.unitary_problem
        if not isinstance(up.H0, OperatorBasisHamiltonian):
            raise TypeError("device path needs an OperatorBasisHamiltonian H0")
        if not isinstance(fp.target_unitary, OperatorBasisTarget):
            raise TypeError("device path needs an OperatorBasisTarget target_unitary")
        for es in up.error_sources:
            if not isinstance(es.Herror, OperatorBasisError):
                raise TypeError("device path needs OperatorBasisError error sources")
        ops: List[np.ndarray] = []
        index = {}

        def op_id(m):
            key = id(m)
            if key not in index:
                index[key] = len(ops)
                ops.append(np.asarray(m, np.complex128))
            return index[key]

        def cterms(terms):
            arr = (CTerm * max(1, len(terms)))()
            for i, t in enumerate(terms):
                s = complex(t.scale)
                arr[i] = CTerm(op_id(t.op), t.var, t.index, t.func, t.a, t.b, s.real, s.imag)
            return arr

        self.h0 = cterms(up.H0.terms)
        err_terms: List[Term] = []
        offs = [0]
        for es in up.error_sources:
            err_terms.extend(es.Herror.terms)
            offs.append(len(err_terms))
        self.err = cterms(err_terms)
        self.offs = (ctypes.c_int32 * len(offs))(*offs)
        self.target = cterms(fp.target_unitary.terms)
        d = up.ndim
        stack = np.stack([np.asfortranarray(o) for o in ops])  # (n_ops, d, d)
        inter = np.empty((len(ops), d * d * 2), np.float64)
        for k, o in enumerate(ops):
            flat = o.reshape(-1, order="F")
            inter[k, 0::2] = flat.real
            inter[k, 1::2] = flat.imag
        self.ops = np.ascontiguousarray(inter.reshape(-1))
        self.pdiag, self.pfull = projector_arrays(fp)
        dp = ctypes.POINTER(ctypes.c_double)
        self.desc = CDesc(
            ndim=d, ntimes=up.ntimes, nparam=nparam, nadd=up.nb_additional_param,
            nerr=len(up.error_sources), n_ops=len(ops), t0=float(up.t0), eps=float(up.eps),
            eps2=float(up.eps2), projector_diag=self.pdiag.ctypes.data_as(dp),
            ops=self.ops.ctypes.data_as(dp), n_h0_terms=len(up.H0.terms), h0_terms=self.h0,
            err_term_offsets=self.offs, err_terms=self.err,
            n_target_terms=len(fp.target_unitary.terms), target_terms=self.target,
            max_batch=int(max_batch), reserved=_reserved(0, options, scan_waves),
            projector=self.pfull.ctypes.data_as(dp) if self.pfull is not None else None)
        del stack


# ---------------------------------------------------------------------------
# closure fallback (GRAPE_DESC_HOST_TABLES, grape_fidelity_grad_tables)
# ---------------------------------------------------------------------------
GRAPE_DESC_HOST_TABLES = 1  # include/grape.h


def has_operator_basis_h(up) -> bool:
    """True when H0 and every error source of a UnitaryRobustGRAPEProblem are operator bases."""
    return isinstance(up.H0, OperatorBasisHamiltonian) and all(
        isinstance(es.Herror, OperatorBasisError) for es in up.error_sources)


def has_operator_basis(fp) -> bool:
    """True when H0, every error source and the target are operator bases (the fused device path)."""
    up = fp.unitary_problem
    return (isinstance(up.H0, OperatorBasisHamiltonian) and isinstance(fp.target_unitary, OperatorBasisTarget)
            and all(isinstance(es.Herror, OperatorBasisError) for es in up.error_sources))


class TableDescriptor:
    """grape_desc of a closure problem: no operator basis; the host evaluates the closures
    (host_tables) and the device does the rest (the SURVEY.md 8b fallback)."""

    def __init__(self, fp, nparam: int, max_batch: int = 256, options: int = 0, scan_waves: int = 0):
        up = fp.unitary_problem
        self.pdiag, self.pfull = projector_arrays(fp)
        dp = ctypes.POINTER(ctypes.c_double)
        self.desc = CDesc(
            ndim=up.ndim, ntimes=up.ntimes, nparam=nparam, nadd=up.nb_additional_param,
            nerr=len(up.error_sources), n_ops=0, t0=float(up.t0), eps=float(up.eps), eps2=float(up.eps2),
            projector_diag=self.pdiag.ctypes.data_as(dp), n_h0_terms=0, n_target_terms=0,
            max_batch=int(max_batch), reserved=_reserved(GRAPE_DESC_HOST_TABLES, options, scan_waves),
            projector=self.pfull.ctypes.data_as(dp) if self.pfull is not None else None)


# the closure tables themselves: robustgrape_amd/tables.py
from .tables import host_tables, is_hermitian_h0, table_variants  # noqa: E402,F401


def host_interaction_tables(up, x, nparam: int):
    """Closure calls of calculate_interaction_error_operators (src/UnitaryCalculations.jl:180-204)
    for ONE x: H0(k, x_k, x_add) (:196) and Oerr_e = (1/eps) Herror_e(k, x_k, x_add, eps) (:193),
    as the grape_interaction_error_operators_tables layouts H0 (N_t, d, d) and
    Oerr (N_t, ne, d, d), column-major matrices."""
    from .types import split_x
    d, nt = up.ndim, up.ntimes
    errs = up.error_sources
    eps = float(up.eps)
    x_main, x_add, _ = split_x(up, np.asarray(x, np.float64))
    H0 = np.empty((nt, d, d), np.complex128)
    Oerr = np.empty((nt, len(errs), d, d), np.complex128)
    for k in range(nt):
        xk = x_main[:, k]
        H0[k] = np.asarray(up.H0(k + 1, xk.copy(), x_add.copy()), np.complex128).T
        for e, es in enumerate(errs):
            Oerr[k, e] = ((1 / eps) * np.asarray(es.Herror(k + 1, xk.copy(), x_add.copy(), eps), np.complex128)).T
    return H0, Oerr
