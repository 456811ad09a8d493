"""ctypes wrapper of oracle/build/libgrape_cref.so (test infrastructure / CPU baseline)."""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(os.path.dirname(HERE), "build", "libgrape_cref.so")
_lib = None


def available():
    return os.path.exists(LIB)


def lib():
    global _lib
    if _lib is None:
        if not available():
            from . import build as _b
            _b.build()
        L = ctypes.CDLL(LIB)
        dp = ctypes.POINTER(ctypes.c_double)
        L.grape_cref_fidelity_grad.argtypes = [ctypes.c_void_p, dp, dp, dp, dp, dp]
        L.grape_cref_fidelity_grad.restype = ctypes.c_int
        L.grape_cref_fidelity_grad_batch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, dp, dp, dp, dp, dp]
        L.grape_cref_fidelity_grad_batch.restype = ctypes.c_int
        L.grape_cref_unitary_derivs.argtypes = [ctypes.c_void_p, dp, dp, dp, dp, dp, dp, dp]
        L.grape_cref_unitary_derivs.restype = ctypes.c_int
        L.grape_cref_expm.argtypes = [ctypes.c_int, dp, dp]
        L.grape_cref_exp_calls.restype = ctypes.c_long
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _desc(fp, nparam):
    from robustgrape_amd.operators import DescriptorBuffers
    return DescriptorBuffers(fp, nparam, 1)


def fidelity_grad(fp, x):
    """One evaluation: (F, F_dx (n_x,), F_d2err (ne,), F_d2err_dx (n_x, ne))."""
    up = fp.unitary_problem
    x = np.ascontiguousarray(x, dtype=np.float64)
    nparam = (len(x) - up.nb_additional_param) // up.ntimes
    buf = _desc(fp, nparam)
    ne = len(up.error_sources)
    F = np.zeros(1)
    Fdx = np.zeros(len(x))
    d2 = np.zeros(max(ne, 1))
    d2dx = np.zeros((max(ne, 1), len(x)))
    rc = lib().grape_cref_fidelity_grad(ctypes.addressof(buf.desc), _p(x), _p(F), _p(Fdx), _p(d2), _p(d2dx))
    if rc != 0:
        raise RuntimeError(f"grape_cref_fidelity_grad returned {rc}")
    return float(F[0]), Fdx, d2[:ne], d2dx[:ne].T.copy()


def fidelity_grad_batch(fp, X, nthreads):
    """Independent evaluations of the rows of X on `nthreads` OpenMP threads: (F (nb,), F_dx (nb, n_x))."""
    up = fp.unitary_problem
    X = np.ascontiguousarray(X, dtype=np.float64)
    nb, nx = X.shape
    nparam = (nx - up.nb_additional_param) // up.ntimes
    buf = _desc(fp, nparam)
    ne = len(up.error_sources)
    F = np.zeros(nb)
    Fdx = np.zeros((nb, nx))
    d2 = np.zeros((nb, max(ne, 1)))
    d2dx = np.zeros((nb, max(ne, 1), nx))
    rc = lib().grape_cref_fidelity_grad_batch(ctypes.addressof(buf.desc), nb, int(nthreads), _p(X), _p(F), _p(Fdx),
                                             _p(d2), _p(d2dx))
    if rc != 0:
        raise RuntimeError(f"grape_cref_fidelity_grad_batch returned {rc}")
    return F, Fdx


def unitary_derivs(fp, x):
    up = fp.unitary_problem
    x = np.ascontiguousarray(x, dtype=np.float64)
    n, Nt, na, ne = up.ndim, up.ntimes, up.nb_additional_param, len(up.error_sources)
    nparam = (len(x) - na) // Nt
    buf = _desc(fp, nparam)
    shp = dict(U=(n, n), U_dx=(n, n, nparam, Nt), U_dx_add=(n, n, na), U_derr=(n, n, ne),
               U_derr_dx=(n, n, nparam, Nt, ne), U_derr_dx_add=(n, n, na, ne))
    out = {k: np.zeros(int(np.prod(s)) * 2 or 2) for k, s in shp.items()}
    rc = lib().grape_cref_unitary_derivs(ctypes.addressof(buf.desc), _p(x), *[_p(out[k]) for k in shp])
    if rc != 0:
        raise RuntimeError(f"grape_cref_unitary_derivs returned {rc}")
    res = []
    for k, s in shp.items():
        c = out[k][0::2] + 1j * out[k][1::2]
        res.append(c[:int(np.prod(s))].reshape(s, order="F"))
    return tuple(res)
