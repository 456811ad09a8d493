"""ctypes binding of libgrape.so (include/grape.h).

Loading fails loudly: there is no CPU fallback for the product path.
"""
from __future__ import annotations

import ctypes
import os

from .operators import CDesc

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GRAPE_LIB") or os.path.join(HERE, "libgrape.so")

GRAPE_OK = 0
STATUS_NAMES = {-1: "GRAPE_ERR_INVALID", -2: "GRAPE_ERR_UNSUPPORTED", -3: "GRAPE_ERR_ALLOC",
                -4: "GRAPE_ERR_HIP", -5: "GRAPE_ERR_SINGULAR", -6: "GRAPE_ERR_NO_DEVICE"}

# every symbol include/grape.h declares
EXPORTED = ["grape_abi_version", "grape_build_id", "grape_last_error", "grape_install_fault_handler", "grape_device_count", "grape_plan_create",
            "grape_plan_destroy", "grape_plan_stream", "grape_plan_set_stream", "grape_fidelity_grad",
            "grape_fidelity_grad_device_async", "grape_plan_synchronize", "grape_unitary_derivs",
            "grape_expm_batch", "grape_plan_set_profiling", "grape_plan_kernel_times",
            "grape_interaction_error_operators", "grape_interaction_error_operators_device",
            "grape_expectation_values", "grape_fidelity_grad_tables",
            "grape_lbfgs_direction", "grape_unitary_derivs_tables", "grape_interaction_error_operators_tables",
            "grape_expectation_values_tables", "grape_plan_sectors", "grape_lbfgs_ls_init", "grape_lbfgs_ls_begin",
            "grape_lbfgs_ls_end", "grape_lbfgs_step", "grape_robust_cost", "grape_slice_forward",
            "grape_slice_gradient", "grape_symmetry_basis", "grape_plan_sector_info", "grape_lbfgs_async_advance",
            "grape_slice_forward_device", "grape_slice_gradient_device", "grape_plan_gauge_info", "grape_plan_eval1"]
KERNEL_NAMES = ["k_expm", "k_expm_high", "k_scan", "k_grad/k_err_local", "k_reduce_add", "k_err_scan", "k_err_grad",
                "k_expm_grad", "k_grad_high", "k_dexp", "k_dscan", "k_dcarry", "k_dmc", "k_dgrad",
                "k_walk_fwd", "k_walk_grad", "k_eval1"]
ABI_VERSION = 11  # GRAPE_ABI_VERSION in include/grape.h


class GrapeError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{STATUS_NAMES.get(code, code)}: {msg}")
        self.code = code


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run `python -m robustgrape_amd.build` "
                              "(the GPU path has no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH)
        dp = ctypes.POINTER(ctypes.c_double)
        vp = ctypes.c_void_p
        L.grape_abi_version.restype = ctypes.c_int
        L.grape_build_id.restype = ctypes.c_char_p
        L.grape_last_error.restype = ctypes.c_char_p
        L.grape_install_fault_handler.restype = ctypes.c_int
        L.grape_device_count.restype = ctypes.c_int
        L.grape_plan_create.argtypes = [ctypes.POINTER(CDesc), ctypes.c_int, ctypes.POINTER(vp)]
        L.grape_plan_create.restype = ctypes.c_int
        L.grape_plan_destroy.argtypes = [vp]
        L.grape_plan_destroy.restype = None
        L.grape_plan_stream.argtypes = [vp]
        L.grape_plan_stream.restype = vp
        L.grape_plan_set_stream.argtypes = [vp, vp]
        L.grape_plan_set_stream.restype = ctypes.c_int
        L.grape_fidelity_grad.argtypes = [vp, ctypes.c_int, dp, dp, dp, dp, dp]
        L.grape_fidelity_grad.restype = ctypes.c_int
        L.grape_fidelity_grad_device_async.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, vp]
        L.grape_fidelity_grad_device_async.restype = ctypes.c_int
        L.grape_fidelity_grad_tables.argtypes = [vp, ctypes.c_int, dp, dp, dp, dp, dp, dp, dp]
        L.grape_fidelity_grad_tables.restype = ctypes.c_int
        L.grape_lbfgs_direction.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int] + [vp] * 9
        L.grape_lbfgs_direction.restype = ctypes.c_int
        for name in ("grape_lbfgs_ls_init", "grape_lbfgs_ls_begin", "grape_lbfgs_step"):
            getattr(L, name).argtypes = [vp, vp]
            getattr(L, name).restype = ctypes.c_int
        L.grape_lbfgs_ls_end.argtypes = [vp, ctypes.c_int, vp, vp, vp]
        L.grape_lbfgs_ls_end.restype = ctypes.c_int
        L.grape_lbfgs_async_advance.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, vp]
        L.grape_lbfgs_async_advance.restype = ctypes.c_int
        for name in ("grape_slice_forward_device", "grape_slice_gradient_device"):
            getattr(L, name).argtypes = [vp, vp, vp]
            getattr(L, name).restype = ctypes.c_int
        L.grape_robust_cost.argtypes = [ctypes.c_int] * 5 + [vp] * 12
        L.grape_robust_cost.restype = ctypes.c_int
        L.grape_slice_forward.argtypes = [vp, dp, dp]
        L.grape_slice_forward.restype = ctypes.c_int
        L.grape_slice_gradient.argtypes = [vp, dp, dp]
        L.grape_slice_gradient.restype = ctypes.c_int
        L.grape_plan_synchronize.argtypes = [vp]
        L.grape_plan_synchronize.restype = ctypes.c_int
        L.grape_unitary_derivs.argtypes = [vp, dp, dp, dp, dp, dp, dp, dp]
        L.grape_unitary_derivs.restype = ctypes.c_int
        L.grape_expm_batch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, dp, dp,
                                       ctypes.POINTER(ctypes.c_int)]
        L.grape_expm_batch.restype = ctypes.c_int
        L.grape_interaction_error_operators.argtypes = [vp, dp, dp]
        L.grape_interaction_error_operators.restype = ctypes.c_int
        L.grape_interaction_error_operators_device.argtypes = [vp, dp, vp]
        L.grape_interaction_error_operators_device.restype = ctypes.c_int
        L.grape_expectation_values.argtypes = [vp, dp, dp]
        L.grape_expectation_values.restype = ctypes.c_int
        L.grape_unitary_derivs_tables.argtypes = [vp, dp, dp, dp, dp, dp, dp, dp, dp]
        L.grape_unitary_derivs_tables.restype = ctypes.c_int
        L.grape_interaction_error_operators_tables.argtypes = [vp, dp, dp, dp, vp, ctypes.c_int]
        L.grape_interaction_error_operators_tables.restype = ctypes.c_int
        L.grape_expectation_values_tables.argtypes = [vp, dp, dp, dp, dp]
        L.grape_expectation_values_tables.restype = ctypes.c_int
        L.grape_plan_set_profiling.argtypes = [vp, ctypes.c_int]
        L.grape_plan_set_profiling.restype = ctypes.c_int
        L.grape_plan_kernel_times.argtypes = [vp, dp, ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]
        L.grape_plan_kernel_times.restype = ctypes.c_int
        L.grape_plan_sectors.argtypes = [vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), ctypes.c_int]
        L.grape_plan_sectors.restype = ctypes.c_int
        L.grape_plan_sector_info.argtypes = [vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), ctypes.c_int]
        L.grape_plan_sector_info.restype = ctypes.c_int
        L.grape_plan_gauge_info.argtypes = [vp, ctypes.POINTER(ctypes.c_int), ctypes.c_int]
        L.grape_plan_gauge_info.restype = ctypes.c_int
        L.grape_plan_eval1.argtypes = [vp]
        L.grape_plan_eval1.restype = ctypes.c_int
        L.grape_symmetry_basis.argtypes = [ctypes.POINTER(CDesc), dp, ctypes.POINTER(ctypes.c_int)]
        L.grape_symmetry_basis.restype = ctypes.c_int
        if L.grape_abi_version() != ABI_VERSION:
            raise ImportError("libgrape.so ABI version mismatch")
        # provenance: the library must have been built from the csrc/ next to it (content hash of the
        # sources, flags and -- for an A/B variant loaded through GRAPE_LIB -- its recorded defines)
        from .build import read_id_file, source_id
        _, defines = read_id_file(LIB_PATH)
        got, want = L.grape_build_id().decode(), source_id(defines)
        if got != want:
            raise ImportError(f"{LIB_PATH} was built from other sources (build id {got}, csrc/ hashes to {want}): "
                              "rebuild with `python -m robustgrape_amd.build`")
        if os.environ.get("GRAPE_NO_SIGNAL_HANDLER", "0") != "1":
            L.grape_install_fault_handler()  # native frames of a fault inside libgrape (opt-in, ABI 11)
        _lib = L
    return _lib


def build_id() -> str:
    """Source hash the loaded library was built from (robustgrape_amd/build.py source_id)."""
    return lib().grape_build_id().decode()


def build_defines():
    """The -D defines of the loaded library's variant (empty for the in-tree default build)."""
    from .build import read_id_file
    return read_id_file(LIB_PATH)[1]


def check(code):
    if code != GRAPE_OK:
        raise GrapeError(code, lib().grape_last_error().decode())


def dptr(a):
    """double* of a C-contiguous float64 (or complex128) numpy array (None -> NULL)."""
    if a is None:
        return None
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
