"""include/grape.h from a plain-C caller (tests/c/abi_check.c, gcc): the struct layout seen by C
equals the ctypes mirror (robustgrape_amd/operators.py) and the Julia shim's isbits structs
(julia/RobustGRAPEMI355X.jl, laid out by the C rules Julia uses for ccall), and on a GPU one
grape_fidelity_grad call from C matches the CPU oracle."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "c", "abi_check.c")
LIBDIR = os.path.join(ROOT, "robustgrape_amd")


def _binary(tmp_path_factory=None):
    out = os.path.join(ROOT, "tests", "c", "abi_check")
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(SRC),
                                                              os.path.getmtime(os.path.join(ROOT, "include", "grape.h"))):
        subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-O1", "-I" + os.path.join(ROOT, "include"), SRC,
                        "-L" + LIBDIR, "-lgrape", "-Wl,-rpath," + LIBDIR, "-o", out], check=True)
    return out


def _layout():
    out = subprocess.run([_binary(), "layout"], check=True, capture_output=True, text=True).stdout
    return {k: int(v) for k, v in (line.split() for line in out.splitlines())}


JULIA_TYPES = {"Int32": (4, 4), "Float64": (8, 8)}


def _julia_layout(struct):
    """Offsets of a Julia isbits struct declared in the shim, by the C layout rules."""
    src = open(os.path.join(ROOT, "julia", "RobustGRAPEMI355X.jl")).read()
    body = re.search(r"struct %s\n(.*?)\nend" % struct, src, re.S).group(1)
    fields = re.findall(r"(\w+)::([\w{},]+)", body)
    off, offs, align_max = 0, {}, 1
    for name, ty in fields:
        if ty.startswith("Ptr{"):
            size, align = 8, 8
        elif ty.startswith("NTuple{"):
            n, el = re.match(r"NTuple\{(\d+),(\w+)\}", ty).groups()
            size, align = int(n) * JULIA_TYPES[el][0], JULIA_TYPES[el][1]
        else:
            size, align = JULIA_TYPES[ty]
        off = (off + align - 1) // align * align
        offs[name] = off
        off += size
        align_max = max(align_max, align)
    return offs, (off + align_max - 1) // align_max * align_max


def test_c_layout_matches_ctypes_and_julia_shim():
    from robustgrape_amd import _capi
    from robustgrape_amd.operators import CDesc, CTerm
    lay = _layout()
    assert lay["abi_version"] == _capi.ABI_VERSION
    for cname, cty, jname in (("grape_term", CTerm, "GrapeTerm"), ("grape_desc", CDesc, "GrapeDesc")):
        assert lay[f"sizeof.{cname}"] == ctypes.sizeof(cty)
        joffs, jsize = _julia_layout(jname)
        assert lay[f"sizeof.{cname}"] == jsize, (cname, jsize)
        for field, _ in cty._fields_:
            off = lay[f"{cname}.{field}"]
            assert off == getattr(cty, field).offset, (cname, field)
            assert off == joffs[field], (cname, field, joffs[field])
    # the device L-BFGS state (robustgrape_amd/optimize.py mirror; not part of the Julia shim)
    from robustgrape_amd.optimize import _CLbfgsState
    cst = _CLbfgsState.get()
    assert lay["sizeof.grape_lbfgs_state"] == ctypes.sizeof(cst)
    for field, _ in cst._fields_:
        if field != "reserved0":
            assert lay[f"grape_lbfgs_state.{field}"] == getattr(cst, field).offset, field


@pytest.mark.gpu
def test_c_caller_fidelity_grad_matches_oracle():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = subprocess.run([_binary(), "gpu"], check=True, capture_output=True, text=True, timeout=120).stdout
    vals = {}
    for line in out.splitlines():
        parts = line.split()
        vals[" ".join(parts[:-1])] = float(parts[-1])
    from oracle import grape_oracle as O
    from robustgrape_amd.types import FidelityRobustGRAPEProblem, UnitaryRobustGRAPEProblem
    X = np.array([[0, 1], [1, 0]], complex)
    Y = np.array([[0, -1j], [1j, 0]])
    Z = np.diag([1.0, -1.0]).astype(complex)
    up = UnitaryRobustGRAPEProblem(t0=1.7, ntimes=4, ndim=2, nb_additional_param=1,
                                   H0=lambda t, x, xa: np.cos(x[0]) * X + np.sin(x[0]) * Y + 0.3 * Z)
    fp = FidelityRobustGRAPEProblem(up, np.eye(2), lambda xa: X * np.exp(1j * xa[0]))
    x = np.array([0.1, 0.7, -0.4, 1.3, 0.25])
    F0, g0, _, _ = O.calculate_fidelity_and_derivatives(fp, x)
    assert abs(vals["F"] - F0) <= 1e-12
    g = np.array([vals[f"F_dx {i}"] for i in range(5)])
    assert np.max(np.abs(g - g0)) <= 1e-6 * np.max(np.abs(g0)) + 1e-8


def test_fault_handler_is_opt_in():
    """loading libgrape installs no SIGSEGV / SIGBUS handler (a Julia host uses SIGSEGV
    itself); grape_install_fault_handler (ABI 11, called by the Python binding) installs it."""
    out = subprocess.run([_binary(), "signals"], check=True, capture_output=True, text=True).stdout
    got = {k: int(v) for k, v in (line.split() for line in out.splitlines())}
    assert got == {"segv_default_at_load": 1, "bus_default_at_load": 1, "installed": 1, "segv_default_after": 0}
