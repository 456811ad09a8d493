"""Build libgrape.so (the HIP engine + C ABI) in-tree for gfx950.

    python -m robustgrape_amd.build          # or __graft_entry__.build()

The library lands next to this file so it travels with the repo snapshot to
the GPU box (built .so files are git-ignored but not gpurun-ignored).
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libgrape.so")
SOURCES = [os.path.join(CSRC, "grape_engine.hip")]
DEPS = SOURCES + [os.path.join(CSRC, f) for f in ("grape_device.hpp", "grape_kernels.hpp", "grape_errpath.hpp")] + \
    [os.path.join(ROOT, "include", "grape.h")]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("GRAPE_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", f"--offload-arch={ARCH}",
         # no implicit FMA contraction: the reference (Julia) never fuses; the
         # kernels use explicit fma() where fusion is intended (complex MACs)
         "-ffp-contract=off",
         "-I" + os.path.join(ROOT, "include"), "-I" + CSRC]


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(d) > t for d in DEPS if os.path.exists(d))


def build_library(force: bool = False, verbose: bool = True, out: str = LIB, defines=()) -> str:
    """Build libgrape.so (or a variant with extra -D defines into `out`, for tuning runs)."""
    if out == LIB and not defines and not force and not needs_build():
        return LIB
    tmp = out + ".tmp"
    cmd = [HIPCC] + FLAGS + [f"-D{d}" for d in defines] + SOURCES + ["-o", tmp]
    if verbose:
        print("[robustgrape_amd] building", os.path.relpath(out, ROOT), *defines, flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    build_library(force="--force" in sys.argv)
