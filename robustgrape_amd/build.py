"""Build libgrape.so (the HIP engine + C ABI) in-tree for gfx950.

    python -m robustgrape_amd.build          # or __graft_entry__.build()

The library lands next to this file so it travels with the repo snapshot to
the GPU box (built .so files are git-ignored but not gpurun-ignored).
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libgrape.so")
OBJ = os.path.join(HERE, "_obj")
ENGINE = os.path.join(CSRC, "grape_engine.hip")
INST = os.path.join(CSRC, "grape_inst.hip")
DENSE = os.path.join(CSRC, "grape_dense.hip")
UNITARY = os.path.join(CSRC, "grape_unitary.hip")
LBFGS = os.path.join(CSRC, "grape_lbfgs.hip")
PROJ = os.path.join(CSRC, "grape_projector.hip")
WALK = os.path.join(CSRC, "grape_walk_inst.hip")
EVAL1 = os.path.join(CSRC, "grape_eval1.hip")
DIMS = list(range(2, 13))  # GRAPE_DIMS in grape_launch.hpp; GRAPE_MAX_SMALL_DIM = 12
SOURCES = [ENGINE, INST, DENSE, UNITARY, LBFGS, PROJ, WALK, EVAL1]
DEPS = SOURCES + [os.path.join(CSRC, f) for f in
                  ("grape_device.hpp", "grape_kernels.hpp", "grape_errpath.hpp", "grape_launch.hpp", "grape_lane.hpp",
                   "grape_walk.hpp", "grape_walk_api.hpp", "grape_eval1_api.hpp",
                   "grape_dense.hpp", "grape_dense_api.hpp", "grape_unitary_api.hpp",
                   "grape_projector_api.hpp")] + \
    [os.path.join(ROOT, "include", "grape.h")]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("GRAPE_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
         # no implicit FMA contraction: the reference (Julia) never fuses; the
         # kernels use explicit fma() where fusion is intended (complex MACs)
         "-ffp-contract=off",
         "-I" + os.path.join(ROOT, "include"), "-I" + CSRC]


def source_id(defines=()) -> str:
    """Content hash of every source the library is built from (DEPS), the compiler flags (the common
    ones and every unit's own) and the variant's -D defines: the library embeds it (grape_build_id())
    and _capi.lib() refuses a library whose id differs from the sources next to it, so a test or bench
    run names the sources -- and the A/B variant (scripts/build_variants.py) -- it ran."""
    h = hashlib.sha256()
    for d in sorted(DEPS):
        h.update(os.path.relpath(d, ROOT).encode() + b"\0")
        with open(d, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    h.update(" ".join(f for f in FLAGS if not f.startswith("-I")).encode() + b"\0")
    for src, extra, _ in _units(())[1]:
        h.update(os.path.basename(src).encode() + b":" + " ".join(extra).encode() + b"\0")
    h.update(("defines:" + " ".join(sorted(defines))).encode())
    return h.hexdigest()[:16]


ID_FILE = LIB + ".id"  # the id the in-tree library was linked with (read without loading it)


def read_id_file(lib_path):
    """(build id, defines) recorded next to a built library (`<lib>.id`: the id, then the variant's
    -D defines on the second line), or (None, ()) when there is no record."""
    try:
        with open(lib_path + ".id") as fh:
            lines = fh.read().splitlines()
    except OSError:
        return None, ()
    sid = lines[0].strip() if lines else None
    defines = tuple(lines[1].split()) if len(lines) > 1 else ()
    return sid, defines


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    sid, defines = read_id_file(LIB)
    return defines != () or sid != source_id()


def _units(defines):
    """(source, extra -D flags, object path): the C ABI + one object per dimension."""
    tag = "_".join(d.replace("=", "") for d in defines)
    sub = os.path.join(OBJ, tag or "default")
    units = [(DENSE, [], os.path.join(sub, "grape_dense.o")), (ENGINE, [], os.path.join(sub, "grape_engine.o")),
             (UNITARY, [], os.path.join(sub, "grape_unitary.o")), (LBFGS, [], os.path.join(sub, "grape_lbfgs.o")),
             (PROJ, [], os.path.join(sub, "grape_projector.o")),
             # the chunk walks: no MachineLICM (grape_walk.hpp explains the register budget)
             (WALK, ["-mllvm", "-disable-machine-licm"], os.path.join(sub, "grape_walk.o")),
             # the one-workgroup-per-evaluation kernel (latency-bound calls): the walks' arithmetic
             (EVAL1, ["-mllvm", "-disable-machine-licm"], os.path.join(sub, "grape_eval1.o"))]
    units += [(INST, [f"-DGRAPE_INST_DIM={d}"], os.path.join(sub, f"grape_inst_d{d}.o")) for d in DIMS]
    return sub, units


def build_library(force: bool = False, verbose: bool = True, out: str = LIB, defines=()) -> str:
    """Build libgrape.so (or a variant with extra -D defines into `out`, for tuning runs).

    Every translation unit is compiled in parallel (one per dimension D: the
    kernels are templates on D), then linked into one shared library."""
    if out == LIB and not defines and not force and not needs_build():
        return LIB
    sub, units = _units(defines)
    os.makedirs(sub, exist_ok=True)
    if verbose:
        print("[robustgrape_amd] building", os.path.relpath(out, ROOT), *defines,
              f"({len(units)} translation units)", flush=True)
    sid = source_id(defines)
    dflags = [f"-D{d}" for d in defines]
    jobs = max(1, min(len(units), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16))
    pending = list(units)
    running = []
    failed = []
    while pending or running:
        while pending and len(running) < jobs:
            src, extra, obj = pending.pop(0)
            cmd = [HIPCC] + FLAGS + dflags + extra + ["-c", src, "-o", obj]
            if src == ENGINE:
                cmd.insert(1, f'-DGRAPE_BUILD_ID="{sid}"')
            running.append((subprocess.Popen(cmd), obj))
        proc, obj = running.pop(0)
        if proc.wait() != 0:
            failed.append(obj)
    if failed:
        raise RuntimeError("hipcc failed for " + ", ".join(os.path.basename(f) for f in failed))
    tmp = out + ".tmp"
    subprocess.run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}"] + [u[2] for u in units] + ["-o", tmp],
                   check=True)
    os.replace(tmp, out)
    with open(out + ".id", "w") as fh:
        fh.write(sid + "\n" + " ".join(defines) + "\n")
    return out


if __name__ == "__main__":
    build_library(force="--force" in sys.argv)
