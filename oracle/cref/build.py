"""Build the reference-faithful C++ restatement into oracle/build/libgrape_cref.so.

Test infrastructure / CPU baseline only (see grape_cref.cpp).  Portable x86-64-v3
code (the GPU box's host CPU is not this container's), no FMA contraction (Julia
does not fuse), -O3.
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(os.path.dirname(HERE), "build", "libgrape_cref.so")
SRC = os.path.join(HERE, "grape_cref.cpp")


def build(force=False):
    hdr = os.path.join(ROOT, "include", "grape.h")
    if not force and os.path.exists(OUT) and os.path.getmtime(OUT) > max(os.path.getmtime(SRC), os.path.getmtime(hdr)):
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cmd = ["g++", "-O3", "-march=x86-64-v3", "-ffp-contract=off", "-std=c++17", "-fPIC", "-shared", "-fopenmp",
           "-I" + os.path.join(ROOT, "include"), SRC, "-o", f"{OUT}.{os.getpid()}.tmp"]
    subprocess.run(cmd, check=True)
    os.replace(f"{OUT}.{os.getpid()}.tmp", OUT)  # per-process temporary: parallel test workers may race
    return OUT


if __name__ == "__main__":
    print(build())
