"""Build A/B variants of libgrape.so with extra -D defines into abvar/libgrape_<name>.so.
    python scripts/build_variants.py name=DEF1=1,DEF2=3 name2=DEF=0 ...
(the in-tree library is the "base" variant of scripts/gpu_ab_c2.sh)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robustgrape_amd.build import ROOT, build_library  # noqa: E402

os.makedirs(os.path.join(ROOT, "abvar"), exist_ok=True)
for arg in sys.argv[1:]:
    name, _, defs = arg.partition("=")
    defines = tuple(d for d in defs.split(",") if d)
    build_library(force=True, out=os.path.join(ROOT, "abvar", f"libgrape_{name}.so"), defines=defines)
