"""Instruction mix and executed FP64 work per kernel from rocprofv3 --pmc passes (scripts/gpu_pmc.sh).

    python scripts/pmc_mix.py OUT_PREFIX [--json FILE] [--batch EVALUATIONS_PER_DEVICE_PASS]

reads every OUT_PREFIX_p*/run_counter_collection.csv and, per kernel (template arguments kept,
parameter lists dropped), averages each counter over the kernel's dispatches.  SQ_INSTS_VALU_*_F64
count wave-level instructions, so the executed FP64 FLOP of one dispatch are
64 lanes x (2 FMA + MUL + ADD) (transcendentals not counted).  The bench reads the JSON
(profiles/pmc_mix_latest.json) for the roofline kernel's executed rate beside the algorithmic one."""
import csv
import glob
import json
import sys
from collections import defaultdict


def kname(n):
    n = n.strip('"')
    if n.startswith("void "):
        n = n[5:]
    depth, out = 0, []
    for ch in n:  # drop the parameter list, keep template arguments
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            break
        out.append(ch)
    return "".join(out).replace("grape::", "").strip()


def main(prefix, out_json=None, batch=None):
    vals = defaultdict(lambda: defaultdict(list))
    disp = defaultdict(set)  # dispatches per kernel in the first pass (the bench's timed steps + warm-up)
    files = sorted(glob.glob(prefix + "_p*/run_counter_collection.csv"))
    for fi, f in enumerate(files):
        for r in csv.DictReader(open(f)):
            vals[kname(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if fi == 0:
                disp[kname(r["Kernel_Name"])].add(r["Dispatch_Id"])
    res = {}
    for k, cs in vals.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        row = dict(m)
        row["dispatches"] = len(disp.get(k, ()))
        fma, mul, add = (m.get("SQ_INSTS_VALU_%s_F64" % t) for t in ("FMA", "MUL", "ADD"))
        if fma is not None and mul is not None and add is not None:
            row["fp64_flop_per_dispatch"] = 64.0 * (2.0 * fma + mul + add)
        res[k] = row
    for k in sorted(res, key=lambda k: -res[k].get("fp64_flop_per_dispatch", 0.0))[:12]:
        r = res[k]
        print(f"{k[:60]:60s} waves {r.get('SQ_WAVES', 0):10.0f} VALU {r.get('SQ_INSTS_VALU', 0):14.0f} "
              f"FP64 FLOP/dispatch {r.get('fp64_flop_per_dispatch', 0):.4g}")
    if out_json:
        import os
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        try:  # the library the profiled bench ran (robustgrape_amd/build.py writes libgrape.so.id)
            build_id = open(os.path.join(root, "robustgrape_amd", "libgrape.so.id")).read().split()[0]
        except (OSError, IndexError):
            build_id = None
        json.dump({"batch": batch, "build_id": build_id, "kernels": res,
                   "note": "per-dispatch means of rocprofv3 --pmc counters (scripts/pmc_mix.py)"},
                  open(out_json, "w"), indent=1)


if __name__ == "__main__":
    args = sys.argv[1:]
    opt = {}
    for flag in ("--json", "--batch"):
        if flag in args:
            i = args.index(flag)
            opt[flag] = args[i + 1]
            del args[i:i + 2]
    main(args[0], opt.get("--json"), int(opt["--batch"]) if "--batch" in opt else None)
