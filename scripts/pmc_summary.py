"""Summarise rocprofv3 --pmc pass directories: per kernel, the mean of every counter per
dispatch, plus per-wave instruction mixes and the HBM bytes per launch.

    python scripts/pmc_summary.py gpurun_out/pmc_p1 gpurun_out/pmc_p2 ... [--json out.json]

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md (HBM/rocprofv3 section): on gfx950
FETCH_SIZE (KiB) reports half of the bytes of wide coalesced reads, so read bytes are
2 * FETCH_SIZE * 1024; WRITE_SIZE (KiB) is taken as is.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    for pre in ("void ", "grape::"):
        n = n.replace(pre, "")
    return n


def load(dirs):
    # (kernel, counter) -> list of per-dispatch values (summed over the dispatch's rows)
    per = defaultdict(lambda: defaultdict(float))
    for d in dirs:
        files = [d] if os.path.isfile(d) else (glob.glob(os.path.join(d, "**", "*counter_collection.csv"),
                                                         recursive=True) or glob.glob(os.path.join(d, "*.csv")))
        for f in files:
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    key = (short(row["Kernel_Name"]), row["Counter_Name"], row["Dispatch_Id"], f)
                    per[key[:2]][key[2:]] += float(row["Counter_Value"])
    out = defaultdict(dict)
    for (k, c), disp in per.items():
        vals = list(disp.values())
        out[k][c] = sum(vals) / len(vals)
        out[k]["_dispatches_" + c] = len(vals)
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    if "--batch" in sys.argv:
        args.remove(sys.argv[sys.argv.index("--batch") + 1])
    js = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    batch = int(sys.argv[sys.argv.index("--batch") + 1]) if "--batch" in sys.argv else None
    if js in args:
        args.remove(js)
    data = load(args)
    summary = {}
    for k, cs in sorted(data.items()):
        if k.startswith("__amd"):
            continue
        waves = cs.get("SQ_WAVES", 0.0)
        row = {c: v for c, v in cs.items() if not c.startswith("_")}
        row["dispatches"] = max((v for c, v in cs.items() if c.startswith("_dispatches_")), default=0)
        if waves:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64",
                      "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
                if c in cs:
                    row[c + "_per_wave"] = cs[c] / waves
        if "FETCH_SIZE" in cs or "WRITE_SIZE" in cs:
            row["hbm_bytes_per_launch"] = 2 * cs.get("FETCH_SIZE", 0.0) * 1024 + cs.get("WRITE_SIZE", 0.0) * 1024
        summary[k] = row
        print(k)
        for c, v in sorted(row.items()):
            print(f"    {c:36s} {v:16.1f}")
    if js:
        with open(js, "w") as fh:
            json.dump({"batch": batch, "kernels": summary}, fh, indent=1)


if __name__ == "__main__":
    main()
