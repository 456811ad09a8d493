"""Summarise the dense engine's MFMA / LDS PMC passes (scripts/gpu_pmc_dense.sh) per kernel:
counters summed over dispatches and the derived MFMA-pipe occupancy
    mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (kernel cycles x 1024 SIMDs)
with kernel cycles = GRBM_GUI_ACTIVE / 8 (the counter sums the eight XCDs' GRBMs; cross-checked
against the kernel trace's durations at the measured clock).
    python scripts/pmc_dense_summary.py gpurun_out/TAG_p1 gpurun_out/TAG_p2 > pmc_mfma_lds.txt"""
import collections
import csv
import re
import sys

SIMDS = 1024
# per pass: counters summed over the dispatches; a counter collected in several passes is averaged over them
per_pass = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
dur = collections.defaultdict(float)
for d in sys.argv[1:]:
    for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        if not m:
            continue
        per_pass[m.group(1)][r["Counter_Name"]][d] += float(r["Counter_Value"])
    if d.endswith("1"):
        for r in csv.DictReader(open(d + "/run_kernel_trace.csv")):
            m = re.search(r"(k_\w+)", r["Kernel_Name"])
            if m:
                dur[m.group(1)] += (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-9
res = {k: {c: sum(v.values()) / len(v) for c, v in cs.items()} for k, cs in per_pass.items()}
for k in sorted(res):
    v = res[k]
    print(k)
    for c in sorted(v):
        print(f"    {c:34s} {v[c]:16.4g}")
    if v.get("GRBM_GUI_ACTIVE"):
        cyc = v["GRBM_GUI_ACTIVE"] / 8
        print(f"    {'kernel_cycles (GRBM/8)':34s} {cyc:16.4g}")
        if dur.get(k):
            print(f"    {'clock from trace (GHz)':34s} {cyc / dur[k] / 1e9:16.3f}")
        if v.get("SQ_VALU_MFMA_BUSY_CYCLES"):
            print(f"    {'mfma_busy (of SIMD cycles)':34s} {v['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * SIMDS):16.3f}")
        if v.get("SQ_INSTS_MFMA") and v.get("SQ_WAVES"):
            print(f"    {'mfma_per_wave':34s} {v['SQ_INSTS_MFMA'] / v['SQ_WAVES']:16.1f}")
        if v.get("SQ_LDS_IDX_ACTIVE"):
            print(f"    {'lds_bank_conflict / lds_idx_active':34s} {v.get('SQ_LDS_BANK_CONFLICT', 0.0) / v['SQ_LDS_IDX_ACTIVE']:16.3f}")
        if v.get("SQ_INSTS_VALU") and v.get("SQ_WAVES"):
            print(f"    {'valu_per_wave':34s} {v['SQ_INSTS_VALU'] / v['SQ_WAVES']:16.1f}")
