"""Register / scratch / occupancy of every kernel of one translation unit (hipcc's
-Rpass-analysis=kernel-resource-usage remarks), one line per kernel.
    python scripts/kernel_resources.py robustgrape_amd/csrc/grape_walk_inst.hip [name-filter]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off",
       "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "robustgrape_amd", "csrc"),
       "-Rpass-analysis=kernel-resource-usage", "-c", src, "-o", "/dev/null"]
if "walk" in src:
    cmd[1:1] = ["-mllvm", "-disable-machine-licm"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, rows = None, []
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for key in ("VGPRs", "AGPRs", "ScratchSize \\[bytes/lane\\]", "Occupancy \\[waves/SIMD\\]"):
        m = re.search(key + r": (\d+)", line)
        if m and cur is not None:
            cur[key.split()[0].split("\\")[0]] = int(m.group(1))
for r in rows:
    if filt in r["name"]:
        dm = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
        dm = re.sub(r"\(grape::DevProblem.*", "", dm)
        print(f"{r.get('VGPRs', '?'):>4} v {r.get('AGPRs', 0):>4} a {r.get('ScratchSize', 0):>5} B scratch "
              f"{r.get('Occupancy', '?'):>2} w  {dm}")
