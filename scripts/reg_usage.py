#!/usr/bin/env python3
"""Per-kernel register / spill / occupancy table of a HIP source for gfx950
(hipcc -Rpass-analysis=kernel-resource-usage).  usage: reg_usage.py FILE.hip [filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/lib/llvm/bin/clang++", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
       "-c", "-x", "hip", src, "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: +([A-Za-z /\[\]]+?): (\S+) \[", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
print("| kernel | VGPRs | AGPRs | VGPR spill | SGPRs | scratch B | waves/SIMD |")
print("|---|---|---|---|---|---|---|")
for r in rows:
    if flt and flt not in r["name"]:
        continue
    print(f"| {r['name']} | {r.get('VGPRs')} | {r.get('AGPRs')} | {r.get('VGPRs Spill')} | "
          f"{r.get('TotalSGPRs')} | {r.get('ScratchSize [bytes/lane]')} | "
          f"{r.get('Occupancy [waves/SIMD]')} |")
