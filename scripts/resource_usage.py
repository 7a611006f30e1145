#!/usr/bin/env python3
"""Per-kernel resource usage of one HIP source (VGPRs, spills, LDS, occupancy),
from hipcc's -Rpass-analysis=kernel-resource-usage remarks.  Host-side tool.

    python scripts/resource_usage.py cfd-simulations_amd/csrc/jacobi3d_tbr.hip [filter [hipcc flags...]]
"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
extra = sys.argv[3:]
out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                      "-ffp-contract=off", "-c", src, "-o", "/tmp/_ru.o",
                      "-Rpass-analysis=kernel-resource-usage", *extra], capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (?:\s*)(Function Name|VGPRs|VGPRs Spill|LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]|SGPRs): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None:
        cur[k.split(" ")[0] + ("_spill" if "Spill" in k else "")] = v
for r in rows:
    if flt in r["name"]:
        print(f'{r.get("VGPRs","?"):>4} vgpr {r.get("VGPRs_spill","?"):>3} spill {r.get("LDS","?"):>6} lds '
              f'occ {r.get("Occupancy","?")}  {r["name"][:150]}')
