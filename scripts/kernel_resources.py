#!/usr/bin/env python3
"""Per-kernel VGPR / spill / LDS / occupancy from hipcc's -Rpass-analysis=kernel-resource-usage remarks.
Usage: kernel_resources.py file.hip [name-filter]   (bf16 instantiations only unless the filter says otherwise)"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-mllvm",
       "-amdgpu-mfma-vgpr-form", "-Rpass-analysis=kernel-resource-usage", "-c", src, "-o", "/tmp/_kr.o"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"remark:\s+(\w[\w /]*?)(?: \[bytes/block\])?: (\S+) \[", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    if flt and flt not in r["name"]:
        continue
    if not flt and "DF16b" not in r["name"]:
        continue
    print(f"{r.get('VGPRs', '?'):>4} vgpr  spill {r.get('VGPRs Spill', '?'):>3}  lds {r.get('LDS Size', '?'):>6}  "
          f"occ {r.get('Occupancy [waves/SIMD]', '?')}  {r['name'][:90]}")
