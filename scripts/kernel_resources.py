#!/usr/bin/env python3
"""Per-kernel VGPR / spill / occupancy table from `hipcc -Rpass-analysis=kernel-resource-usage`.
Usage: kernel_resources.py <file.hip> [name-filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-Icsrc/kernels", "-c", src,
                    "-o", "/tmp/_kr.o", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
cur = None
rows = {}
for line in r.stderr.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        cur = re.sub(r"\(unsigned.*", "", cur).replace("void (anonymous namespace)::", "")
        rows[cur] = {}
        continue
    m = re.search(r"(VGPRs|AGPRs|VGPRs Spill|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1)] = int(m.group(2))
for k, v in rows.items():
    if flt in k:
        print(f"{k:60s} vgpr {v.get('VGPRs', '?'):>4} agpr {v.get('AGPRs', '?'):>3} spill {v.get('VGPRs Spill', '?'):>3} "
              f"scratch {v.get('ScratchSize [bytes/lane]', '?'):>4} occ {v.get('Occupancy [waves/SIMD]', '?')} "
              f"lds {v.get('LDS Size [bytes/block]', '?')}")
if r.returncode:
    print(r.stderr[-3000:])
