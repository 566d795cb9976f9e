#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy table of one HIP source (tuning aid): compiles the
device side with -Rpass-analysis=kernel-resource-usage and prints the kernels whose demangled-ish
name matches the optional filter.
    python3 tools/kernel_resources.py plonk.c_amd/csrc/ntt_wave.hip [substring] [extra hipcc flags...]"""
import re
import subprocess
import sys

src = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "--cuda-device-only",
       "-Rpass-analysis=kernel-resource-usage", "-c", src, "-o", "/dev/null"] + sys.argv[3:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|VGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur["VGPRs Spill" if k == "VGPRs Spill" else k.split()[0]] = v
for r in rows:
    if filt in r["name"]:
        print("%-90s vgpr %4s spill %4s scratch %4s occ %2s lds %6s" % (r["name"][:90], r.get("VGPRs"), r.get("VGPRs Spill"), r.get("ScratchSize"),
                                                               r.get("Occupancy"), r.get("LDS")))
