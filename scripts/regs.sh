#!/bin/bash
# Per-kernel register / occupancy summary of a HIP source for gfx950: scripts/regs.sh file.hip
f=${1:?usage: regs.sh file.hip}
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I"$(dirname "$0")/../rvc-maker_amd/csrc" -c "$f" \
  -o /tmp/regs_$$.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  python3 -c '
import re, sys
rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}; rows.append(cur); continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|VGPRs Spill|Occupancy \[waves/SIMD\]|ScratchSize \[bytes/lane\]): (\d+)", line)
    if m and cur is not None: cur[m.group(1).split()[0] + ("S" if "Spill" in m.group(1) else "")] = m.group(2)
for r in rows:
    print(r["name"][:80].ljust(80), "V", r.get("VGPRs"), "A", r.get("AGPRs"), "spill", r.get("VGPRsS"),
          "scratch", r.get("ScratchSize"), "occ", r.get("Occupancy"))'
rm -f /tmp/regs_$$.o
