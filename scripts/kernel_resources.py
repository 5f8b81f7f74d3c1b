#!/usr/bin/env python3
"""Per-kernel resources from `make asm` output (build/kernels.s): VGPRs, AGPRs, SGPRs, LDS, scratch."""
import re
import subprocess
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "build/scan_sum.s"
pat = sys.argv[2] if len(sys.argv) > 2 else "scan_tiles"
cur = None
rows = []
for line in open(path):
    m = re.match(r"\s*\.amdhsa_kernel (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        continue
    if cur is None:
        continue
    m = re.match(r"\s*\.amdhsa_(next_free_vgpr|next_free_sgpr|accum_offset|group_segment_fixed_size|"
                 r"private_segment_fixed_size)\s+(\d+)", line)
    if m:
        cur[m.group(1)] = int(m.group(2))
    if re.match(r"\s*\.end_amdhsa_kernel", line):
        rows.append(cur)
        cur = None
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
for r, n in zip(rows, names):
    if pat in n:
        print(f"{n[:60]:60s} vgpr {r.get('next_free_vgpr')} sgpr {r.get('next_free_sgpr')} "
              f"lds {r.get('group_segment_fixed_size')} scratch {r.get('private_segment_fixed_size')}")
