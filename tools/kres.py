#!/usr/bin/env python3
"""Per-kernel VGPR / SGPR / scratch / LDS from the device assembly's metadata
(make -C clusteringsegmentation-1_amd asm).  Development tool."""
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "clusteringsegmentation-1_amd/build/dq_kernels-gfx950.s"
txt = open(path).read()
meta = txt[txt.index("amdhsa.kernels:"):]
blocks = re.split(r"\n  - ", meta)[1:]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for b in blocks:
    f = dict(re.findall(r"\.(name|vgpr_count|sgpr_count|private_segment_fixed_size|group_segment_fixed_size|agpr_count):\s+(\S+)", b))
    if "name" not in f or pat not in f["name"]:
        continue
    print("%-60s vgpr %4s agpr %3s sgpr %4s scratch %4s lds %6s" % (f["name"][:60], f.get("vgpr_count"), f.get("agpr_count"),
          f.get("sgpr_count"), f.get("private_segment_fixed_size"), f.get("group_segment_fixed_size")))
