#!/usr/bin/env python3
"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output (one line per kernel)."""
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "/tmp/lbk8s_resource.txt"
cur, rows = None, []
for line in open(path):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    if cur is None:
        continue
    for key, pat in (("vgpr", r" VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("sgpr", r"TotalSGPRs: (\d+)"),
                     ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"), ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"),
                     ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
        m = re.search(pat, line)
        if m:
            cur[key] = int(m.group(1))
for r in rows:
    print(f"{r['name'][:60]:60s} vgpr={r.get('vgpr')} sgpr={r.get('sgpr')} scratch={r.get('scratch')} "
          f"lds={r.get('lds')} occ={r.get('occ')}")
