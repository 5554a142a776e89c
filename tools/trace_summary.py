#!/usr/bin/env python3
"""Summarise rocprofv3 kernel-trace CSVs of bench.py runs: per kernel the mean duration, and
for k_encode the time from its start to the previous tail kernel's end (overlap)."""
import csv
import sys
from collections import defaultdict

for path in sys.argv[1:]:
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    dur = defaultdict(list)
    last_tail_end = 0
    overlap = []
    gaps = []
    prev_enc_end = None
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mjg::", "")
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        dur[name.split("<")[0]].append((e - s) / 1e3)
        if name.startswith("k_encode"):
            overlap.append(max(0, last_tail_end - s) / 1e3)
            if prev_enc_end is not None:
                gaps.append((s - prev_enc_end) / 1e3)
            prev_enc_end = e
        if name.startswith(("k_write", "k_count_ff", "k_scan", "k_frame_hdr")):
            last_tail_end = max(last_tail_end, e)
    print(path)
    for k, v in dur.items():
        if not k.startswith("k_"):
            continue
        v = v[2:] if len(v) > 4 else v
        print(f"  {k:14s} n={len(v):3d} mean {sum(v) / len(v):9.1f} us  min {min(v):9.1f}")
    print(f"  k_encode start inside the previous tail: mean {sum(overlap) / len(overlap):.1f} us;"
          f" gap between k_encode launches: mean {sum(gaps) / max(1, len(gaps)):.1f} us")
