#!/usr/bin/env python3
"""Per-step timeline of a bench.py run from a rocprofv3 kernel-trace CSV: for each k_encode
dispatch s, its start S, end E, and its stuffing tail's end T (k_write, the last kernel of
the chain that follows it).  Reports the step period S[s+1] - S[s], k_encode's span E - S,
how long after the previous-but-one submit's tail ended the next k_encode started
(S[s+1] - T[s-1]: the host's sync -> submit latency when the two-slot queue is full), and the
time from E[s] to S[s+1] (negative: the next k_encode started inside this one's drain).
usage: timeline.py trace.csv"""
import csv
import statistics as st
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
enc, tails = [], []
for r in rows:
    name = r["Kernel_Name"]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if "k_encode" in name:
        enc.append([s, e])
    elif "k_write" in name:
        tails.append(e)
n = min(len(enc), len(tails))
enc, tails = enc[:n], tails[:n]
per, span, lat, ovl, tail_after = [], [], [], [], []
for i in range(2, n - 1):
    per.append((enc[i + 1][0] - enc[i][0]) / 1e3)
    span.append((enc[i][1] - enc[i][0]) / 1e3)
    lat.append((enc[i + 1][0] - tails[i - 1]) / 1e3)
    ovl.append((enc[i + 1][0] - enc[i][1]) / 1e3)
    tail_after.append((tails[i] - enc[i][1]) / 1e3)
f = lambda v: f"median {st.median(v):8.1f}  min {min(v):8.1f}  max {max(v):8.1f} us"
print(f"{sys.argv[1]}: {n} k_encode dispatches")
print("  step period S[s+1]-S[s]        ", f(per))
print("  k_encode span E-S              ", f(span))
print("  tail end after its k_encode     ", f(tail_after))
print("  next k_encode start - E[s]      ", f(ovl))
print("  next k_encode start - T[s-1]    ", f(lat))
