#!/usr/bin/env python3
"""Group a rocprofv3 --pmc CSV's k_encode dispatches by launch order: tools/ablate.py runs
variants in interleaved rounds of `per` launches each, so dispatch i belongs to variant
(i // per) % nvar.  usage: pmc_by_order.py DIR nvar per"""
import csv
import glob
import sys
from collections import defaultdict

d, nvar, per = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
rows = defaultdict(lambda: defaultdict(float))
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_encode" in r["Kernel_Name"]:
            rows[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
ids = sorted(rows)
acc = defaultdict(lambda: defaultdict(list))
for i, did in enumerate(ids):
    for c, v in rows[did].items():
        acc[(i // per) % nvar][c].append(v)
for k in sorted(acc):
    print(k, {c: round(sum(v) / len(v) / 364560, 1) for c, v in sorted(acc[k].items())}, "(per chunk)")
