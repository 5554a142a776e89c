#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs: per kernel, mean counter value per dispatch."""
import csv
import glob
import json
import sys
from collections import defaultdict


def load(dirs):
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            per = defaultdict(float)
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"].split("(")[0]
                per[(name, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            for (name, _, cn), v in per.items():
                acc[name][cn].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def load_totals(dirs):
    """Per kernel: {counter: sum over all dispatches}, plus "dispatches"."""
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"].split("(")[0]
                acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[name].add((f, r["Dispatch_Id"]))
    return {k: dict(cs, dispatches=len(disp[k])) for k, cs in acc.items()}


if __name__ == "__main__":
    res = load(sys.argv[1:])
    print(json.dumps(res, indent=1))
