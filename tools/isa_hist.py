#!/usr/bin/env python3
"""Static instruction histogram of one kernel from `hipcc --cuda-device-only -S` output.
usage: isa_hist.py FILE.s [kernel-substring] [top-N]"""
import sys
from collections import Counter

path = sys.argv[1]
name = sys.argv[2] if len(sys.argv) > 2 else "k_encode"
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
lines = open(path).read().splitlines()
start = next(i for i, l in enumerate(lines) if l.endswith(":") is False and name in l and "; @" in l)
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
ins = [l.split()[0] for l in lines[start:end] if l.startswith("\t") and l.strip() and
       not l.strip().startswith((".", ";"))]
c = Counter(ins)
cls = Counter()
for k, v in c.items():
    cls["s_" if k.startswith("s_") else "v_" if k.startswith("v_") else "ds_" if k.startswith("ds_")
        else "global/buffer" if k.startswith(("global_", "buffer_")) else "other"] += v
print(f"{name}: {len(ins)} instructions; {dict(cls)}")
for k, v in c.most_common(top):
    print(f"  {k:28s} {v}")
