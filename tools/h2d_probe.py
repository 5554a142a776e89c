#!/usr/bin/env python3
"""Host -> device copy rate on the GPU box (probe, tool): a raw 4K segment's 1.49 GB from
page-locked host memory, in the worker's batch sizes, to decide whether the end-to-end path
(`bench.py` e2e: page cache -> page-locked batch -> H2D -> encode) is bound by the link.
usage: python3 tools/h2d_probe.py [--mib 96 256 1424]"""
import argparse
import json
import time

import torch


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mib", type=int, nargs="*", default=[96, 256, 1424])
    p.add_argument("--reps", type=int, default=5)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    out = {"device": torch.cuda.get_device_name(0), "rows": []}
    for mib in a.mib:
        n = mib << 20
        h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        h.fill_(7)
        d = torch.empty(n, dtype=torch.uint8, device=dev)
        d.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            d.copy_(h, non_blocking=True)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        out["rows"].append({"MiB": mib, "GBps_median": round(n / ts[len(ts) // 2] / 1e9, 1),
                            "GBps_best": round(n / ts[0] / 1e9, 1)})
        del h, d
    print(json.dumps(out))


if __name__ == "__main__":
    main()
