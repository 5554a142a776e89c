#!/usr/bin/env python3
"""Where the per-segment `gpu:N` process spends a segment (bench.py e2e "per_segment_process").

Runs the dispatcher's per-segment argv (mjg_client -> resident encoder) on one raw 4K segment
`--n` times with MJG_WORKER_TRACE=1 and prints, per segment, the wall time around the client
process, the resident's `mjg-trace:` line (setup / read / submit / sync / fetch / mux / wait
inside worker.run) and the gap between the two (process start, hand-off, close, exit).
Then the same segment through `worker --serve` (-P) for comparison.  Tool, not product.

    python tools/client_latency.py [--workload c2] [--n 6]
"""
from __future__ import annotations

import argparse
import os
import re
import shlex
import sys
import tempfile
import time
from fractions import Fraction

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from ffmpeg_distributed_amd import dispatcher as D, resident  # noqa: E402
from ffmpeg_distributed_amd.testsrc import write_raw_segment  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--n", type=int, default=6)
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args()
    w, h, _, _, _, frames, full, _, _ = bench.WORKLOADS[a.workload]
    fps = Fraction(30) if a.workload == "c1" else Fraction(60)
    args = shlex.split(bench.E2E_ARGS[a.workload])
    d = tempfile.mkdtemp(prefix="mjg_lat_")
    seg = os.path.join(d, "seg.mkv")
    write_raw_segment(seg, w, h, fps, frames, full_range=full)
    os.environ["MJG_WORKER_TRACE"] = "1"
    argv = D.worker_argv(f"gpu:{a.device}", args, resident=True)
    print("argv:", argv[:4], "...", flush=True)
    try:
        for i in range(a.n):
            dst = os.path.join(d, "out.mkv")
            t0 = time.monotonic()
            with open(seg, "rb") as fi, open(dst, "wb") as fo:
                p = D.FFMPEGProc(argv, stdin=fi, stdout=fo)
                rc = p.run()
            wall = time.monotonic() - t0
            tr = [l for l in p.stderr.splitlines() if l.startswith("mjg-trace:")]
            tot = re.search(r"total=([\d.]+) setup=([\d.]+)", tr[0]) if tr else None
            inner = float(tot.group(1)) + float(tot.group(2)) if tot else float("nan")
            print(f"client seg {i}: rc={rc} wall={wall:.4f} run={inner:.4f} gap={wall - inner:.4f}", flush=True)
            for l in tr:
                print("   ", l, flush=True)
            if rc:
                print(p.stderr[-2000:])
        resident.shutdown(D.CLIENT, a.device)
        srv = D.GpuServer(f"gpu:{a.device}")
        try:
            for i in range(a.n):
                t0 = time.monotonic()
                rc = srv.run_task(D.Task(seg, os.path.join(d, "out.mkv"), args))
                print(f"serve seg {i}: rc={rc} wall={time.monotonic() - t0:.4f}", flush=True)
        finally:
            srv.close()
    finally:
        for f in os.listdir(d):
            os.remove(os.path.join(d, f))
        os.rmdir(d)


if __name__ == "__main__":
    main()
