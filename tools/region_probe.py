#!/usr/bin/env python3
"""Timed regions of K steps back to back (probe, tool): bench.py's c2 loop (one segment per
step, library-side merging, queue `enc.depth` deep), each region bracketed by a drain + sync as
bench.py's timed region is, to see whether a region's cost is steady or depends on what ran
just before (the GPU's clock under load; the pipeline's fill and drain).
usage: [K=20] [REGIONS=8] [GAP_MS=0] [TIMING=0|1] [WARMUP=0] python3 tools/region_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from ffmpeg_distributed_amd.encoder import MjpegEncoder
    from ffmpeg_distributed_amd.testsrc import CONTENT
    W, H, DW, DH, Q, SEG, FULL, HUFF, _ = bench.WORKLOADS["c2"]
    K = int(os.environ.get("K", "20"))
    dev = torch.device("cuda", 0)
    nseg = 4
    pool = torch.empty((nseg * SEG, bench.frame_bytes(W, H)), dtype=torch.uint8, device=dev)
    for i in range(0, nseg * SEG, 20):
        pool[i:i + 20] = CONTENT["testsrc"](W, H, i, 20, dev, full_range=FULL)
    torch.cuda.synchronize()
    timing = os.environ.get("TIMING", "0") == "1"  # bench.py's per-kernel HIP events
    enc = MjpegEncoder(0, W, H, DW, DH, full_range=FULL, qscale=Q, max_batch=SEG, huffman=HUFF, timing=timing)
    warm = int(os.environ.get("WARMUP", "0"))  # bench.py: W steps, then a drain, before each region
    depth = enc.depth

    def step(s):
        enc.submit(device_ptr=pool[(s % nseg) * SEG].data_ptr(), nframes=SEG)
        if enc.pending == depth:
            enc.sync()

    def drain():
        while enc.pending:
            enc.sync()
        torch.cuda.synchronize()

    s = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        step(s)
        s += 1
    drain()
    gap = float(os.environ.get("GAP_MS", "0")) / 1e3
    for r in range(int(os.environ.get("REGIONS", "8"))):
        if gap:
            time.sleep(gap)
        for _ in range(warm):
            step(s)
            s += 1
        if warm:
            drain()
        if timing:
            enc.kernel_times(reset=True)
        t = time.perf_counter()
        for _ in range(K):
            step(s)
            s += 1
        drain()
        dt = time.perf_counter() - t
        print(f"region {r}: {K} steps {dt * 1e3:.3f} ms, {dt / K * 1e3:.4f} ms/step, {K * SEG / dt:.0f} fps", flush=True)
    enc.close()


if __name__ == "__main__":
    main()
