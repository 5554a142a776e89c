#!/usr/bin/env python3
"""k_encode's per-launch fixed cost (its drain and launch ramp) from synced launches of 60 /
120 / 240 / 480 4K frames: T(n) = a + b n, after a 1 s prewarm, sizes interleaved over ROUNDS.
usage (GPU box): [WL=c2] [CONTENT=testsrc] python3 tools/drain_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import bench
    from ffmpeg_distributed_amd.encoder import MjpegEncoder
    from ffmpeg_distributed_amd.testsrc import CONTENT
    W, H, DW, DH, Q, N, FULL, HUFF, _ = bench.WORKLOADS[os.environ.get("WL", "c2")]
    content = os.environ.get("CONTENT", "testsrc")
    dev = torch.device("cuda", 0)
    nmax = 480
    pool = torch.empty((nmax, W * H + 2 * ((W + 1) // 2) * ((H + 1) // 2)), dtype=torch.uint8, device=dev)
    for i in range(0, nmax, 20):
        pool[i:i + 20] = CONTENT[content](W, H, i % 120, 20, dev, full_range=FULL)
    torch.cuda.synchronize()
    enc = MjpegEncoder(0, W, H, DW, DH, full_range=FULL, qscale=Q, max_batch=nmax, timing=True, huffman=HUFF)
    import time
    ns = [60, 120, 240, 480]
    # prewarm: the GPU leaves its idle clocks only after ~0.3 s of load (bench.py --prewarm-ms)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < float(os.environ.get("PREWARM_S", "1.0")):
        enc.submit(device_ptr=pool.data_ptr(), nframes=120)
        enc.sync()
    res = {n: [] for n in ns}
    for rnd in range(int(os.environ.get("ROUNDS", "3"))):  # sizes interleaved, not one block each
        for n in ns:
            enc.kernel_times(reset=True)
            for _ in range(5):
                enc.submit(device_ptr=pool.data_ptr(), nframes=n)
                enc.sync()
            kt, nl = enc.kernel_times()
            res[n].append(kt["encode"])
    ts = []
    for n in ns:
        t = sorted(res[n])[len(res[n]) // 2]
        ts.append(t)
        print(f"{content} n={n}: k_encode median {t:.4f} ms ({t / n * 1e3:.2f} us/frame), rounds {[round(x, 4) for x in res[n]]}", flush=True)
    b, a = np.polyfit(ns, ts, 1)
    print(f"fit T(n) = {a:.4f} ms + {b * 1e3:.3f} us x n: fixed part at n=120 = {a / (a + b * 120) * 100:.1f}%")
    enc.close()


if __name__ == "__main__":
    main()
