#!/usr/bin/env python3
"""k_encode's per-launch fixed cost (its drain and launch ramp) from synced launches of 60 /
120 / 240 / 480 4K frames: T(n) = a + b n.  usage (GPU box): python3 tools/drain_probe.py"""
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
    ns, ts = [60, 120, 240, 480], []
    for n in ns:
        enc.submit(device_ptr=pool.data_ptr(), nframes=n)
        enc.sync()
        enc.kernel_times(reset=True)
        for _ in range(5):
            enc.submit(device_ptr=pool.data_ptr(), nframes=n)
            enc.sync()
        kt, nl = enc.kernel_times()
        ts.append(kt["encode"])
        print(f"{content} n={n}: k_encode {kt['encode']:.4f} ms ({kt['encode'] / n * 1e3:.2f} us/frame)", flush=True)
    b, a = np.polyfit(ns, ts, 1)
    print(f"fit T(n) = {a:.4f} ms + {b * 1e3:.3f} us x n: fixed part at n=120 = {a / (a + b * 120) * 100:.1f}%")
    enc.close()


if __name__ == "__main__":
    main()
