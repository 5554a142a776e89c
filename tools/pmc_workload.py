#!/usr/bin/env python3
"""Small fixed workload for rocprofv3 PMC passes: one BASELINE config of bench.py
(`--workload c2|c1|c4|c5`), `--launches` submits of one segment of resident frames, each
synced before the next (so no two kernels of the encoder overlap)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", default="c2")
    p.add_argument("--content", default="testsrc")
    p.add_argument("--launches", type=int, default=3)
    a = p.parse_args()
    import torch
    import bench
    from ffmpeg_distributed_amd.encoder import MjpegEncoder
    from ffmpeg_distributed_amd.testsrc import CONTENT
    W, H, DW, DH, Q, SEG, FULL, HUFF, _ = bench.WORKLOADS[a.workload]
    dev = torch.device("cuda", 0)
    fb = W * H + 2 * ((W + 1) // 2) * ((H + 1) // 2)
    pool = torch.empty((SEG, fb), dtype=torch.uint8, device=dev)
    gen = CONTENT[a.content]
    for i in range(0, SEG, 10):
        k = min(10, SEG - i)
        pool[i:i + k] = gen(W, H, i, k, dev, full_range=FULL)
    torch.cuda.synchronize()
    enc = MjpegEncoder(0, W, H, DW, DH, full_range=FULL, qscale=Q, max_batch=SEG, huffman=HUFF)
    tot = 0
    for _ in range(a.launches):
        enc.submit(device_ptr=pool.data_ptr(), nframes=SEG)
        tot += int(enc.sync().sum())
    print(f"workload {a.workload} content {a.content} frames/launch {SEG} launches {a.launches} "
          f"mean_jpeg {tot / a.launches / SEG:.1f}")
    enc.close()


if __name__ == "__main__":
    main()
