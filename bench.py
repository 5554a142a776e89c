#!/usr/bin/env python3
"""Benchmark of the hot path named by BASELINE.json: 4K yuv420p MJPEG q=5 segment encode
(configs[1]: "4K60 60 s testsrc2 yuv420p MJPEG q=5 on one MI355X").  `--workload` selects
the other BASELINE configs at their own segment sizes (c1 1080p with FFmpeg's default
-huffman optimal, c4 4K->1080p bicubic q=3, c5 8K yuvj420p 0.5 s segments); the default
run (no flags) is configs[1], the line the driver records.

A step = one 2-second segment (120 frames of 3840x2160 yuv420p) encoded on one GPU,
frames already resident in HBM (a pool of distinct synthetic testsrc2-like frames
generated on the device), JPEG output packed in HBM.  Default K=30 steps = the 60 s
(3600-frame) clip of configs[1].  Multi-GPU: one process per GPU
(torch.distributed.run), segments sharded with no data-path collective (weak scaling);
the barrier / max-over-ranks timing uses the process group only for bookkeeping.

Prints ONE JSON line on rank 0 (see the driver contract in the task description).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "encoded frames/sec (node), 4K yuv420p MJPEG q=5 at 1/2/4/8 GPUs; HBM GB/s"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

# BASELINE.json configs: (src W, H, dst W, H, q, frames per segment, yuvj420p input, huffman, text)
WORKLOADS = {
    "c2": (3840, 2160, 3840, 2160, 5, 120, False, "default",
           "4K60 testsrc2 yuv420p MJPEG q=5 (BASELINE configs[1]); step = one 2 s segment"),
    "c1": (1920, 1080, 1920, 1080, 5, 250, False, "optimal",
           "1080p30 testsrc2 yuv420p MJPEG q=5, FFmpeg's default -huffman optimal (BASELINE "
           "configs[0] profile + -dct int -bitexact); step = one 250-frame (keyint) segment"),
    "c4": (3840, 2160, 1920, 1080, 3, 120, False, "default",
           "4K->1080p bicubic scale + MJPEG q=3 (BASELINE configs[3]); step = one 2 s segment"),
    "c5": (7680, 4320, 7680, 4320, 5, 15, True, "default",
           "8K30 yuvj420p MJPEG q=5, 0.5 s segments (BASELINE configs[4]); step = one segment"),
}
W, H, DW, DH, Q, SEG, FULL, HUFF, WTEXT = WORKLOADS["c2"]


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--workload", choices=sorted(WORKLOADS), default="c2")
    p.add_argument("--huffman", choices=["default", "optimal"], default=None)
    p.add_argument("--rst", action="store_true",
                   help="slice-threaded layout (-slices N: DRI + one restart interval per MCU row)")
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--pool", type=int, default=480, help="distinct resident frames per GPU")
    p.add_argument("--seg", type=int, default=None)
    p.add_argument("--cpu-sample-frames", type=int, default=96)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-kernel-timing", action="store_true", help="diagnostics: no HIP events at all")
    p.add_argument("--kernel-timing-detail", action="store_true",
                   help="events around every tail kernel too (adds ~10 us idle per event)")
    p.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_encode_4k_q5.json"),
                   help="PMC traffic summary written by tools/pmc_traffic.py")
    return p.parse_args()


def cpu_baseline(nframes: int):
    """Oracle ('port') on the host cores: bounded sample of the same workload."""
    import multiprocessing as mp
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, 16))
    ctx = mp.get_context("fork")
    with ctx.Pool(cores, initializer=_cpu_init) as pool:
        pool.map(_cpu_warm, range(cores))
        t0 = time.perf_counter()
        sizes = pool.map(_cpu_encode, range(nframes))
        dt = time.perf_counter() - t0
    return {"value": nframes / dt, "unit": "frames/s", "cores": cores, "kind": "port",
            "sample": f"{nframes} frames {W}x{H}{'->%dx%d' % (DW, DH) if (DW, DH) != (W, H) else ''} "
                      f"{'yuvj420p' if FULL else 'yuv420p'} q={Q} -huffman {HUFF} (testsrc2-like, 8 distinct), "
                      f"oracle/mjpeg_oracle.c (C restatement of FFmpeg's mjpeg+swscale path), "
                      f"{cores} processes, {dt:.1f} s wall",
            "mean_jpeg_bytes": float(sum(sizes) / len(sizes))}


_CPU_FRAMES = None


def _cpu_init():
    global _CPU_FRAMES
    from ffmpeg_distributed_amd.testsrc import testsrc2_i420
    from ffmpeg_distributed_amd.encoder import split_i420
    _CPU_FRAMES = [split_i420(testsrc2_i420(W, H, t, full_range=FULL), W, H) for t in range(0, 8)]


def _cpu_warm(_):
    import oracle
    oracle.lib()
    return 0


def _cpu_encode(i):
    import oracle
    y, u, v = _CPU_FRAMES[i % len(_CPU_FRAMES)]
    return len(oracle.encode_frame(y, u, v, dst_w=DW, dst_h=DH, full_range=FULL, qscale=Q,
                                   huffman=HUFF))


def main():
    global W, H, DW, DH, Q, SEG, FULL, HUFF, WTEXT
    a = parse()
    W, H, DW, DH, Q, SEG, FULL, HUFF, WTEXT = WORKLOADS[a.workload]
    if a.huffman:
        HUFF = a.huffman
    if a.seg is None:
        a.seg = SEG
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))

    import torch
    import torch.distributed as dist
    from ffmpeg_distributed_amd import build as B
    B.build()
    from ffmpeg_distributed_amd.encoder import MjpegEncoder
    from ffmpeg_distributed_amd.shard import max_over_ranks, segments_for_rank, timed_region
    from ffmpeg_distributed_amd.testsrc import testsrc2_i420_torch

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)

    def barrier():
        if world > 1:
            dist.barrier()

    # The job is (warmup + steps) x world segments of `seg` frames, split round-robin over
    # ranks (shard.segments_for_rank).  Each rank keeps a resident pool of its first
    # segments' frames (testsrc2-like, time index = global frame number) and cycles it.
    seg = a.seg
    my_segs = segments_for_rank((a.warmup + a.steps) * world, rank, world)
    nseg_pool = max(1, min(len(my_segs), a.pool // seg))
    pool_n = nseg_pool * seg
    fb = W * H + 2 * ((W + 1) // 2) * ((H + 1) // 2)
    pool = torch.empty((pool_n, fb), dtype=torch.uint8, device=dev)
    gen = 20 if W * H <= 3840 * 2160 else 5
    for j in range(nseg_pool):
        for i in range(0, seg, gen):
            k = min(gen, seg - i)
            pool[j * seg + i: j * seg + i + k] = testsrc2_i420_torch(W, H, my_segs[j] * seg + i, k, dev,
                                                                     full_range=FULL)
    torch.cuda.synchronize()

    if a.rst:
        HUFF = "default"  # slice threading forces the default tables
    enc = MjpegEncoder(local, W, H, DW, DH, full_range=FULL, qscale=Q, max_batch=seg,
                       timing=False if a.no_kernel_timing else ("detail" if a.kernel_timing_detail else True),
                       huffman=HUFF, rst=a.rst)
    bytes_out = []

    # Segments are pipelined two deep (mjg_submit queues up to two): segment s+1's kernels
    # are queued behind segment s's before s is synced, so the GPU does not idle while the
    # host collects a segment's sizes and issues the next launches.
    def step(s):
        base = pool[(s % nseg_pool) * seg]
        enc.submit(device_ptr=base.data_ptr(), nframes=seg)
        if enc.pending == 2:
            bytes_out.append(int(enc.sync().sum()))

    def drain_and_sync():
        while enc.pending:
            bytes_out.append(int(enc.sync().sum()))
        torch.cuda.synchronize()

    def reset():
        drain_and_sync()
        enc.kernel_times(reset=True)
        bytes_out.clear()

    dt = timed_region(step, a.warmup, a.steps, barrier, drain_and_sync, reset)
    if a.no_kernel_timing:
        from ffmpeg_distributed_amd._lib import KERNEL_NAMES
        kt, nl = {k: 0.0 for k in KERNEL_NAMES}, 0
    else:
        kt, nl = enc.kernel_times()
    dt = max_over_ranks(dt, dist if world > 1 else None, dev)

    frames_total = a.steps * seg * world
    value = frames_total / dt
    mean_jpeg = sum(bytes_out) / max(1, len(bytes_out) * seg)

    # Roofline of the dominant kernel (k_encode): algorithmic bytes per launch =
    # (input planes 12,441,600 B at 4K + JPEG bytes written) x frames per launch.
    # With -vf scale the input planes are the scaled frame's (k_scale reads the source and
    # writes them; its own line is in kernel_ms_per_step).
    enc_ms = kt["encode"]
    efb = DW * DH + 2 * ((DW + 1) // 2) * ((DH + 1) // 2)
    alg_bytes = (efb + mean_jpeg) * seg
    achieved = alg_bytes / (enc_ms * 1e-3) / 1e9 if enc_ms > 0 else 0.0
    traffic = None
    try:
        with open(a.pmc) as f:
            pm = json.load(f)
        if pm.get("workload", {}).get("frames_per_launch") == seg and a.workload == "c2" and \
                HUFF == "default" and not a.rst:
            traffic = pm.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass

    out = None
    if rank == 0:
        cpu = None
        if not a.no_cpu_baseline and world == 1:
            try:
                cpu = cpu_baseline(a.cpu_sample_frames)
            except Exception as e:  # reported, never fatal for the GPU number
                cpu = {"value": None, "error": repr(e)}
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic: testsrc2-like generator, frames resident in HBM "
                    f"({pool_n} distinct per GPU), output packed in HBM",
            "config": {"workload": WTEXT, "width": W, "height": H, "dst_width": DW,
                       "dst_height": DH, "qscale": Q, "frames_per_step": seg,
                       "global_batch": seg * world, "parallelism": f"segment-dp{world}",
                       "profile": (f"-vf scale={DW}:{DH}:flags=bicubic " if (DW, DH) != (W, H) else "")
                       + f"-c:v mjpeg -q:v {Q} -dct int -huffman {HUFF} -bitexact"
                       + (" -slices 8" if a.rst else "")},
            "roofline": {"bound": "hbm", "kernel": "k_encode",
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "alg_bytes_per_launch": int(alg_bytes),
                         "avg_launch_ms": round(enc_ms, 4), "launches": nl},
            "kernel_ms_per_step": {k: round(v, 4) for k, v in kt.items()},
            "mean_jpeg_bytes": round(mean_jpeg, 1),
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    enc.close()
    if world > 1:
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
