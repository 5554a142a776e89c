#!/usr/bin/env python3
"""Per-phase wall cycles of k_encode (VALU stage, -huffman default) from the phase_clock probe
patch (tools/patches.py): VARIANTS="ph=@phase_clock" tools/variants.py --build, then this on the
GPU box.  For each WL/CONTENT: 3 synced submits, shader-clock cycles per chunk-wave per phase
(wall time of the wave, so other waves' issue on the SIMD is included).

usage: WL=c2 CONTENT=testsrc python3 tools/phase_probe.py [variant-name ...]   (default: ph)"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ["row pass (+ edge refetch)", "next chunk's loads issued", "column screen + mask",
          "DC prediction + wide-block choice", "per-lane emission", "wave-parallel blocks",
          "pack", "unit bookkeeping + loop"]


def main():
    import torch
    import bench
    from ffmpeg_distributed_amd import _lib
    from ffmpeg_distributed_amd.testsrc import CONTENT
    names = sys.argv[1:] or ["ph"]
    W, H, DW, DH, Q, N, FULL, HUFF, _ = bench.WORKLOADS[os.environ.get("WL", "c2")]
    content = os.environ.get("CONTENT", "testsrc")
    dev = torch.device("cuda", 0)
    pool = torch.empty((N, W * H + 2 * ((W + 1) // 2) * ((H + 1) // 2)), dtype=torch.uint8, device=dev)
    for i in range(0, N, 10):
        k = min(10, N - i)
        pool[i:i + k] = CONTENT[content](W, H, i, k, dev, full_range=FULL)
    torch.cuda.synchronize()
    for name in names:
        _lib._lib = None
        _lib.LIB_PATH = os.path.join(ROOT, "ffmpeg_distributed_amd", f"libmjgpu_v_{name}.so")
        from ffmpeg_distributed_amd.encoder import MjpegEncoder
        enc = MjpegEncoder(0, W, H, DW, DH, full_range=FULL, qscale=Q, max_batch=N, huffman="default")
        L = _lib.load()
        L.mjg_probe_phase.argtypes = [C.POINTER(C.c_ulonglong)]
        acc = (C.c_ulonglong * 8)()
        enc.submit(device_ptr=pool.data_ptr(), nframes=N)  # warm
        enc.sync()
        L.mjg_probe_phase(acc)
        runs = 3
        for _ in range(runs):
            enc.submit(device_ptr=pool.data_ptr(), nframes=N)
            enc.sync()
        L.mjg_probe_phase(acc)
        nchunks = -(-((W + 15) // 16) * ((H + 15) // 16) * 6 // 64) * N * runs  # 4:2:0 chunks per frame
        tot = sum(acc)
        print(f"== {name} {os.environ.get('WL', 'c2')} {content}: {tot / nchunks:.0f} cycles per chunk-wave "
              f"({nchunks} chunk-waves)")
        for i, p in enumerate(PHASES):
            print(f"  {p:36s} {acc[i] / nchunks:8.0f}  {100 * acc[i] / max(tot, 1):5.1f}%")
        # per-wave start / end (s_memrealtime, 100 MHz) of one more launch: the drain at its end
        L.mjg_probe_waves.argtypes = [C.POINTER(C.c_ulonglong), C.POINTER(C.c_ulonglong)]
        t0, t1 = (C.c_ulonglong * 32768)(), (C.c_ulonglong * 32768)()  # + hw ids / chunk counts
        L.mjg_probe_waves(t0, t1)
        enc.submit(device_ptr=pool.data_ptr(), nframes=N)
        enc.sync()
        L.mjg_probe_waves(t0, t1)
        import numpy as np
        ext0 = np.frombuffer(bytes(t0), dtype=np.uint32)[32768:]   # hw_id[16384], xcc_id[16384]
        ext1 = np.frombuffer(bytes(t1), dtype=np.uint32)[32768:]   # chunks per wave
        hw, xcc, nch = ext0[:16384], ext0[16384:], ext1[:16384]
        a, b = np.array(t0[:16384]), np.array(t1[:16384])
        ok = (a > 0) & (b > 0)
        hw, xcc, nch = hw[ok], xcc[ok] & 0xf, nch[ok]
        a, b = a[ok].astype(np.float64), b[ok].astype(np.float64)
        span = (b.max() - a.min()) / 100.0  # us
        busy = (b - a).sum() / 100.0
        ends = np.sort((b.max() - b) / 100.0)
        starts = np.sort((a - a.min()) / 100.0)
        print(f"  waves {ok.sum()}: launch span {span:.1f} us, wave-time utilisation {busy / (ok.sum() * span):.3f}; "
              f"start spread p50/p99/max {starts[len(starts) // 2]:.1f}/{starts[int(len(starts) * .99)]:.1f}/"
              f"{starts[-1]:.1f} us; idle before the launch end p10/p50/p90/max "
              f"{ends[len(ends) // 10]:.1f}/{ends[len(ends) // 2]:.1f}/{ends[int(len(ends) * .9)]:.1f}/{ends[-1]:.1f} us")
        busyw = (b - a) / 100.0
        end_idle = (b.max() - b) / 100.0
        simd = (hw >> 4) & 3
        cu = (hw >> 8) & 15
        se = (hw >> 13) & 3
        for name, key in (("xcc", xcc), ("simd", simd), ("se", se)):
            parts = [f"{int(v)}: busy {busyw[key == v].mean():.0f} us, chunks {nch[key == v].mean():.1f}, "
                     f"us/chunk {(busyw[key == v] / np.maximum(nch[key == v], 1)).mean():.2f}, end-idle "
                     f"{end_idle[key == v].mean():.0f}" for v in np.unique(key)]
            print(f"  by {name}: " + " | ".join(parts))
        slot = hw & 15  # wave slot on its SIMD
        parts = [f"{int(v)}: us/chunk {(busyw[slot == v] / np.maximum(nch[slot == v], 1)).mean():.2f} "
                 f"chunks {nch[slot == v].mean():.1f}" for v in np.unique(slot)]
        print("  by wave slot: " + " | ".join(parts))
        enc.close()


if __name__ == "__main__":
    main()
