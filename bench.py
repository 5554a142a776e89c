#!/usr/bin/env python3
"""Benchmark of the hot path named by BASELINE.json: 4K yuv420p MJPEG q=5 segment encode
(configs[1]: "4K60 60 s testsrc2 yuv420p MJPEG q=5 on one MI355X").  `--workload` selects
the other BASELINE configs at their own segment sizes (c1 1080p with FFmpeg's default
-huffman optimal, c4 4K->1080p bicubic q=3, c5 8K yuvj420p 0.5 s segments); the default
run (no flags) is configs[1], the line the driver records.  `--content` swaps the
testsrc2-like frames for fractal "natural" content or testsrc2 with noise macroblocks
(content sensitivity of the entropy coder).

A step = one 2-second segment (120 frames of 3840x2160 yuv420p) encoded on one GPU,
frames already resident in HBM (a pool of distinct synthetic frames generated on the
device), JPEG output packed in HBM.  Multi-GPU: one process per GPU
(torch.distributed.run), segments sharded with no data-path collective (weak scaling);
the barrier / max-over-ranks timing uses the process group only for bookkeeping.

Roofline: algorithmic bytes = input planes read + JPEG bytes written; the
primary `roofline` is the kernel that reads the input planes, `roofline_kernels` lists every
timed kernel with its own algorithmic bytes and, when profiles/pmc_<workload>.json holds a
PMC pass of the same configuration, its counted HBM traffic.

Prints ONE JSON line on rank 0 (see the driver contract in the task description).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import subprocess
import sys
import threading
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
    p.add_argument("--content", choices=["testsrc", "natural", "noise-patches"], default="testsrc")
    p.add_argument("--huffman", choices=["default", "optimal"], default=None)
    p.add_argument("--rst", action="store_true",
                   help="slice-threaded layout (-slices N: DRI + one restart interval per MCU row)")
    p.add_argument("--prewarm-ms", type=float, default=500.0,
                   help="untimed encode steps for this long before the W warmup steps: the GPU leaves its "
                        "idle clocks only after ~0.3 s of load (without: c2 -7%%, DESIGN §6); 0 turns it off")
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--pool", type=int, default=480, help="distinct resident frames per GPU")
    p.add_argument("--seg", type=int, default=None)
    p.add_argument("--cpu-seconds", type=float, default=4.0,
                   help="CPU baseline: wall seconds per point of the core-count sweep")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-baseline-only", action="store_true",
                   help="internal: run the CPU baseline sweep alone (no torch, no GPU) and print it")
    p.add_argument("--no-e2e", action="store_true", help="skip the end-to-end leg (rank 0, N=1 only)")
    p.add_argument("--e2e-only", action="store_true",
                   help="internal: run the end-to-end leg alone (no torch, no GPU in this process) and print it")
    p.add_argument("--device", type=int, default=0, help="internal (--e2e-only): the GPU of the worker path")
    p.add_argument("--e2e-segments", type=int, default=6)
    p.add_argument("--segments-per-launch", action="store_true",
                   help="also time K = 2, 4 segments per submit (mjg_submit_segments, N=1 only); off by "
                        "default so a profile of the default command holds only the headline's launches")
    p.add_argument("--no-kernel-timing", action="store_true", help="diagnostics: no HIP events at all")
    p.add_argument("--kernel-timing-detail", action="store_true",
                   help="events around every tail kernel too (adds ~10 us idle per event)")
    return p.parse_args()


# ------------------------------------------------------------------------ CPU baseline
def host_cpu():
    """Cores this process may use (affinity, capped by the cgroup CPU quota), the machine's
    CPU count and model."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, math.ceil(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = min(aff, quota) if quota else aff
    return {"usable": usable, "affinity": aff, "cgroup_quota": quota, "machine_cpus": os.cpu_count(),
            "model": model}


_CPU_FRAMES = None


def _cpu_init():
    global _CPU_FRAMES
    from ffmpeg_distributed_amd.testsrc import testsrc2_i420
    from ffmpeg_distributed_amd.encoder import split_i420
    import oracle
    oracle.lib()
    _CPU_FRAMES = [split_i420(testsrc2_i420(W, H, t, full_range=FULL), W, H) for t in range(0, 8)]


def _cpu_encode_until(args):
    """Encode frames until the deadline (time.time() seconds); returns (frames, bytes, end)."""
    deadline, rank = args
    import oracle
    n = nbytes = 0
    while True:
        y, u, v = _CPU_FRAMES[(rank + n) % len(_CPU_FRAMES)]
        nbytes += len(oracle.encode_frame(y, u, v, dst_w=DW, dst_h=DH, full_range=FULL, qscale=Q,
                                          huffman=HUFF))
        n += 1
        if time.time() >= deadline:
            return n, nbytes, time.time()


def segments_per_launch(a, pool, seg, nseg_pool, W, H, DW, DH, FULL, Q, HUFF, device, ks=(2, 4), nsegs=240):
    """Reported beside the headline, not as it: the same segments handed over K per submit
    (mjg_submit_segments; one k_encode launch and one tail per K segments, each segment's
    bytes those of its own submit).  The headline stays one segment per submit, which is what
    the per-segment worker path (fd.py:139-141 once per segment) does today."""
    import torch
    from ffmpeg_distributed_amd.encoder import MjpegEncoder
    res = {}
    for k in ks:
        if k > nseg_pool:
            continue
        enc = MjpegEncoder(device, W, H, DW, DH, full_range=FULL, qscale=Q, max_batch=k * seg,
                           huffman=HUFF, merge=False)
        if k > enc.max_segments:
            enc.close()
            continue
        ptrs = [pool[j * seg].data_ptr() for j in range(nseg_pool)]

        def run(n, s0):
            for s in range(s0, s0 + n):
                enc.submit_segments([(ptrs[(s * k + i) % nseg_pool], seg) for i in range(k)])
                if enc.pending == enc.host_depth:
                    enc.sync()
            while enc.pending:
                enc.sync()
            torch.cuda.synchronize()
        steps = max(8, nsegs // k)  # ~240 segments per K: the pipeline's fill and drain are <1%
        run(4, 0)
        t0 = time.perf_counter()
        run(steps, 4)
        dt = time.perf_counter() - t0
        enc.close()
        res[str(k)] = {"value": round(steps * k * seg / dt, 2), "unit": "frames/s",
                       "ms_per_segment": round(dt / (steps * k) * 1e3, 4),
                       "segments_per_submit": k, "submits": steps}
    return res


def cpu_baseline_sweep(seconds: float):
    """The oracle (kind "port": the C restatement of FFmpeg's mjpeg + swscale path, scalar
    C, one frame per process) on this host's cores, swept over process counts
    K in {1, usable/4, usable/2, usable}; each point runs `seconds` of wall time.  The value
    is the best point.  FFmpeg itself (the reference CPU path) is absent on this pool.
    Runs in a process that never touched the GPU (cpu_baseline starts it as a child); the
    pool's workers are closed and joined, never terminated."""
    import multiprocessing as mp
    hc = host_cpu()
    ks = sorted({1, max(1, hc["usable"] // 4), max(1, hc["usable"] // 2), hc["usable"]})
    ctx = mp.get_context("fork")
    sweep = []
    pool = ctx.Pool(hc["usable"], initializer=_cpu_init)
    try:
        pool.map(time.sleep, [0.01] * hc["usable"])  # every worker initialised
        for k in ks:
            t0 = time.time()
            res = pool.map(_cpu_encode_until, [(t0 + seconds, r) for r in range(k)], chunksize=1)
            dt = max(e for _, _, e in res) - t0
            frames = sum(n for n, _, _ in res)
            sweep.append({"processes": k, "frames": frames, "seconds": round(dt, 2),
                          "value": round(frames / dt, 2),
                          "mean_jpeg_bytes": round(sum(b for _, b, _ in res) / max(frames, 1), 1)})
    finally:
        pool.close()  # workers exit on their own: no SIGTERM into forked children
        pool.join()
    best = max(sweep, key=lambda s: s["value"])
    return {"value": best["value"], "unit": "frames/s", "cores": best["processes"], "kind": "port",
            "sample": f"{W}x{H}{'->%dx%d' % (DW, DH) if (DW, DH) != (W, H) else ''} "
                      f"{'yuvj420p' if FULL else 'yuv420p'} q={Q} -huffman {HUFF}, 8 distinct "
                      f"testsrc2-like frames cycled, {seconds:g} s of wall time per sweep point; "
                      f"oracle/mjpeg_oracle.c (scalar C restatement of FFmpeg's mjpeg + swscale "
                      f"path, not FFmpeg's SIMD encoder: FFmpeg is absent on this pool), one frame "
                      f"per process at a time",
            "host": hc, "sweep": sweep}


def cpu_baseline(seconds: float, workload: str, huffman: str):
    """cpu_baseline_sweep in a fresh interpreter (`bench.py --cpu-baseline-only`), which never
    imports torch or HIP: the benchmark process has initialised the GPU, and forking pool
    workers off it (round 3) left them with the GPU runtime's state and, under rocprofv3, the
    profiler's signal handlers."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-only", "--workload", workload,
           "--huffman", huffman, "--cpu-seconds", str(seconds)]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=60 + 8 * seconds)
    if r.returncode != 0:
        raise RuntimeError(f"cpu baseline child exited {r.returncode}: {r.stderr[-1000:]}")
    return json.loads(r.stdout.strip().splitlines()[-1])


# ------------------------------------------------------------------------ end to end
E2E_ARGS = {  # remote_args of each workload (fd.py:190 splits them from the CLI string)
    "c2": "-c:v mjpeg -q:v 5 -dct int -huffman default -bitexact",
    "c1": "-c:v mjpeg -q:v 5 -dct int -bitexact",
    "c4": "-vf scale=1920:1080:flags=bicubic -c:v mjpeg -q:v 3 -dct int -huffman default -bitexact",
    "c5": "-c:v mjpeg -q:v 5 -dct int -huffman default -bitexact",
}


def parse_worker_trace(line: str) -> dict:
    """worker.py's `mjg-trace: frames=N total=S setup=S read=S ...` line: the float phases
    (seconds) and the placement text after them."""
    out, rest = {}, []
    for tok in line.split()[1:]:
        k, sep, v = tok.partition("=")
        if k in ("frames", "total", "setup", "handoff", "client", "read", "submit", "sync", "fetch", "mux", "wait"):
            try:
                out[k] = float(v)
                continue
            except ValueError:
                pass
        rest.append(tok)
    out["placement"] = " ".join(rest)
    return out


def e2e(workload: str, device: int, segments: int, tmpdir=None):
    """End-to-end frames/s through the reference's worker contract (fd.py:131-141: segment
    file on stdin, Matroska on stdout, progress on stderr, exit code), timed outside the
    `value` region: one raw I420 Matroska segment of the workload (page cache) encoded
    `segments` times by
      per_segment_process: the dispatcher's TaskThread path for -H gpu:N, one process per
                           segment (mjg_client -> the resident encoder of the GPU);
      persistent:          the dispatcher's -P path (one `worker --serve` per host);
      python_worker:       one `python -m ffmpeg_distributed_amd.worker` process per segment
                           (MJG_RESIDENT=0; round 2's per-segment path), 2 segments.
    Steady fps = frames / median seconds of the segments after the first (which starts the
    resident encoder or the server: reported as first_segment_s)."""
    import shlex
    import statistics
    import subprocess
    import tempfile
    from fractions import Fraction
    from ffmpeg_distributed_amd import dispatcher as D
    from ffmpeg_distributed_amd.testsrc import write_raw_segment
    w, h, _, _, _, seg_frames, full, _, _ = WORKLOADS[workload]
    fps = Fraction(30) if workload == "c1" else Fraction(60) if workload in ("c2", "c4") else Fraction(30)
    args = shlex.split(E2E_ARGS[workload])
    d = tempfile.mkdtemp(prefix="mjg_e2e_", dir=tmpdir)
    seg = os.path.join(d, "seg.mkv")
    host = f"gpu:{device}"
    out = {"segment": f"{seg_frames} frames {w}x{h} raw I420 Matroska (V_UNCOMPRESSED), page cache",
           "remote_args": E2E_ARGS[workload]}
    try:
        t = time.monotonic()
        nbytes = write_raw_segment(seg, w, h, fps, seg_frames, full_range=full)
        out["segment_bytes"] = nbytes
        out["segment_write_s"] = round(time.monotonic() - t, 2)

        traces = []

        def leg(run_one, n):
            secs = []
            traces.clear()
            for i in range(n):
                dst = os.path.join(d, f"out{i}.mkv")  # a new file per segment, as the dispatcher writes
                t0 = time.monotonic()
                rc = run_one(dst)
                secs.append(time.monotonic() - t0)
                if rc != 0:
                    raise RuntimeError(f"segment {i} exited {rc}")
            steady = statistics.median(secs[1:]) if n > 1 else secs[0]
            r = {"segments": n, "first_segment_s": round(secs[0], 4),
                 "steady_s_per_segment": round(steady, 4), "fps_steady": round(seg_frames / steady, 1),
                 "seconds": [round(x, 4) for x in secs]}
            if len(traces) > 1:  # the worker's MJG_WORKER_TRACE phases (and the process's start /
                # exit as the dispatcher sees them), median over the steady segments
                keys = [k for k in traces[-1] if isinstance(traces[-1][k], float)]
                r["worker_trace_median_s"] = {k: round(statistics.median(t[k] for t in traces[1:] if k in t), 4)
                                              for k in keys}
                r["worker_trace_placement"] = traces[-1].get("placement")
            return r

        class TimedProc(D.FFMPEGProc):
            """FFMPEGProc noting when each stderr line arrives (start / trace line / exit)."""
            def _line(self, line):
                self.times.append((time.monotonic(), line[:16]))
                super()._line(line)

        def per_process(resident):
            argv = D.worker_argv(host, args, resident=resident)
            env = dict(os.environ, MJG_WORKER_TRACE="1")  # one mjg-trace: line per segment (worker.py)

            def one(dst):
                t0 = time.monotonic()
                with open(seg, "rb") as fi, open(dst, "wb") as fo:
                    p = TimedProc(argv, stdin=fi, stdout=fo, env=env)
                    p.times = []
                    rc = p.run()
                t_end = time.monotonic()
                if rc != 0:
                    sys.stderr.write(p.stderr[-2000:])
                for line in p.stderr.splitlines():
                    if line.startswith("mjg-trace:"):
                        traces.append(parse_worker_trace(line))
                if traces and p.times:
                    first = p.times[0][0]
                    tr_t = next((t for t, l in p.times if l.startswith("mjg-trace")), None)
                    traces[-1]["client_first_line"] = first - t0  # process start .. the worker's Duration line
                    if tr_t is not None:
                        traces[-1]["client_after_trace"] = t_end - tr_t  # the worker's last line .. process exit
                return rc
            return one

        if D.resident_enabled():
            r = leg(per_process(True), segments)
            r["argv"] = "mjg_client --device N -- <remote_args> (resident encoder per GPU)"
            out["per_segment_process"] = r
            # two -H gpu:N entries for one GPU (fd.py: two TaskThreads, fd.py:185-192): two
            # per-segment processes at a time, so one segment's host read and H2D overlap the
            # other's (one segment at a time is bound by its own 1.49 GB crossing PCIe)
            one = per_process(True)
            errs = []

            def client(j):
                for i in range(segments):
                    rc = one(os.path.join(d, f"out_c{j}_{i}.mkv"))
                    if rc != 0:
                        errs.append(rc)
            ths = [threading.Thread(target=client, args=(j,)) for j in range(2)]
            t0 = time.monotonic()
            for th in ths:
                th.start()
            for th in ths:
                th.join()
            wall = time.monotonic() - t0
            if errs:
                raise RuntimeError(f"concurrent e2e segments exited {errs}")
            out["per_segment_process_2clients"] = {
                "clients": 2, "segments": 2 * segments, "seconds": round(wall, 4),
                "fps": round(2 * segments * seg_frames / wall, 1),
                "argv": "two mjg_client processes at a time on one GPU (-H gpu:N given twice)"}
            from ffmpeg_distributed_amd import resident
            if not resident.shutdown(D.CLIENT, device):
                r["warning"] = "resident encoder still running after its shutdown"
        srv = D.GpuServer(host)
        try:
            r = leg(lambda dst: srv.run_task(D.Task(seg, dst, args)), segments)
        finally:
            srv.close()
        r["argv"] = "python -m ffmpeg_distributed_amd.worker --device N <remote_args> --serve (-P)"
        out["persistent"] = r
        r = leg(per_process(False), 2)
        r["argv"] = "python -m ffmpeg_distributed_amd.worker --device N <remote_args> (MJG_RESIDENT=0)"
        r["fps_steady"] = round(seg_frames / min(r["seconds"]), 1)
        out["python_worker"] = r
    finally:
        for f in os.listdir(d):
            os.remove(os.path.join(d, f))
        os.rmdir(d)
    return out


def e2e_child(workload: str, device: int, segments: int):
    """e2e in a fresh interpreter (`bench.py --e2e-only`) that never imports torch or HIP: the
    dispatcher's process (fd.py:120-148) holds no GPU state, while this benchmark process holds
    the HIP runtime and a resident frame pool, and forking the per-segment processes off it
    (subprocess.Popen) costs milliseconds per segment that the dispatcher never pays."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--e2e-only", "--workload", workload,
           "--device", str(device), "--e2e-segments", str(segments)]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=600)
    if r.returncode != 0:
        raise RuntimeError(f"e2e child exited {r.returncode}: {r.stderr[-1500:]}")
    return json.loads(r.stdout.strip().splitlines()[-1])


# ------------------------------------------------------------------------ roofline
def frame_bytes(w, h):
    return w * h + 2 * ((w + 1) // 2) * ((h + 1) // 2)


def load_pmc(workload, content, digest):
    """profiles/pmc_<workload>.json's per-kernel counts, only when the file was counted on the
    library this run loaded (its `library_digest` equals build.source_digest()); otherwise
    ({}, reason) and every `traffic` is null: counters of another build are never reported."""
    if content != "testsrc":
        return {}, "no PMC pass for this content"
    path = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return {}, f"no {os.path.relpath(path, ROOT)}"
    if d.get("library_digest") != digest:
        return {}, (f"{os.path.relpath(path, ROOT)} was counted on library {str(d.get('library_digest'))[:12]}, "
                    f"this run loaded {digest[:12]}: traffic not reported")
    fpl = d.get("workload", {}).get("frames_per_launch") or WORKLOADS[workload][5]
    # per frame: the PMC passes count single-segment launches (tools/pmc_workload.py syncs each),
    # the bench's launches may carry two merged segments
    kern = {k: dict(v, hbm_bytes_per_frame=v["hbm_bytes_per_launch"] / fpl) for k, v in d.get("kernels", {}).items()}
    return kern, os.path.relpath(path, ROOT)


def pmc_traffic(pmc, fpl, *names):
    """HBM bytes per launch of `fpl` frames of the kernels whose names contain any of `names`
    (None when the PMC file has none of them)."""
    hit = [v["hbm_bytes_per_frame"] * fpl for k, v in pmc.items() if any(n in k for n in names)]
    return round(sum(hit)) if hit else None


def roofline_entry(kernel, alg_bytes, ms, traffic, what):
    ach = alg_bytes / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    return {"bound": "hbm", "kernel": kernel, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
            "alg_bytes_per_launch": int(alg_bytes), "avg_launch_ms": round(ms, 4), "bytes": what}


def rooflines(kt, fpl, mean_jpeg, pmc, optimal, scaled, step_ms=None, seg=None):
    """Per-kernel roofline entries (SURVEY §8d bytes per launch: `fpl` frames per launch, a
    merged launch carrying two segments) and the primary one (reads the input).
    step_ms: consecutive launches run on two streams and overlap (csrc/api.hip alloc_slot: the
    next launch starts in the previous one's drain), so a kernel's event interval includes time
    shared with the other launch's kernels; the primary entry is then one step's bytes (`seg`
    frames) over the wall time per step, which the kernel trace's launch period reproduces
    (tools/timeline.py, profiles/r05*_timeline.txt); the per-kernel entries stay as measured,
    overlap included, and bench.py adds isolated launches beside them."""
    src_b, dst_b, jpeg_b = frame_bytes(W, H) * fpl, frame_bytes(DW, DH) * fpl, mean_jpeg * fpl
    sstep = (seg or fpl) / fpl  # one step's share of a launch's bytes

    def per_step(tr):
        # the primary entry's bytes and traffic are one step's when it is timed per step
        return None if tr is None else round(tr * sstep) if step_ms else tr
    out = []
    if scaled:  # k_scale writes the scaled planes to HBM, k_encode reads them
        out.append(roofline_entry("k_scale", src_b + dst_b, kt["scale"], pmc_traffic(pmc, fpl, "k_scale"),
                                  "source planes read + scaled planes written"))
        enc_in = dst_b
    else:
        enc_in = src_b
    if optimal:
        out.append(roofline_entry("k_encode<count> + k_huff_build", enc_in, kt["huff"],
                                  pmc_traffic(pmc, fpl, "k_encode", "k_huff_build"),
                                  "input planes read (symbol records are not credited)"))
        out.append(roofline_entry("k_emit_syms", jpeg_b, kt["encode"], pmc_traffic(pmc, fpl, "k_emit_syms"),
                                  "JPEG scan bits written"))
        primary = roofline_entry("count pass + emission (k_encode<count>, k_huff_build, k_emit_syms)"
                                 + (", wall time per step" if step_ms else ""),
                                 (enc_in + jpeg_b) * (sstep if step_ms else 1), step_ms or (kt["huff"] + kt["encode"]),
                                 per_step(pmc_traffic(pmc, fpl, "k_encode", "k_huff_build", "k_emit_syms")),
                                 "input planes read + JPEG written")
    else:
        name = "k_encode"
        out.append(roofline_entry(name, enc_in + jpeg_b, kt["encode"],
                                  pmc_traffic(pmc, fpl, "k_encode", "k_scale_encode"),
                                  ("scaled" if enc_in == dst_b and scaled else "input") +
                                  " planes read + JPEG written"))
        primary = out[0]
        if scaled and step_ms:
            primary = roofline_entry("k_scale + k_encode, wall time per step", (src_b + jpeg_b) * sstep, step_ms,
                                     per_step(pmc_traffic(pmc, fpl, "k_scale", "k_encode")),
                                     "source planes read + JPEG written")
        elif step_ms:
            primary = roofline_entry(name + ", wall time per step (launches overlap)", (enc_in + jpeg_b) * sstep,
                                     step_ms, per_step(out[0]["traffic"]), out[0]["bytes"])
    return primary, out


def torchrun_argv(gpus: int, argv, port: int):
    """`--gpus N` (N > 1) outside a launcher: the driver's own launch line, one rank per GPU."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]


def main():
    global W, H, DW, DH, Q, SEG, FULL, HUFF, WTEXT
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ and not (a.cpu_baseline_only or a.e2e_only):
        # started without a launcher: run the ranks as a child (before anything touches the GPU)
        # and exit with its code, so `python bench.py --gpus N` measures N GPUs, not one
        import socket
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        sys.exit(subprocess.run(torchrun_argv(a.gpus, sys.argv[1:], port)).returncode)
    if "WORLD_SIZE" in os.environ and a.gpus != int(os.environ["WORLD_SIZE"]):
        print(f"bench.py: --gpus {a.gpus} under a launcher of {os.environ['WORLD_SIZE']} ranks: "
              "measuring the launcher's ranks", file=sys.stderr)
    W, H, DW, DH, Q, SEG, FULL, HUFF, WTEXT = WORKLOADS[a.workload]
    if a.huffman:
        HUFF = a.huffman
    if a.rst:
        HUFF = "default"  # slice threading forces the default tables
    if a.seg is None:
        a.seg = SEG
    if a.cpu_baseline_only:  # the child of cpu_baseline: nothing here touches the GPU
        res = cpu_baseline_sweep(a.cpu_seconds)
        print(json.dumps(res), flush=True)
        return res
    if a.e2e_only:  # the child of e2e_child: the dispatcher's side, no GPU in this process
        res = e2e(a.workload, a.device, a.e2e_segments)
        print(json.dumps(res), flush=True)
        return res
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))

    import torch
    import torch.distributed as dist
    from ffmpeg_distributed_amd import build as B
    B.build()
    from ffmpeg_distributed_amd.encoder import MjpegEncoder
    from ffmpeg_distributed_amd.shard import max_over_ranks, segments_for_rank, timed_region
    from ffmpeg_distributed_amd.testsrc import CONTENT

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
    # segments' frames (time index = global frame number) and cycles it.
    seg = a.seg
    my_segs = segments_for_rank((a.warmup + a.steps) * world, rank, world)
    nseg_pool = max(1, min(len(my_segs), a.pool // seg))
    pool_n = nseg_pool * seg
    pool = torch.empty((pool_n, frame_bytes(W, H)), dtype=torch.uint8, device=dev)
    gen_fn = CONTENT[a.content]
    gen = 20 if W * H <= 3840 * 2160 else 5
    for j in range(nseg_pool):
        for i in range(0, seg, gen):
            k = min(gen, seg - i)
            pool[j * seg + i: j * seg + i + k] = gen_fn(W, H, my_segs[j] * seg + i, k, dev, full_range=FULL)
    torch.cuda.synchronize()

    enc = MjpegEncoder(local, W, H, DW, DH, full_range=FULL, qscale=Q, max_batch=seg,
                       timing=False if a.no_kernel_timing else ("detail" if a.kernel_timing_detail else True),
                       huffman=HUFF, rst=a.rst, merge=True)
    bytes_out = []

    # Segments are pipelined enc.depth (mjg_queue_depth(): 2) deep, as mjg_submit queues them: later segments'
    # kernels are queued behind segment s's before s is synced, so the GPU does not idle while
    # the host collects a segment's sizes and issues the next launches.
    depth = enc.depth

    def step(s):
        base = pool[(s % nseg_pool) * seg]
        enc.submit(device_ptr=base.data_ptr(), nframes=seg)
        if enc.pending == depth:
            bytes_out.append(int(enc.sync().sum()))

    def drain_and_sync():
        while enc.pending:
            bytes_out.append(int(enc.sync().sum()))
        torch.cuda.synchronize()

    def trace_marker():
        # a tiny kernel on torch's stream (rocprofv3 kernel trace: "spin_kernel"), outside the
        # timed region, that brackets the timed steps' launches for tools/timeline.py
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()

    def reset():
        drain_and_sync()
        if not a.no_kernel_timing:
            enc.kernel_times(reset=True)
        bytes_out.clear()
        trace_marker()

    # The marker kernel's first launch loads its code object (~2.6 ms on the host, measured in
    # the r05 HEAD trace): done here, not in the idle gap right before the timed steps, where the
    # GPU would drop its clock (a 2 ms idle gap before 20 steps costs 7%: tools/region_probe.py,
    # profiles/r05/region_probe.txt)
    trace_marker()
    # ranks start the prewarm together, so none idles long at the barrier before the timed steps
    # (an idle GPU drops its clock within milliseconds)
    barrier()
    prewarm = 0
    if a.prewarm_ms > 0:
        t_pw = time.perf_counter()
        while (time.perf_counter() - t_pw) * 1e3 < a.prewarm_ms:
            step(prewarm)
            prewarm += 1
        drain_and_sync()
    dt = timed_region(step, a.warmup, a.steps, barrier, drain_and_sync, reset)
    trace_marker()
    if a.no_kernel_timing:
        from ffmpeg_distributed_amd._lib import KERNEL_NAMES
        kt, nl = {k: 0.0 for k in KERNEL_NAMES}, 0
    else:
        kt, nl = enc.kernel_times()
    dt = max_over_ranks(dt, dist if world > 1 else None, dev)

    frames_total = a.steps * seg * world
    value = frames_total / dt
    mean_jpeg = sum(bytes_out) / max(1, len(bytes_out) * seg)
    fpl = a.steps * seg / nl if nl else seg  # frames per launch (merged launches carry two segments)
    pmc, pmc_src = (load_pmc(a.workload, a.content, B.source_digest())
                    if (seg == SEG and not a.rst and HUFF == WORKLOADS[a.workload][7]) else ({}, "no PMC pass for this configuration"))
    overlap = True  # consecutive launches run on two streams (csrc/api.hip alloc_slot; see rooflines)
    primary, per_kernel = rooflines(kt, fpl, mean_jpeg, pmc, HUFF == "optimal", (DW, DH) != (W, H),
                                    dt / a.steps * 1e3 if overlap else None, seg)
    primary = dict(primary, launches=nl, frames_per_launch=round(fpl, 2), traffic_source=pmc_src)

    # isolated launches (after the timed region, each synced before the next, so nothing
    # overlaps them): the kernels' own duration, one segment per launch (the main context: a
    # submit to an idle GPU launches at once) and two segments per launch (the shape of a
    # merged launch, as one two-segment list on a context of twice the frames)
    iso = []
    if not a.no_kernel_timing:
        for k in (1, 2):
            if k > nseg_pool:
                continue
            e2 = enc if k == 1 else MjpegEncoder(local, W, H, DW, DH, full_range=FULL, qscale=Q, max_batch=k * seg,
                                                  timing=True, huffman=HUFF, rst=a.rst, merge=False)
            e2.kernel_times(reset=True)
            for r in range(4):
                segs = [(pool[((r * k + i) % nseg_pool) * seg].data_ptr(), seg) for i in range(k)]
                if k == 1:
                    e2.submit(device_ptr=segs[0][0], nframes=seg)
                else:
                    e2.submit_segments(segs)
                e2.sync()
            kti, nli = e2.kernel_times(reset=True)
            if e2 is not enc:
                e2.close()
            _, ents = rooflines(kti, k * seg, mean_jpeg, pmc, HUFF == "optimal", (DW, DH) != (W, H))
            for e in ents:
                e["kernel"] += f" (isolated: {k} segment{'s' if k > 1 else ''} per launch, synced)"
                e["launches"] = nli
            iso += ents
        per_kernel += iso
        trace_marker()

    batched = None
    if a.segments_per_launch and world == 1 and not a.rst and nseg_pool >= 2:
        batched = segments_per_launch(a, pool, seg, nseg_pool, W, H, DW, DH, FULL, Q, HUFF, local)

    out = None
    if rank == 0:
        e2e_res = None
        if not a.no_e2e and world == 1 and a.content == "testsrc" and not a.rst:
            try:
                e2e_res = e2e_child(a.workload, local, a.e2e_segments)
            except Exception as e:  # reported, never fatal for the GPU number
                e2e_res = {"error": repr(e)}
        cpu = None
        if not a.no_cpu_baseline and world == 1:
            try:
                cpu = cpu_baseline(a.cpu_seconds, a.workload, HUFF)
            except Exception as e:  # reported, never fatal for the GPU number
                cpu = {"value": None, "error": repr(e)}
        content = {"testsrc": "testsrc2-like generator", "natural": "fractal (1/f) value noise",
                   "noise-patches": "testsrc2-like with 1/8 of the macroblocks uniform noise"}[a.content]
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "prewarm": {"ms": a.prewarm_ms, "steps": prewarm,
                        "why": "untimed steps before the W warmup steps: the GPU runs at its idle clocks "
                               "for the first ~0.3 s of load (DESIGN §6)"},
            "ms_per_step": round(dt / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": f"synthetic: {content}, frames resident in HBM ({pool_n} distinct per GPU), "
                    "output packed in HBM",
            "config": {"workload": WTEXT, "content": a.content, "width": W, "height": H,
                       "dst_width": DW, "dst_height": DH, "qscale": Q, "frames_per_step": seg,
                       "global_batch": seg * world, "parallelism": f"segment-dp{world}",
                       "profile": (f"-vf scale={DW}:{DH}:flags=bicubic " if (DW, DH) != (W, H) else "")
                       + f"-c:v mjpeg -q:v {Q} -dct int -huffman {HUFF} -bitexact"
                       + (" -slices 8" if a.rst else ""),
                       **({"scale_kernels": "k_scale + k_encode"}
                          if (DW, DH) != (W, H) else {}),
                       "dct": "VALU (k_encode<.., optimal counting pass>)" if HUFF == "optimal" else
                              "VALU (row_pass + column_screen)"},
            "roofline": primary,
            "roofline_kernels": per_kernel,
            "kernel_ms_per_step": {k: round(v, 4) for k, v in kt.items()},
            "mean_jpeg_bytes": round(mean_jpeg, 1),
            "e2e": e2e_res,
            "segments_per_launch": batched,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    enc.close()
    if world > 1:
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
