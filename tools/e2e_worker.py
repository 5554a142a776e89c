"""End-to-end rate of the `gpu:N` segment worker (SURVEY §8d "end-to-end fps").

Each segment is one fresh worker process, exactly as the dispatcher starts it for a
`-H gpu:0` host (fd.py:131-141: segment mkv on stdin, encoded mkv on stdout, progress on
stderr): process start, HIP init, Matroska parse, H2D, encode, mux, all inside the timed
region.  Input segments are raw V_UNCOMPRESSED I420 Matroska (the splitter's `-c` raw
path), so no host decode runs.  Runs `--seq` segments one after another,
then `--par` workers at once on the same GPU (duplicate `-H gpu:0` entries).

    python tools/e2e_worker.py --workload c2 --frames 120 --seq 3 --par 2

Prints one JSON line.  Tool, not product: the oracle is not used here.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time
from fractions import Fraction

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from ffmpeg_distributed_amd import container  # noqa: E402
from ffmpeg_distributed_amd.testsrc import testsrc2_i420  # noqa: E402

WORKLOADS = {
    "c1": (1920, 1080, Fraction(30), ["-c:v", "mjpeg", "-q:v", "5", "-dct", "int", "-bitexact"]),
    "c1d": (1920, 1080, Fraction(30), ["-c:v", "mjpeg", "-q:v", "5", "-dct", "int", "-huffman", "default",
                                       "-bitexact"]),
    "c2": (3840, 2160, Fraction(60), ["-c:v", "mjpeg", "-q:v", "5", "-dct", "int", "-huffman", "default",
                                      "-bitexact"]),
    "c4": (3840, 2160, Fraction(60), ["-vf", "scale=1920:1080:flags=bicubic", "-c:v", "mjpeg", "-q:v", "3",
                                      "-dct", "int", "-huffman", "default", "-bitexact"]),
    # yuvj420p input (Matroska colour range 2: full)
    "c5": (7680, 4320, Fraction(30), ["-c:v", "mjpeg", "-q:v", "5", "-dct", "int", "-huffman", "default",
                                      "-bitexact"]),
}
FULL_RANGE = {"c5"}


def make_segment(path, w, h, fps, frames, distinct=8, full_range=False):
    pool = [testsrc2_i420(w, h, t, full_range=full_range).tobytes() for t in range(min(distinct, frames))]
    with open(path, "wb") as f:
        wr = container.MkvWriter(f, w, h, fps, codec="V_UNCOMPRESSED", colour_space=b"I420",
                                 colour_range=2 if full_range else 0)
        for i in range(frames):
            wr.write_frame(pool[i % distinct])
        wr.close()


def start(seg, out, args):
    argv = [sys.executable, "-m", "ffmpeg_distributed_amd.worker", "--device", "0", *args]
    return subprocess.Popen(argv, stdin=open(seg, "rb"), stdout=open(out, "wb"),
                            stderr=subprocess.PIPE, cwd=ROOT)


def finish(p):
    _, err = p.communicate()
    if p.returncode != 0:
        sys.stderr.write(err.decode(errors="replace")[-2000:])
        raise SystemExit(f"worker exited {p.returncode}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c2")
    ap.add_argument("--frames", type=int, default=120)
    ap.add_argument("--seq", type=int, default=3)
    ap.add_argument("--par", type=int, default=2)
    ap.add_argument("--dir", default=None)
    ap.add_argument("--persistent", type=int, default=0,
                    help="also time this many segments through one `worker --serve` process (dispatcher -P)")
    a = ap.parse_args()
    w, h, fps, args = WORKLOADS[a.workload]
    d = tempfile.mkdtemp(dir=a.dir)
    seg = os.path.join(d, "seg.mkv")
    t0 = time.monotonic()
    make_segment(seg, w, h, fps, a.frames, full_range=a.workload in FULL_RANGE)
    gen_s = time.monotonic() - t0
    seg_bytes = os.path.getsize(seg)

    seq = []
    for i in range(a.seq):
        out = os.path.join(d, f"out{i}.mkv")
        t = time.monotonic()
        finish(start(seg, out, args))
        seq.append(time.monotonic() - t)
    out_bytes = os.path.getsize(os.path.join(d, "out0.mkv"))
    par_s = None
    if a.par > 1:
        t = time.monotonic()
        ps = [start(seg, os.path.join(d, f"par{i}.mkv"), args) for i in range(a.par)]
        for p in ps:
            finish(p)
        par_s = time.monotonic() - t
    pers = None
    if a.persistent:
        argv = [sys.executable, "-m", "ffmpeg_distributed_amd.worker", "--device", "0", *args, "--serve"]
        p = subprocess.Popen(argv, stdin=subprocess.PIPE, stderr=subprocess.PIPE, stdout=subprocess.DEVNULL,
                             universal_newlines=True, bufsize=1, cwd=ROOT)
        pers = []
        for i in range(a.persistent):
            t = time.monotonic()
            p.stdin.write(json.dumps([seg, os.path.join(d, f"pers{i}.mkv")]) + "\n")
            p.stdin.flush()
            for line in p.stderr:
                if line.startswith("mjg-serve: segment done rc="):
                    if line.strip()[-2:] != "=0":
                        raise SystemExit(line)
                    break
            else:
                raise SystemExit("server exited")
            pers.append(time.monotonic() - t)
        p.stdin.close()
        p.wait()
    # an empty segment: process start + HIP init + context, no frames
    empty = os.path.join(d, "empty.mkv")
    make_segment(empty, w, h, fps, 0, full_range=a.workload in FULL_RANGE)
    t = time.monotonic()
    finish(start(empty, os.path.join(d, "empty_out.mkv"), args))
    startup_s = time.monotonic() - t
    for f in os.listdir(d):
        os.remove(os.path.join(d, f))
    os.rmdir(d)

    best = min(seq)
    print(json.dumps({
        "metric": "end-to-end worker frames/s (one process per segment, raw I420 mkv in, MJPEG mkv out)",
        "workload": a.workload, "size": f"{w}x{h}", "args": " ".join(args), "frames_per_segment": a.frames,
        "segment_mb": round(seg_bytes / 1e6, 1), "out_mb": round(out_bytes / 1e6, 2),
        "seq_seconds": [round(s, 3) for s in seq], "seq_fps_best": round(a.frames / best, 1),
        "par_workers": a.par, "par_seconds": round(par_s, 3) if par_s else None,
        "par_fps": round(a.par * a.frames / par_s, 1) if par_s else None,
        "empty_segment_seconds": round(startup_s, 3),
        "fps_excluding_startup": round(a.frames / max(best - startup_s, 1e-6), 1),
        "input_gbps_excluding_startup": round(seg_bytes / max(best - startup_s, 1e-6) / 1e9, 2),
        "segment_gen_seconds": round(gen_s, 1),
        "persistent_seconds": [round(x, 3) for x in pers] if pers else None,
        "persistent_fps_steady": round(a.frames / (sum(pers[1:]) / (len(pers) - 1)), 1) if pers and len(pers) > 1
        else None,
    }))


if __name__ == "__main__":
    main()
