"""Per-segment time of `worker --serve` (tool), and where it goes: P server processes are
started one after another; each encodes R copies of one segment, requests sent one at a
time (the dispatcher's pattern).  Workers run with MJG_WORKER_TRACE=1, so every segment
also reports its reader / submit / sync / fetch / mux seconds and the process's CPU and
NUMA placement (and the GPU's NUMA node); MJG_NUMA_BIND=0 turns the worker's binding off.
    python tools/serve_latency.py c1d 250 --servers 6 --reps 4 [--no-bind]"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import e2e_worker as E  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("workload")
ap.add_argument("frames", type=int)
ap.add_argument("--servers", type=int, default=4)
ap.add_argument("--reps", type=int, default=4)
ap.add_argument("--no-bind", action="store_true")
ap.add_argument("--dir", default=None)
a = ap.parse_args()
w, h, fps, args = E.WORKLOADS[a.workload]
d = tempfile.mkdtemp(dir=a.dir)
seg = os.path.join(d, "seg.mkv")
E.make_segment(seg, w, h, fps, a.frames, full_range=a.workload in E.FULL_RANGE)
argv = [sys.executable, "-m", "ffmpeg_distributed_amd.worker", "--device", "0", *args, "--serve"]
env = dict(os.environ, MJG_WORKER_TRACE="1", MJG_NUMA_BIND="0" if a.no_bind else "1")

for s in range(a.servers):
    p = subprocess.Popen(argv, stdin=subprocess.PIPE, stderr=subprocess.PIPE, stdout=subprocess.DEVNULL,
                         universal_newlines=True, bufsize=1, cwd=ROOT, env=env)
    times, traces = [], []
    for i in range(a.reps):
        t0 = time.monotonic()
        p.stdin.write(json.dumps([seg, f"{d}/o{s}_{i}.mkv"]) + "\n")
        p.stdin.flush()
        for line in p.stderr:
            if line.startswith("mjg-trace:"):
                traces.append(line.split(":", 1)[1].strip())
            if line.startswith("mjg-serve: segment done"):
                times.append(round(time.monotonic() - t0, 4))
                break
        else:
            raise SystemExit("server exited")
    p.stdin.close()
    p.wait()
    print(f"{a.workload} {a.frames} server {s} bind={not a.no_bind} seconds {times}", flush=True)
    for t in traces[1:]:
        print("   ", t, flush=True)
for f in os.listdir(d):
    os.remove(os.path.join(d, f))
os.rmdir(d)
