"""Per-segment time of `worker --serve` (tool): requests one at a time (the dispatcher's
pattern) vs all at once, and in-process serve() for comparison.
    python tools/serve_latency.py c1d 250 5"""
import io
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import e2e_worker as E  # noqa: E402

wl, frames, reps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
w, h, fps, args = E.WORKLOADS[wl]
d = tempfile.mkdtemp()
seg = os.path.join(d, "seg.mkv")
E.make_segment(seg, w, h, fps, frames, full_range=wl in E.FULL_RANGE)
argv = [sys.executable, "-m", "ffmpeg_distributed_amd.worker", "--device", "0", *args, "--serve"]


def done_lines(p, k):
    t = []
    for line in p.stderr:
        if line.startswith("mjg-serve: segment done"):
            t.append(time.monotonic())
            if len(t) == k:
                return t
    raise SystemExit("server exited")


p = subprocess.Popen(argv, stdin=subprocess.PIPE, stderr=subprocess.PIPE, stdout=subprocess.DEVNULL,
                     universal_newlines=True, bufsize=1, cwd=ROOT)
one = []
for i in range(reps):
    t0 = time.monotonic()
    p.stdin.write(f"{seg}\t{d}/o{i}.mkv\n")
    p.stdin.flush()
    one.append(done_lines(p, 1)[0] - t0)
t0 = time.monotonic()
p.stdin.write("".join(f"{seg}\t{d}/p{i}.mkv\n" for i in range(reps)))
p.stdin.flush()
ts = done_lines(p, reps)
allat = [b - a for a, b in zip([t0] + ts[:-1], ts)]
p.stdin.close()
p.wait()
from ffmpeg_distributed_amd import worker  # noqa: E402
err = io.StringIO()
t0 = time.monotonic()
worker.serve(0, args, requests=io.StringIO("".join(f"{seg}\t{d}/q{i}.mkv\n" for i in range(reps))), stderr=err)
inproc = time.monotonic() - t0
print(wl, frames, "one-at-a-time", [round(x, 3) for x in one])
print(wl, frames, "all-at-once", [round(x, 3) for x in allat])
print(wl, frames, "in-process total incl. init", round(inproc, 3))
for f in os.listdir(d):
    os.remove(os.path.join(d, f))
os.rmdir(d)
