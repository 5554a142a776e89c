"""cProfile of worker.serve over N copies of one synthetic raw segment (tool).
    python tools/profile_serve.py c1d 250 4"""
import cProfile
import io
import os
import pstats
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import e2e_worker as E  # noqa: E402
from ffmpeg_distributed_amd import worker  # noqa: E402

wl, frames, reps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
w, h, fps, args = E.WORKLOADS[wl]
d = tempfile.mkdtemp()
seg = os.path.join(d, "seg.mkv")
E.make_segment(seg, w, h, fps, frames, full_range=wl in E.FULL_RANGE)
reqs = io.StringIO("".join(f"{seg}\t{d}/out{i}.mkv\n" for i in range(reps)))
err = io.StringIO()
pr = cProfile.Profile()
pr.enable()
worker.serve(0, args, requests=reqs, stderr=err)
pr.disable()
print(err.getvalue().count("rc=0"), "segments ok")
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(18)
for f in os.listdir(d):
    os.remove(os.path.join(d, f))
os.rmdir(d)
