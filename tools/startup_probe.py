"""Where a gpu:N worker process spends its start-up (tool): interpreter + imports, HIP
init + library load, encoder context, page-locked batch buffers.  One JSON line."""
import json
import os
import sys
import time

t0 = time.monotonic()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ffmpeg_distributed_amd import worker  # noqa: E402
t_import = time.monotonic()
from ffmpeg_distributed_amd import _lib  # noqa: E402
from ffmpeg_distributed_amd.encoder import MjpegEncoder, PinnedBuffer  # noqa: E402
L = _lib.load()
t_lib = time.monotonic()
w, h = (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "3840x2160").split("x"))
batch = max(1, min(32, worker.BATCH_BYTES // (w * h * 3 // 2)))
enc = MjpegEncoder(0, w, h, qscale=5, max_batch=batch)
t_ctx = time.monotonic()
bufs = [PinnedBuffer(batch * w * h * 3 // 2) for _ in range(3)]
t_pin = time.monotonic()
for b in bufs:
    b.free()
enc.close()
t_close = time.monotonic()
print(json.dumps({"size": f"{w}x{h}", "batch": batch, "imports_s": round(t_import - t0, 3),
                  "lib_and_hip_s": round(t_lib - t_import, 3), "context_s": round(t_ctx - t_lib, 3),
                  "pinned_3_batches_s": round(t_pin - t_ctx, 3), "teardown_s": round(t_close - t_pin, 3)}))
