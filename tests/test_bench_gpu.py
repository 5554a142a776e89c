"""bench.py's output contract on the GPU (the driver parses this line): one short run of the
headline workload in a child process, checked field by field.  The numbers themselves are the
bench's business; here the line's shape, its units and the roofline / traffic bookkeeping."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_line_contract():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "4", "--warmup", "1",
           "--pool", "240", "--prewarm-ms", "0", "--no-cpu-baseline", "--no-e2e"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 4 and d["warmup"] == 1
    assert d["unit"] == "frames/s" and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["dtype"] == "u8" and d["vs_baseline"] is None and d["cpu_baseline"] is None
    seg = d["config"]["frames_per_step"]
    assert seg == 120 and d["config"]["width"] == 3840 and d["config"]["height"] == 2160
    # value is the whole job's frames over the timed steps' wall time
    assert d["value"] == pytest.approx(4 * seg / (d["ms_per_step"] * 4 / 1e3), rel=1e-3)
    rl = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in rl, k
    assert rl["bound"] == "hbm" and rl["unit"] == "GB/s" and rl["peak"] == 8000.0
    assert rl["frac"] == pytest.approx(rl["achieved"] / rl["peak"], rel=1e-3)
    assert 0 < rl["frac"] < 1
    # a JPEG of 4K testsrc at q5 is ~320 KB (the oracle's CPU sweep agrees)
    assert 250e3 < d["mean_jpeg_bytes"] < 400e3
