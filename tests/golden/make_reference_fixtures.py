#!/usr/bin/env python3
"""Generate tests/golden/reference_dispatch.json by running the REAL reference
(/root/reference/ffmpeg_distributed.py) under the fake ffmpeg/ssh/ionice shims in
tests/shims, in this container (the reference never travels to the GPU box).

Captured behaviour (normalised paths): split / worker / concat argv, the concat list
file, the final output, exit status, retry on a failing worker, resume (-r) with a
partial output, split failure, copy-input (-c), and the progress / duration regex
parse of sample stderr lines (reference FFMPEGProc, imported read-only).

`gpu_*` scenarios run the reference *with INTEGRATION.md's patch applied* (the python block
after "replacing lines 131-138", spliced over ffmpeg_distributed.py:131-138 into a temporary
copy; the reference itself is never written) and a stand-in `ffmpeg_distributed_amd`
package on PYTHONPATH whose `mjg_client` / `worker` log their argv like the ffmpeg shim: the
argv a maintainer's patched reference builds for `-H gpu:N`, which tests/test_dispatcher.py
compares with dispatcher.worker_argv.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_reference_fixtures.py
"""
import importlib.util
import json
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
SHIMS = os.path.join(os.path.dirname(HERE), "shims")
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/ffmpeg_distributed.py"
PATCHED_LINES = (131, 138)  # TaskThread.run's argv construction, replaced by INTEGRATION.md §1

REMOTE = "-c:v mjpeg -q:v 5 -dct int -huffman default -bitexact"

SCENARIOS = {
    "basic_two_hosts": {"args": ["-s", "2", "-H", "localhost", "-H", "user@hostB", "-k", "-t", "segs",
                                 "--", "input.mp4", "out.mkv", REMOTE, "-an"]},
    "retry_once": {"args": ["-s", "2", "-H", "localhost", "-k", "-t", "segs", "--", "input.mp4",
                            "out.mkv", REMOTE, "-an"],
                   "env": {"SHIM_FAIL_ONCE": "{tmp}/failed.marker", "SHIM_FAIL_MATCH": "SEG1:"}},
    "resume_partial": {"args": ["-r", "-H", "localhost", "-t", "segs", "--", "input.mp4", "out.mkv",
                                REMOTE, ""],
                       "pre": {"segs/in/00000000.mkv": "SEG0:input.mp4", "segs/in/00000001.mkv": "SEG1:input.mp4",
                               "segs/in/00000002.mkv": "SEG2:input.mp4", "segs/out/00000001.mkv": "PARTIAL"}},
    "split_fails": {"args": ["-H", "localhost", "-t", "segs", "--", "input.mp4", "out.mkv", REMOTE, ""],
                    "env": {"SHIM_SPLIT_FAIL": "1"}},
    "copy_input_default_tmp": {"args": ["-c", "-s", "0.5", "-H", "localhost", "--", "input.mp4",
                                        "out.mkv", REMOTE, "-an"],
                               "env": {"SHIM_SEGMENTS": "3"}},
    "scale_profile": {"args": ["-s", "2", "-H", "localhost", "-H", "localhost", "-t", "segs", "--",
                               "input.mp4", "out.mkv",
                               "-vf scale=1920:1080:flags=bicubic -c:v mjpeg -q:v 3 -dct int -huffman default -bitexact",
                               "-an"],
                      "env": {"SHIM_SEGMENTS": "4"}},
    # the INTEGRATION.md patch: gpu:N hosts through mjg_client, and its fallback
    "gpu_resident": {"args": ["-s", "2", "-H", "gpu:0", "-H", "gpu:1", "-t", "segs", "--", "input.mp4",
                              "out.mkv", REMOTE, "-an"], "patched": True},
    "gpu_worker_fallback": {"args": ["-s", "2", "-H", "gpu:3", "-t", "segs", "--", "input.mp4", "out.mkv",
                                     REMOTE, "-an"], "patched": True, "env": {"MJG_RESIDENT": "0"}},
}

# stand-in for the package the patched reference imports: its mjg_client and worker module
# behave like the ffmpeg shim's worker role and log the argv they were started with
_STANDIN = r"""import json, os, sys
argv = list(sys.orig_argv) if sys.argv[0].endswith("worker.py") else list(sys.argv)
with open(os.environ["SHIM_LOG"], "a") as f:
    f.write(json.dumps({"prog": os.path.basename(sys.argv[0]), "argv": argv}) + "\n")
data = sys.stdin.read()
sys.stderr.write("  Duration: 00:00:10.00, start: 0.000000, bitrate: N/A\n")
sys.stderr.write("frame=  100 fps= 25 q=-0.0 Lsize=N/A time=00:00:04.00 bitrate=N/A speed=2.00x\n")
sys.stdout.write("GPU[" + data + "]")
"""


def integration_patch():
    """The python block of INTEGRATION.md §1 (after 'replacing lines 131-138'), without its
    comment line."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    i = text.index("# ffmpeg_distributed.py, TaskThread.run, replacing lines 131-138")
    block = text[i:text.index("```", i)]
    return [l for l in block.splitlines()[1:] if l.strip()]


def patched_reference(tmp):
    """A copy of the reference with INTEGRATION.md's patch over lines 131-138, plus the
    stand-in package; returns (script path, PYTHONPATH entry)."""
    lines = open(REF).read().split("\n")
    a, b = PATCHED_LINES
    indent = lines[a - 1][:len(lines[a - 1]) - len(lines[a - 1].lstrip())]
    assert lines[a - 1].strip() == "ffmpeg_cmd = [" and lines[b - 1].strip().startswith("ffmpeg_cmd = ['ssh'")
    lines[a - 1:b] = [indent + l for l in integration_patch()]
    src = os.path.join(tmp, "fd_patched", "ffmpeg_distributed.py")
    pkg = os.path.join(tmp, "fd_patched", "pkg", "ffmpeg_distributed_amd")
    os.makedirs(pkg)
    with open(src, "w") as f:
        f.write("\n".join(lines))
    open(os.path.join(pkg, "__init__.py"), "w").close()
    with open(os.path.join(pkg, "worker.py"), "w") as f:
        f.write(_STANDIN)
    with open(os.path.join(pkg, "mjg_client"), "w") as f:
        f.write("#!" + sys.executable + "\n" + _STANDIN)
    os.chmod(os.path.join(pkg, "mjg_client"), 0o755)
    return src, os.path.dirname(pkg)

PROGRESS_LINES = [
    "frame=   42 fps= 21 q=-0.0 size=N/A time=00:00:05.00 bitrate=N/A speed=2.5x",
    "frame=  100 fps= 25 q=-0.0 Lsize=N/A time=00:00:04.00 bitrate=N/A speed=2.00x",
    "frame= 3600 fps=120 q=2.0 size=  123456kB time=00:01:00.00 bitrate=16853.9kbits/s speed=2.01x elapsed=0:00:29.80",
    "frame=    0 fps=0.0 q=0.0 size=       0kB time=N/A bitrate=N/A speed=N/A",
    "frame=   10 fps=5 q=3.0 size=1kB time=-00:00:00.03 bitrate=N/A speed=0.1x",
    "Input #0, matroska,webm, from 'pipe:':",
    "  Duration: 01:02:03.50, start: 0.000000, bitrate: N/A",
    "  Duration: N/A, start: 0.000000, bitrate: N/A",
    "  Duration: -00:00:01.00, start: 0.000000",
]


def norm(x, tmp):
    if isinstance(x, str):
        x = x.replace(os.path.join(tmp, "fd_patched", "pkg", "ffmpeg_distributed_amd"), "<PKG>")
        return x.replace(tmp, "<TMP>").replace(sys.executable, "<PYTHON>")
    if isinstance(x, list):
        return [norm(v, tmp) for v in x]
    if isinstance(x, dict):
        return {k: norm(v, tmp) for k, v in x.items()}
    return x


def run_scenario(name, sc, program):
    tmp = tempfile.mkdtemp(prefix="fdref_")
    try:
        with open(os.path.join(tmp, "input.mp4"), "w") as f:
            f.write("RAWINPUT")
        for rel, body in sc.get("pre", {}).items():
            p = os.path.join(tmp, rel)
            os.makedirs(os.path.dirname(p), exist_ok=True)
            with open(p, "w") as f:
                f.write(body)
        env = dict(os.environ, PATH=SHIMS + os.pathsep + os.environ["PATH"], PYTHONDONTWRITEBYTECODE="1",
                   SHIM_LOG=os.path.join(tmp, "shim.log"), SHIM_DIR=tmp)
        env.pop("MJG_RESIDENT", None)
        if sc.get("patched"):
            script, pypath = patched_reference(tmp)
            program = [sys.executable, script]
            env["PYTHONPATH"] = pypath
        for k, v in sc.get("env", {}).items():
            env[k] = v.replace("{tmp}", tmp)
        p = subprocess.run(program + sc["args"], cwd=tmp, env=env, capture_output=True, text=True,
                           timeout=120)
        calls = []
        if os.path.exists(env["SHIM_LOG"]):
            calls = [json.loads(l) for l in open(env["SHIM_LOG"])]
        out = os.path.join(tmp, "out.mkv")
        tree = sorted(os.path.relpath(os.path.join(d, f), tmp) for d, _, fs in os.walk(tmp) for f in fs
                      if not os.path.relpath(d, tmp).startswith("fd_patched"))
        res = {
            "returncode": p.returncode,
            "calls": calls,
            "concat_list": open(os.path.join(tmp, "concat_list_copy.txt")).read()
            if os.path.exists(os.path.join(tmp, "concat_list_copy.txt")) else None,
            "output": open(out).read() if os.path.exists(out) else None,
            "files_after": [t for t in tree if t not in ("shim.log", "concat_list_copy.txt")],
            "stderr_has_failure_report": "failed on host" in p.stderr,
        }
        return norm(res, tmp)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def regex_fixture():
    spec = importlib.util.spec_from_file_location("fd_reference", REF)
    mod = importlib.util.module_from_spec(spec)
    sys.dont_write_bytecode = True
    spec.loader.exec_module(mod)
    P = mod.FFMPEGProc
    out = []
    for line in PROGRESS_LINES:
        m = P._progress_re.match(line)
        d = P._duration_re.match(line)
        out.append({
            "line": line,
            "progress": None if not m else [int(m.group("frame")), int(m.group("fps")),
                                            P._match_to_sec(m), float(m.group("speed"))],
            "duration": None if not d else P._match_to_sec(d),
        })
    return out


def main():
    program = [sys.executable, REF]
    fx = {"reference": "Rouji/ffmpeg_distributed @ /root/reference/ffmpeg_distributed.py",
          "generator": "tests/golden/make_reference_fixtures.py",
          "remote_args": REMOTE,
          "scenarios": {name: run_scenario(name, sc, program) for name, sc in SCENARIOS.items()},
          "scenario_args": {name: sc["args"] for name, sc in SCENARIOS.items()},
          "scenario_env": {name: sc.get("env", {}) for name, sc in SCENARIOS.items()},
          "scenario_pre": {name: sc.get("pre", {}) for name, sc in SCENARIOS.items()},
          "scenario_patched": {name: bool(sc.get("patched")) for name, sc in SCENARIOS.items()},
          "integration_patch": integration_patch(),
          "progress_regex": regex_fixture()}
    with open(os.path.join(HERE, "reference_dispatch.json"), "w") as f:
        json.dump(fx, f, indent=1, sort_keys=True)
    print("wrote", os.path.join(HERE, "reference_dispatch.json"))


if __name__ == "__main__":
    main()
