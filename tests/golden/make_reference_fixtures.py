#!/usr/bin/env python3
"""Generate tests/golden/reference_dispatch.json by running the REAL reference
(/root/reference/ffmpeg_distributed.py) under the fake ffmpeg/ssh/ionice shims in
tests/shims, in this container (the reference never travels to the GPU box).

Captured behaviour (normalised paths): split / worker / concat argv, the concat list
file, the final output, exit status, retry on a failing worker, resume (-r) with a
partial output, split failure, copy-input (-c), and the progress / duration regex
parse of sample stderr lines (reference FFMPEGProc, imported read-only).

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
REF = "/root/reference/ffmpeg_distributed.py"

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
}

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
        return x.replace(tmp, "<TMP>")
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
        for k, v in sc.get("env", {}).items():
            env[k] = v.replace("{tmp}", tmp)
        p = subprocess.run(program + sc["args"], cwd=tmp, env=env, capture_output=True, text=True,
                           timeout=120)
        calls = []
        if os.path.exists(env["SHIM_LOG"]):
            calls = [json.loads(l) for l in open(env["SHIM_LOG"])]
        out = os.path.join(tmp, "out.mkv")
        tree = sorted(os.path.relpath(os.path.join(d, f), tmp) for d, _, fs in os.walk(tmp) for f in fs)
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
          "progress_regex": regex_fixture()}
    with open(os.path.join(HERE, "reference_dispatch.json"), "w") as f:
        json.dump(fx, f, indent=1, sort_keys=True)
    print("wrote", os.path.join(HERE, "reference_dispatch.json"))


if __name__ == "__main__":
    main()
