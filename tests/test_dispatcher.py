"""Dispatcher parity with the reference, pinned by fixtures captured from the real
reference (tests/golden/make_reference_fixtures.py -> reference_dispatch.json) under
the same fake ffmpeg/ssh/ionice shims (tests/shims)."""
import hashlib
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

import pytest

from ffmpeg_distributed_amd import dispatcher as D

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SHIMS = os.path.join(HERE, "shims")
FX = json.load(open(os.path.join(HERE, "golden", "reference_dispatch.json")))


def run_ours(name):
    args = FX["scenario_args"][name]
    tmp = tempfile.mkdtemp(prefix="fdours_")
    try:
        with open(os.path.join(tmp, "input.mp4"), "w") as f:
            f.write("RAWINPUT")
        for rel, body in FX["scenario_pre"][name].items():
            p = os.path.join(tmp, rel)
            os.makedirs(os.path.dirname(p), exist_ok=True)
            with open(p, "w") as f:
                f.write(body)
        env = dict(os.environ, PATH=SHIMS + os.pathsep + os.environ["PATH"],
                   SHIM_LOG=os.path.join(tmp, "shim.log"), SHIM_DIR=tmp,
                   PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
        for k, v in FX["scenario_env"][name].items():
            env[k] = v.replace("{tmp}", tmp)
        p = subprocess.run([sys.executable, "-m", "ffmpeg_distributed_amd.dispatcher", *args], cwd=tmp,
                           env=env, capture_output=True, text=True, timeout=120)
        calls = [json.loads(l) for l in open(env["SHIM_LOG"])] if os.path.exists(env["SHIM_LOG"]) else []
        out = os.path.join(tmp, "out.mkv")
        cl = os.path.join(tmp, "concat_list_copy.txt")
        tree = sorted(os.path.relpath(os.path.join(d, f), tmp) for d, _, fs in os.walk(tmp) for f in fs)
        res = {"returncode": p.returncode, "calls": calls,
               "concat_list": open(cl).read() if os.path.exists(cl) else None,
               "output": open(out).read() if os.path.exists(out) else None,
               "files_after": [t for t in tree if t not in ("shim.log", "concat_list_copy.txt")],
               "stderr_has_failure_report": "failed on host" in p.stderr}
        digest = hashlib.md5(os.path.join(os.path.realpath(tmp), "input.mp4").encode()).hexdigest()
        text = json.dumps(res)
        if "ffmpeg_segments_" in text:  # default tmp dir = ffmpeg_segments_<md5(abs input)>
            assert digest in text or hashlib.md5(os.path.join(tmp, "input.mp4").encode()).hexdigest() in text
        return json.loads(norm_md5(text.replace(os.path.realpath(tmp), "<TMP>").replace(tmp, "<TMP>"))), p.stderr
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def norm_md5(text):
    return re.sub(r"ffmpeg_segments_[0-9a-f]{32}", "ffmpeg_segments_<MD5>", text)


def canon_calls(calls):
    """Split and concat calls in order; worker calls as a multiset (host assignment is
    dynamic pull, so which host ran which segment is not deterministic); ssh hops as the
    set of distinct remote commands (how many segments went through ssh varies per run,
    in the reference as here)."""
    def role(c):
        a = c.get("argv", [])
        if c["prog"] == "ssh":
            return "ssh"
        if "segment" in a:
            return "split"
        if "concat" in a:
            return "concat"
        return "worker"
    seq = [c for c in calls if role(c) in ("split", "concat")]
    workers = sorted(json.dumps({k: v for k, v in c.items() if k != "host"}, sort_keys=True)
                     for c in calls if role(c) == "worker")
    ssh = sorted({c["cmd"] for c in calls if role(c) == "ssh"})
    return seq, workers, ssh


PATCHED = sorted(n for n, v in FX["scenario_patched"].items() if v)


@pytest.mark.parametrize("name", sorted(set(FX["scenarios"]) - set(PATCHED)))
def test_dispatcher_matches_reference(name):
    ref = json.loads(norm_md5(json.dumps(FX["scenarios"][name])))
    ours, err = run_ours(name)
    assert ours["returncode"] == ref["returncode"], err
    assert canon_calls(ours["calls"]) == canon_calls(ref["calls"])
    for key in ("concat_list", "output", "files_after", "stderr_has_failure_report"):
        assert ours[key] == ref[key], key


def test_single_host_call_sequence_is_identical():
    for name in ("retry_once", "resume_partial", "split_fails"):
        ref = FX["scenarios"][name]
        ours, _ = run_ours(name)
        assert ours["calls"] == ref["calls"], name


@pytest.mark.parametrize("case", FX["progress_regex"], ids=lambda c: c["line"][:30])
def test_progress_and_duration_parse_like_reference(case):
    p = D.parse_progress(case["line"])
    assert (None if p is None else [p[0], p[1], pytest.approx(p[2]), pytest.approx(p[3])]) == \
        (None if case["progress"] is None else [case["progress"][0], case["progress"][1],
                                                 pytest.approx(case["progress"][2]),
                                                 pytest.approx(case["progress"][3])])
    d = D.parse_duration(case["line"])
    if case["progress"] is None:  # the reference only looks for Duration on non-progress lines
        assert d == (None if case["duration"] is None else pytest.approx(case["duration"]))


def test_worker_argv():
    args = ["-c:v", "mjpeg", "-q:v", "5"]
    assert D.worker_argv("localhost", args) == ["nice", "-n10", "ionice", "-c3", "ffmpeg", "-f", "matroska",
                                                "-i", "pipe:", *args, "-f", "matroska", "pipe:"]
    ssh = D.worker_argv("me@box", args)
    assert ssh[:2] == ["ssh", "me@box"] and ssh[2].startswith("nice -n10 ionice -c3 ffmpeg -f matroska")
    g = D.worker_argv("gpu:3", args, resident=False)
    assert g == [sys.executable, "-m", "ffmpeg_distributed_amd.worker", "--device", "3", *args]


def test_cli_quirk_copy_flag_needs_double_dash():
    # reference quirk kept: a remote_args string starting with -c is taken by -c/--copy-input
    with pytest.raises(SystemExit):
        D.build_parser().parse_args(["-H", "localhost", "in", "out", "-c:v mjpeg", "-an"])
    a = D.build_parser().parse_args(["-H", "gpu:0", "-H", "gpu:1", "--", "in", "out", "-c:v mjpeg", "-an"])
    assert a.host == ["gpu:0", "gpu:1"] and a.remote_args == "-c:v mjpeg" and a.segment_length == 10


def _integration_patch():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    i = text.index("# ffmpeg_distributed.py, TaskThread.run, replacing lines 131-138")
    return [l for l in text[i:text.index("```", i)].splitlines()[1:] if l.strip()]


def test_integration_patch_is_the_one_pinned():
    """INTEGRATION.md §1's patch is the text the gpu_* fixtures ran inside the reference."""
    assert FX["integration_patch"] == _integration_patch()


@pytest.mark.parametrize("name", PATCHED)
def test_patched_reference_gpu_argv_is_worker_argv(name):
    """The reference patched as INTEGRATION.md says builds, for -H gpu:N, exactly the argv
    dispatcher.worker_argv builds (mjg_client -> the GPU's resident encoder; with
    MJG_RESIDENT=0 one Python worker per segment), and the rest of its flow is unchanged."""
    sc = FX["scenarios"][name]
    resident = FX["scenario_env"][name].get("MJG_RESIDENT", "1") != "0"
    args = __import__("shlex").split(FX["remote_args"])
    workers = [c for c in sc["calls"] if c["prog"] != "ffmpeg"]
    hosts = [FX["scenario_args"][name][i + 1] for i, a in enumerate(FX["scenario_args"][name]) if a == "-H"]
    expect = {}
    for h in hosts:
        argv = D.worker_argv(h, args, resident=resident)
        expect[h] = [a.replace(os.path.dirname(D.CLIENT), "<PKG>") if a == D.CLIENT else
                     "<PYTHON>" if a == sys.executable else a for a in argv]
    assert workers and all(c["argv"] in expect.values() for c in workers), (workers, expect)
    assert len(workers) == sc["output"].count("GPU[")  # one worker per segment, none retried
    assert sc["returncode"] == 0 and not sc["stderr_has_failure_report"]
    # split and concat calls are the unpatched reference's
    base = FX["scenarios"]["basic_two_hosts"]["calls"]
    assert [c for c in sc["calls"] if c["prog"] == "ffmpeg"][0] == base[0]
