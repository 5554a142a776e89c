"""Segment dispatcher: the reference's split -> per-host worker queue -> concat flow
(Rouji/ffmpeg_distributed, ffmpeg_distributed.py:150-236) with one addition: a host
named `gpu:N` runs a local per-segment process instead of `ssh HOST ffmpeg ...`:
`mjg_client --device N --python PY -- <remote_args>` (csrc/mjg_client.c), which hands its
stdin / stdout / stderr to GPU N's resident encoder (resident.py), or, when the client is
not built or MJG_RESIDENT=0, `python -m ffmpeg_distributed_amd.worker --device N
<remote_args>` (worker_argv; INTEGRATION.md §1 is the same argv as a patch to the
reference, pinned by the gpu_* fixtures).

Everything observable is kept as in the reference and pinned by
tests/golden/reference_dispatch.json (captured from the reference itself):
  * split argv (ffmpeg_distributed.py:166-177), skipped on resume when tmp/in is non-empty
    (:164-165); a failed split prints stderr and returns with exit status 0 (:181-183);
  * queue = sorted tmp/in/* whose tmp/out counterpart does not exist (:185-190);
  * one worker thread per -H entry pulling from one queue (:105-148); worker argv
    `nice -n10 ionice -c3 ffmpeg -f matroska -i pipe: ARGS -f matroska pipe:`, through
    `ssh HOST "<shlex.join>"` unless HOST is localhost (:131-138); a nonzero exit reports
    stderr and re-queues the segment, with no retry cap (:142-145);
  * CWD/output_segments.txt with `file '<path>'` lines and no trailing newline (:209-210);
  * concat argv (:216-227); the list file is removed and tmp deleted unless -k (:233-236);
  * progress / duration parsing of ffmpeg stderr (:39-40, :59-91).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import queue
import re
import shlex
import shutil
import signal
import subprocess
import sys
import threading
import time
from dataclasses import dataclass, field
from glob import glob
from typing import Callable, List, Optional

try:
    from tqdm import tqdm
except ImportError:  # progress bars are cosmetic
    tqdm = None

GPU_HOST = re.compile(r"^gpu:(\d+)$")

# ffmpeg stderr grammar the reference parses (ffmpeg_distributed.py:39-40)
_HMS = r"(?P<h>\d+):(?P<m>\d+):(?P<s>[\d.]+)"
DURATION_RE = re.compile(r".*Duration:\s*-?" + _HMS + ",")
PROGRESS_RE = re.compile(r"frame=\s*(?P<frame>\d+)\s+fps=\s*(?P<fps>\d+).*time=-?(?P<h>\d+):(?P<m>\d+):"
                         r"(?P<s>[\d,.]+)\s+.*speed=(?P<speed>[\d.]+)x")


def _seconds(m) -> float:
    return int(m.group("h")) * 3600 + int(m.group("m")) * 60 + float(m.group("s"))


def parse_progress(line: str):
    """(frame, fps, time_s, speed) of an ffmpeg progress line, else None."""
    m = PROGRESS_RE.match(line)
    if not m:
        return None
    return int(m.group("frame")), int(m.group("fps")), _seconds(m), float(m.group("speed"))


def parse_duration(line: str) -> Optional[float]:
    m = DURATION_RE.match(line)
    return _seconds(m) if m else None


@dataclass(frozen=True)
class Task:
    """One segment: input file, output file, worker arguments (fd.py:33-36)."""
    input_file: str
    output_file: str
    ffmpeg_args: List[str] = field(default_factory=list)


class _LineFeed:
    """Lines of a text pipe (universal newlines: ffmpeg ends progress lines with \\r),
    read by a daemon thread into a queue so the follower can wait with a timeout and
    notice stop() promptly, as the reference's select.poll loop does (fd.py:61-68)."""

    _EOF = object()

    def __init__(self, pipe):
        self.q: "queue.Queue" = queue.Queue()
        self.eof = False
        threading.Thread(target=self._pump, args=(pipe,), daemon=True).start()

    def _pump(self, pipe):
        try:
            for line in pipe:
                self.q.put(line)
        except (OSError, ValueError):
            pass
        self.q.put(self._EOF)

    def get(self, timeout: float):
        """The next line, None on timeout; sets .eof (and returns None) at end of stream."""
        try:
            item = self.q.get(timeout=timeout)
        except queue.Empty:
            return None
        if item is self._EOF:
            self.eof = True
            return None
        return item


class FFMPEGProc:
    """Runs one command with stdin/stdout redirected, follows its stderr: progress lines
    go to `update_callback(frame, fps, time_s, duration_s, speed)`, every other line is
    kept in `.stderr` (reported if the command fails).  stop() only stops following
    (the reference never kills the child either, fd.py:56-57); it takes effect within
    0.1 s even while the child writes nothing (fd.py:61-68 polls stderr with a timeout)."""

    def __init__(self, cmd, shell=False, stdin=subprocess.DEVNULL, stdout=subprocess.DEVNULL,
                 update_callback: Optional[Callable] = None, env=None):
        self.cmd = cmd
        self.shell = shell
        self.stdin = stdin
        self.stdout = stdout
        self.update_callback = update_callback
        self.env = env
        self.duration: Optional[float] = None
        self.stderr = ""
        self._stop = threading.Event()
        self.proc: Optional[subprocess.Popen] = None

    def stop(self):
        self._stop.set()

    def _line(self, line: str):
        prog = parse_progress(line)
        if prog is None:
            self.stderr += line
            if self.duration is None:
                self.duration = parse_duration(line)
        elif self.update_callback:
            frame, fps, t, speed = prog
            self.update_callback(frame, fps, t, self.duration, speed)

    def run(self) -> int:
        self.proc = subprocess.Popen(self.cmd, shell=self.shell, stdin=self.stdin, stdout=self.stdout,
                                     stderr=subprocess.PIPE, universal_newlines=True, env=self.env)
        feed = _LineFeed(self.proc.stderr)
        while not self._stop.is_set():
            line = feed.get(0.1)
            if line is not None:
                self._line(line)
            elif feed.eof:
                break
        # stderr can reach EOF a moment before the child exits: the reference's loop runs
        # until poll() sees the exit (fd.py:62), so wait for it unless stop() was called
        # (then, like fd.py:85-89, give it one second and report whatever is there)
        if not self._stop.is_set():
            self.proc.wait()
            return self.proc.returncode
        try:
            self.proc.wait(timeout=1)
        except subprocess.TimeoutExpired:
            pass
        while True:
            line = feed.get(0)
            if line is None:
                break
            self.stderr += line
        return self.proc.returncode


def _bar(desc, position=0):
    if tqdm is None:
        return None
    return tqdm(desc=desc, position=position, total=99999999, leave=False, dynamic_ncols=True,
                bar_format="{l_bar}{bar}|{n:.1f}/{total:.1f} [{elapsed}<{remaining}]")


def _bar_to(bar, value, total):
    if bar is None:
        return
    bar.total = total or 999
    bar.update(value - bar.n)


def _report(msg: str):
    (tqdm.write if tqdm else print)(msg, file=sys.stderr)


CLIENT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mjg_client")


def resident_enabled() -> bool:
    """gpu:N segments go through mjg_client and the resident encoder (resident.py) when the
    client is built, unless MJG_RESIDENT=0 asks for one Python worker process per segment."""
    return os.environ.get("MJG_RESIDENT", "1") != "0" and os.access(CLIENT, os.X_OK)


def worker_argv(host: str, ffmpeg_args: List[str], resident: Optional[bool] = None) -> List[str]:
    """The per-segment worker command for one -H entry (fd.py:131-138 + gpu:N).  gpu:N:
    `mjg_client` (hands the segment to its GPU's resident encoder; the same stdin / stdout /
    stderr / exit-code contract) or, with resident=False, a `worker` process of its own."""
    g = GPU_HOST.match(host)
    if g:
        if resident if resident is not None else resident_enabled():
            return [CLIENT, "--device", g.group(1), "--python", sys.executable, "--", *ffmpeg_args]
        return [sys.executable, "-m", "ffmpeg_distributed_amd.worker", "--device", g.group(1),
                *ffmpeg_args]
    cmd = ["nice", "-n10", "ionice", "-c3", "ffmpeg", "-f", "matroska", "-i", "pipe:",
           *ffmpeg_args, "-f", "matroska", "pipe:"]
    if host != "localhost":
        cmd = ["ssh", host, shlex.join(cmd)]
    return cmd


def server_argv(host: str, ffmpeg_args: List[str]) -> List[str]:
    """The persistent worker for a gpu:N host (--persistent-gpu-workers): worker.serve."""
    return worker_argv(host, ffmpeg_args, resident=False) + ["--serve"]


SERVE_DONE = "mjg-serve: segment done rc="


def serve_request(input_file: str, output_file: str) -> str:
    """One worker.serve request line: the two absolute paths as a JSON array, so any path
    (tabs, newlines, quotes) survives the one-line-per-segment protocol."""
    return json.dumps([os.path.abspath(input_file), os.path.abspath(output_file)]) + "\n"


class GpuServer:
    """One long-lived `worker --serve` process per gpu:N TaskThread.  run_task hands it one
    segment (a request line with the input and output paths) and follows its stderr like
    FFMPEGProc follows a per-segment worker, up to the segment's done line; its exit code is
    the segment's.  A server that dies fails the segment (re-queued by the caller, as for a
    failed per-segment worker) and is started again for the next one.  A stop event set
    while a segment runs closes the server and fails the segment."""

    def __init__(self, host: str):
        self.host = host
        self.proc: Optional[subprocess.Popen] = None
        self.feed: Optional[_LineFeed] = None
        self.args: Optional[List[str]] = None
        self.stderr = ""
        self.duration: Optional[float] = None

    def _start(self, ffmpeg_args: List[str]):
        self.close()
        self.args = list(ffmpeg_args)
        self.proc = subprocess.Popen(server_argv(self.host, ffmpeg_args), stdin=subprocess.PIPE,
                                     stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                                     universal_newlines=True, bufsize=1)
        self.feed = _LineFeed(self.proc.stderr)

    def run_task(self, task: "Task", update_callback: Optional[Callable] = None,
                 stop: Optional[threading.Event] = None) -> int:
        if self.proc is None or self.proc.poll() is not None or self.args != list(task.ffmpeg_args):
            self._start(task.ffmpeg_args)
        self.stderr, self.duration = "", None
        try:
            self.proc.stdin.write(serve_request(task.input_file, task.output_file))
            self.proc.stdin.flush()
        except (BrokenPipeError, OSError):
            self.stderr = f"{self.host}: worker server is gone\n"
            self.close()
            return 1
        while True:
            if stop is not None and stop.is_set():
                self.stderr += f"{self.host}: stopped\n"
                self.close(kill=True)
                return 1
            line = self.feed.get(0.1)
            if line is None:
                if self.feed.eof:
                    break
                continue
            if line.startswith(SERVE_DONE):
                return int(line[len(SERVE_DONE):].strip() or 1)
            prog = parse_progress(line)
            if prog is None:
                self.stderr += line
                if self.duration is None:
                    self.duration = parse_duration(line)
            elif update_callback:
                frame, fps, t, speed = prog
                update_callback(frame, fps, t, self.duration, speed)
        rc = self.proc.wait()
        self.stderr += f"{self.host}: worker server exited with {rc}\n"
        self.proc = None
        return rc or 1

    def close(self, kill: bool = False):
        if self.proc is not None:
            try:
                self.proc.stdin.close()
            except OSError:
                pass
            if kill and self.proc.poll() is None:
                self.proc.kill()
            self.proc.wait()
            self.proc = None


class TaskThread(threading.Thread):
    """One consumer per -H entry: pulls segments until the queue is empty and re-queues
    any segment whose worker exits nonzero (fd.py:105-148)."""

    def __init__(self, host: str, task_queue: "queue.SimpleQueue[Task]", bar_pos: int = 0,
                 persistent: bool = False):
        super().__init__(daemon=True)
        self.host = host
        # gpu:N with --persistent-gpu-workers: segments go to one long-lived worker
        self.server = GpuServer(host) if persistent and GPU_HOST.match(host) else None
        self.tasks = task_queue
        self.bar = _bar(host, bar_pos)
        self.current = None
        self._proc: Optional[FFMPEGProc] = None
        self._stop_evt = threading.Event()
        self.done: List[str] = []
        self.failures = 0

    def stop(self):
        self._stop_evt.set()
        if self._proc:
            self._proc.stop()

    def _progress(self, frame, fps, t, duration, speed):
        if self.bar is not None:
            self.bar.desc = f"{self.host}: {self.current}"
            _bar_to(self.bar, t, duration)

    def run(self):
        while not self._stop_evt.is_set():
            try:
                task = self.tasks.get(False)
            except queue.Empty:
                break
            self.current = os.path.basename(task.input_file)
            if self.server is not None:
                rc = self.server.run_task(task, self._progress, self._stop_evt)
                err = self.server.stderr
            else:
                with open(task.input_file, "rb") as src, open(task.output_file, "wb") as dst:
                    self._proc = FFMPEGProc(worker_argv(self.host, task.ffmpeg_args), stdin=src,
                                            stdout=dst, update_callback=self._progress)
                    rc = self._proc.run()
                err = self._proc.stderr
            if rc != 0:
                self.failures += 1
                _report(f"task for {self.current} failed on host {self.host}")
                _report(err)
                self.tasks.put(task)
            else:
                self.done.append(task.input_file)
        if self.server is not None:
            self.server.close()
        if self.bar is not None:
            self.bar.close()


def split_argv(input_file, segment_seconds, tmp_in, copy_input):
    codec = ["copy"] if copy_input else ["libx264", "-crf", "0", "-preset", "ultrafast", "-bf", "0"]
    return ["ffmpeg", "-i", input_file, "-an", "-sn", "-c:v", *codec, "-f", "segment",
            "-reset_timestamps", "1", "-segment_time", str(segment_seconds) + "s",
            tmp_in + "/%08d.mkv"]


def concat_argv(input_file, output_file, concat_args):
    return ["ffmpeg", "-i", input_file, "-f", "concat", "-safe", "0", "-i", "output_segments.txt",
            "-map_metadata", "0:g", "-map", "1:v", "-map", "0:a?", "-map", "0:s?",
            "-c:v", "copy", "-c:s", "copy", *shlex.split(concat_args), "-y", output_file]


def _run_local(argv, desc) -> FFMPEGProc:
    bar = _bar(desc)
    proc = FFMPEGProc(argv, update_callback=lambda f, fps, t, d, s: _bar_to(bar, t, d))
    proc.returncode = proc.run()
    if bar is not None:
        bar.close()
    return proc


def encode(hosts: List[str], input_file: str, output_file: str, segment_seconds: float = 60,
           remote_args: str = "", concat_args: str = "", tmp_dir: Optional[str] = None,
           keep_tmp: bool = False, resume: bool = False, copy_input: bool = False,
           persistent_gpu_workers: bool = False):
    """Split -> distributed per-segment encode -> concat (fd.py:150-236)."""
    input_file = os.path.abspath(os.path.expanduser(input_file))
    output_file = os.path.abspath(os.path.expanduser(output_file))
    tmp_dir = tmp_dir or "ffmpeg_segments_" + hashlib.md5(input_file.encode()).hexdigest()
    tmp_in, tmp_out = f"{tmp_dir}/in", f"{tmp_dir}/out"
    for d in (tmp_dir, tmp_in, tmp_out):
        try:
            os.mkdir(d)
        except FileExistsError:
            if not resume:
                raise

    if not resume or not os.listdir(tmp_in):
        proc = _run_local(split_argv(input_file, segment_seconds, tmp_in, copy_input),
                          "splitting input file")
        if proc.returncode != 0:
            _report(proc.stderr)
            return

    tasks: "queue.SimpleQueue[Task]" = queue.SimpleQueue()
    args = shlex.split(remote_args)
    for seg in sorted(glob(tmp_in + "/*")):
        out = f"{tmp_out}/{os.path.basename(seg)}"
        if not os.path.isfile(out):
            tasks.put(Task(seg, out, list(args)))

    threads = [TaskThread(h, tasks, pos, persistent_gpu_workers) for pos, h in enumerate(hosts)]

    def on_sigint(sig, frame):
        print("Got SIGINT, stopping...")
        for t in threads:
            t.stop()
        for t in threads:
            t.join()
        sys.exit(1)

    if threading.current_thread() is threading.main_thread():
        signal.signal(signal.SIGINT, on_sigint)
    for t in threads:
        t.start()
    for t in threads:
        t.join()

    with open("output_segments.txt", "w") as f:
        f.write("\n".join(f"file '{p}'" for p in sorted(glob(tmp_out + "/*"))))

    proc = _run_local(concat_argv(input_file, output_file, concat_args), "concatenating output segments")
    if proc.returncode != 0:
        _report(proc.stderr)
        return
    os.unlink("output_segments.txt")
    if not keep_tmp:
        shutil.rmtree(tmp_dir)


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(
        description="Splits a file into segments and processes them on multiple hosts in parallel "
                    "using ffmpeg over SSH, or on local MI355X GPUs (-H gpu:N).")
    p.add_argument("input_file", help="File to encode.")
    p.add_argument("output_file", help="Path to encoded output file.")
    p.add_argument("remote_args", help='Arguments to pass to the remote ffmpeg instances. For example: '
                                       '"-c:v libx264 -crf 23 -preset fast"')
    p.add_argument("concat_args", default="", help="Arguments to pass to the local ffmpeg "
                   "concatenating the processed video segments and muxing it with the original "
                   'audio/subs/metadata. Mainly useful for audio encoding options, or "-an" to get rid of it.')
    p.add_argument("-s", "--segment-length", type=float, default=10, help="Segment length in seconds.")
    p.add_argument("-H", "--host", action="append", required=True,
                   help='SSH hostname(s) to encode on. Use "localhost" to include the machine you\'re '
                        'running this from, "gpu:N" for local GPU N. Can include username.')
    p.add_argument("-k", "--keep-tmp", action="store_true",
                   help="Keep temporary segment files instead of deleting them on successful exit.")
    p.add_argument("-r", "--resume", action="store_true",
                   help="Don't split the input file again, keep existing segments and only process "
                        "the missing ones.")
    p.add_argument("-t", "--tmp-dir", default=None, help="Directory to use for temporary files. "
                   "Should not already exist and will be deleted afterwards.")
    p.add_argument("-c", "--copy-input", action="store_true",
                   help="Don't (losslessly) re-encode input while segmenting. Only use this if your "
                        'input segments frame-perfectly with "-c:v copy" (i.e. it has no B-frames)')
    p.add_argument("-P", "--persistent-gpu-workers", action="store_true",
                   help="gpu:N hosts: one long-lived worker per -H entry encodes every segment it "
                        "pulls (no per-segment process start, HIP init and buffer allocation).")
    return p


def main(argv=None):
    a = build_parser().parse_args(argv)
    encode(a.host, a.input_file, a.output_file, segment_seconds=a.segment_length,
           remote_args=a.remote_args, concat_args=a.concat_args, tmp_dir=a.tmp_dir,
           keep_tmp=a.keep_tmp, resume=a.resume, copy_input=a.copy_input,
           persistent_gpu_workers=a.persistent_gpu_workers)


if __name__ == "__main__":
    main()
