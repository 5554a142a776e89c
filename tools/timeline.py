#!/usr/bin/env python3
"""Per-step timeline of a bench.py run from its rocprofv3 kernel trace (`rocprofv3
--kernel-trace --output-format csv -- python3 bench.py ...`).

bench.py brackets its timed steps with a tiny marker kernel on torch's stream (`trace_marker`:
torch.cuda._sleep, "spin_kernel" in the trace; bench.py also launches one at set-up, before the
prewarm, which is skipped here: the last three are used): the first runs after the warmup drain,
the second after the timed steps' final sync, the third after the isolated launches.  So the
k_encode dispatches between markers 1 and 2 are exactly the timed region's launches, and those
between markers 2 and 3 the isolated ones (4 of one segment, then 4 of two segments, each
synced).  Reported:
  * the timed launches: count, span E - S of each k_encode, start-to-start period, the gap to
    the next launch's start (negative: it started inside this one's drain);
  * the union of GPU-busy time (every kernel interval, merged) and the region's span, per step;
  * the launch period per step (median period / segments per launch) against the bench
    line's ms_per_step (bench JSON given as the second argument);
  * the isolated launches' k_encode durations (what bench.py's "(isolated ...)" entries time
    with HIP events).
usage: timeline.py trace.csv [bench.json]"""
import csv
import json
import statistics as st
import sys


def load(path):
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def is_encode(name):
    return "k_encode" in name or "k_emit_syms" in name


def main():
    rows = load(sys.argv[1])
    bench = json.load(open(sys.argv[2])) if len(sys.argv) > 2 else None
    marks = [r for r in rows if "spin" in r[2] or "sleep" in r[2]]
    if len(marks) > 3:  # bench.py r05+: a first marker at set-up (loads its code object early)
        marks = marks[-3:]
    if len(marks) < 2:
        sys.exit(f"{sys.argv[1]}: {len(marks)} marker kernels (spin_kernel); need bench.py's trace markers")
    t0, t1 = marks[0][1], marks[1][0]
    region = [r for r in rows if t0 <= r[0] and r[1] <= t1 and "mjg" in r[2]]
    # the last stage of a launch's encode: k_emit_syms (-huffman optimal) / k_encode
    last_stage = "k_emit_syms" if any("k_emit_syms" in r[2] for r in region) else None
    enc = [r for r in region if (last_stage in r[2] if last_stage else is_encode(r[2]))]
    starts = [r[0] for r in enc]
    n = len(enc)
    f = lambda v: (f"median {st.median(v):9.1f}  min {min(v):9.1f}  max {max(v):9.1f} us" if v else "n/a")
    print(f"{sys.argv[1]}")
    print(f"  timed region: {n} encode launches ({'k_emit_syms' if last_stage else 'k_encode'}), "
          f"{len(region)} mjg kernels between the markers")
    span = [(e - s) / 1e3 for s, e, _ in enc]
    per = [(starts[i + 1] - starts[i]) / 1e3 for i in range(n - 1)]
    gap = [(enc[i + 1][0] - enc[i][1]) / 1e3 for i in range(n - 1)]
    print("  encode span E-S               ", f(span))
    print("  start-to-start period          ", f(per))
    print("  next start - this end          ", f(gap))
    busy = union([(s, e) for s, e, _ in region]) / 1e6
    wall = (max(e for _, e, _ in region) - min(s for s, _, _ in region)) / 1e6
    print(f"  GPU-busy union {busy:.3f} ms over a span of {wall:.3f} ms (first kernel start .. last kernel end)")
    if bench:
        steps, mps = bench["steps"], bench["ms_per_step"]
        launches = bench["roofline"].get("launches", n)
        spl = round(steps / max(launches, 1))  # segments per steady launch (1, or 2 merged)
        print(f"  bench: {steps} steps, ms_per_step {mps:.4f}, {launches} launches (segments per steady launch {spl})")
        print(f"  per step: GPU-busy union {busy / steps:.4f} ms, span {wall / steps:.4f} ms, "
              f"median launch period / {spl} = {st.median(per) / 1e3 / spl:.4f} ms "
              f"({100 * (st.median(per) / 1e3 / spl / mps - 1):+.1f}% vs ms_per_step)")
        if busy / steps > mps * 1.0005:
            print("  WARNING: GPU-busy union per step exceeds ms_per_step")
    if len(marks) >= 3:
        iso = [r for r in rows if marks[1][1] <= r[0] and r[1] <= marks[2][0] and
               (last_stage in r[2] if last_stage else is_encode(r[2]))]
        d = [(e - s) / 1e3 for s, e, _ in iso]
        if len(d) >= 8:
            print("  isolated, 1 segment per launch ", f(d[:4]), f"mean {st.mean(d[:4]):.1f} us")
            print("  isolated, 2 segments per launch", f(d[4:8]), f"mean {st.mean(d[4:8]):.1f} us")
        elif d:
            print("  isolated launches              ", f(d))


if __name__ == "__main__":
    main()
