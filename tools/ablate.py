#!/usr/bin/env python3
"""Phase ablations of k_encode (VALU DCT stage, -huffman default) for a HEAD breakdown.

Each ablation is a COPY of ffmpeg_distributed_amd/csrc with one textual substitution in
kernels.hip (the product sources carry no ablation switches), built into
ffmpeg_distributed_amd/libmjgpu_v_<name>.so for tools/variants.py.  Outputs of an ablated
build are wrong by construction; only kernel times (and SQ counters) are compared.

  noemit   : Huffman emission replaced by 16 fixed bits per block (no exact quantisation, no
             per-lane candidate loop, no wave-parallel blocks); DCT, screen and pack kept
  noexact  : exact_coef returns a constant (the candidate loop and coding kept)
  noscreen : column screen skipped (DC from the row image, no candidates): loads + row pass +
             DC/EOB coding + pack
  nohbm    : every chunk reads frame 0 or 1 (Infinity-Cache resident): memory's share
  nodct    : row pass and column screen skipped (raw rows copied into the LDS image): loads +
             LDS image + DC/EOB coding + pack

usage: tools/ablate.py NAME...      (writes tools/_v<NAME>src/ and builds the .so)
       tools/ablate.py --variants NAME...   (prints the VARIANTS string for variants.py)
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ffmpeg_distributed_amd", "csrc")

EMIT = ("      emit_block(s_pk + lane, mask, diff, s_zd, s_m2, q);\n"
        "      q.finish();\n")
WIDE = "const uint64_t wide = wave_parallel_blocks(cur_active ? __popcll(mask) : 0);"
EXACT = "  const uint32_t *col = pkcol + ((d.y >> 18) & 3u) * 64;\n"
SCREEN = "      if (SCR) column_screen(s_pk, lane, s_skip, s_thr, dc, ca, cb);"
ROWPASS = "      row_pass<RC>(raw, tab, s_rc, s_pk, lane);"

FBASE = "  auto frame_base = [&](int f) { return frames + (size_t)f * g.frame_stride; };"

SUBS = {
    # every chunk reads frame 0 or 1 (25 MB: Infinity-Cache resident): the memory system's share
    "nohbm": [(FBASE, "  auto frame_base = [&](int f) { return frames + (size_t)(f & 1) * g.frame_stride; };")],
    "noemit": [(EMIT, "      q.emit(((uint32_t)__popcll(mask) << 8) ^ ((uint32_t)diff & 255u), 16);\n"
                      "      q.finish();\n"),
               (WIDE, "const uint64_t wide = 0;")],
    "noexact": [(EXACT, "  if (d.x != 0u) return 1 + (int)(d.y & 1u);\n" + EXACT)],
    "noscreen": [(SCREEN, "      if (SCR) dc = (int)(s_pk[lane] & 255u) - 128;")],
    "nodct": [(ROWPASS, "      {\n#pragma unroll\n        for (int r = 0; r < 8; r++) {\n"
                        "          s_pk[(r * 4) * 64 + lane] = (uint32_t)raw[r];\n"
                        "          s_pk[(r * 4 + 1) * 64 + lane] = (uint32_t)(raw[r] >> 32);\n"
                        "        }\n      }"),
              (SCREEN, "      if (SCR) dc = (int)(s_pk[lane] & 255u) - 128;")],
}


def make(name):
    dst = os.path.join(ROOT, "tools", f"_v{name}src")
    if os.path.exists(dst):
        shutil.rmtree(dst)
    shutil.copytree(CSRC, dst)
    p = os.path.join(dst, "kernels.hip")
    src = open(p).read()
    for old, new in SUBS[name]:
        if src.count(old) != 1:
            raise SystemExit(f"{name}: pattern found {src.count(old)} times: {old[:60]!r}")
        src = src.replace(old, new)
    open(p, "w").write(src)
    return os.path.relpath(dst, ROOT)


def main():
    args = sys.argv[1:]
    if args and args[0] == "--variants":
        print(";".join(["full=:"] + [f"{n}=tools/_v{n}src:" for n in args[1:]]))
        return
    names = args or list(SUBS)
    vs = ";".join(["full=:"] + [f"{n}={make(n)}:" for n in names])
    env = dict(os.environ, VARIANTS=vs)
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "variants.py"), "--build"], check=True, env=env)
    print(vs)


if __name__ == "__main__":
    main()
