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
  norc     : yuv420p without the per-pixel tv->pc table lookup (the yuvj420p conversion)
  rc_float : tv->pc in fp32 arithmetic (cvt, fma, round by +kM, med3 clamp): same bytes
  rc_float_nc: rc_float without the clamp (a probe)

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
WIDE = "    const uint64_t wide = wave_parallel_blocks(cur_active ? __popcll(mask) : 0);\n    if (cur_active && !((wide >> lane) & 1ull)) {\n"
EXACT = "  const uint32_t *col = (const uint32_t *)((const uint8_t *)pkcol + d.w);\n"
SCREEN = "      column_screen(s_pk, lane, s_skip, s_thr, dc, mlo, mhi, skip_st, (t & 3) == 0);"
ROWPASS = "    row_pass<RC>(raw, tab, s_rc, s_pk, lane);"
FBASE = "  auto frame_base = [&](int f) { return seg_frame(frames, f, g.frame_stride); };"
RCIF = "    float t0, t1, t2, t3;\n    if (RC) {\n"
RCBODY = """#pragma unroll
      for (int x = 0; x < 8; x++) {
        const uint32_t a = __builtin_amdgcn_perm((uint32_t)tab, x < 4 ? lo : hi,
                                                 0x0c0c0400u | (uint32_t)(x & 3));
        p[x] = __uint_as_float(0x4B400000u | (uint32_t)s_rc[a]);
      }
"""
# swscale's tv->pc in fp32 (exact for p = 0..255, tools/rc_float_check.py): kM + clamp(floor(p a - b))
RCFLOAT = """      const float ra = tab ? 1.138427734375f : 1.16436767578125f;
      const float rb = tab ? -17.719253540039062f : -18.624000549316406f;
#pragma unroll
      for (int x = 0; x < 8; x++)
        p[x] = __builtin_amdgcn_fmed3f(__builtin_fmaf(p[x], ra, rb) + kM, kM, kM + 255.0f);
"""
RCFLOAT_NC = """      const float ra = tab ? 1.138427734375f : 1.16436767578125f;
      const float rb = tab ? -17.719253540039062f : -18.624000549316406f;
#pragma unroll
      for (int x = 0; x < 8; x++)
        p[x] = __builtin_fmaf(p[x], ra, rb) + kM;
"""

SUBS = {
    # every chunk reads frame 0 or 1 (25 MB: Infinity-Cache resident): the memory system's share
    "nohbm": [(FBASE, "  auto frame_base = [&](int f) { return seg_frame(frames, f & 1, g.frame_stride); };")],
    "noemit": [(EMIT, "      q.emit(((uint32_t)__popcll(mask) << 8) ^ ((uint32_t)diff & 255u), 16);\n"
                      "      q.finish();\n"),
               (WIDE, "    const uint64_t wide = 0;\n    if (cur_active && !((wide >> lane) & 1ull)) {\n")],
    "noexact": [(EXACT, "  if (d.x != 0u) return 1 + (int)(d.y & 1u);\n" + EXACT)],
    "noscreen": [(SCREEN, "      dc = (int)(s_pk[lane] & 255u) - 128;")],
    "nodct": [(ROWPASS, "    {\n#pragma unroll\n      for (int r = 0; r < 8; r++) {\n"
                        "        s_pk[(r * 4) * 64 + lane] = (uint32_t)raw[r];\n"
                        "        s_pk[(r * 4 + 1) * 64 + lane] = (uint32_t)(raw[r] >> 32);\n"
                        "      }\n    }"),
              (SCREEN, "      dc = (int)(s_pk[lane] & 255u) - 128;")],
    # yuv420p: the per-pixel tv->pc table lookup dropped (the yuvj420p conversion instead): its share
    "norc": [(RCIF, "    float t0, t1, t2, t3;\n    if (false) {\n")],
    # yuv420p: tv->pc in fp32 arithmetic instead of the LDS table (exact: same bytes)
    "rc_float": [(RCBODY, RCFLOAT)],
    # the same without the clamp (a probe: exact only while every pixel is in 16..235 / 16..240)
    "rc_float_nc": [(RCBODY, RCFLOAT_NC)],
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
