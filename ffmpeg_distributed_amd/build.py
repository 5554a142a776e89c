"""In-tree build of libmjgpu.so (hipcc, gfx950).  The .so stays next to this file so
it travels to the GPU box with the repo snapshot (it is git-ignored).

Staleness is decided by content, not mtime: a sidecar `libmjgpu.so.sha256` records the
SHA-256 of every source, header and the compile command the library was built from, and
build() recompiles whenever that digest differs (or the library or its sidecar is missing).
A pushed binary whose sources changed is therefore always rebuilt where a compiler exists;
where none exists (a box without hipcc), `check()` reports the mismatch."""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libmjgpu.so")
STAMP = LIB + ".sha256"
SOURCES = ["api.hip", "sws_filter.cpp"]
DEPS = SOURCES + ["kernels.hip", "scale.hip", "jpeg_tables.h", "sws_filter.h"]
ARCH = os.environ.get("MJG_OFFLOAD_ARCH", "gfx950")


def _command(out: str):
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    # -fno-slp-vectorize: the SLP vectoriser packs k_encode's per-column fp32 chains into
    # v_pk_fma_f32 across columns, which doubles live registers (123 VGPRs -> 168 + 180 B
    # of scratch spills per lane) and costs ~30% of k_encode time.
    # -dot6-insts / -dot4-insts: without the two-operand v_dot4c_i32_i8 / v_dot2c_i32_i16 forms the
    # compiler emits the three-operand v_dot4_i32_i8 / v_dot2_i32_i16, which take the accumulator
    # (or an SGPR) as a separate operand: no v_mov to copy a shared start value into every
    # accumulator (k_scale_encode's h-pass: 2 per output).  The host compile ignores them.
    # -amdgpu-mfma-vgpr-form: MFMA results in VGPRs, not AGPRs (no v_accvgpr_read per result
    # element in k_scale's matrix-core h-pass: c4 +0.8..2.2%, profiles/r05/c4_scale_mfma_vgpr_form_ab.txt;
    # the default-table k_encode's code is unchanged).
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fno-slp-vectorize", "-fPIC", "-shared",
           "-mllvm", "-amdgpu-mfma-vgpr-form=1",
           "-Xclang", "-target-feature", "-Xclang", "-dot6-insts",
           "-Xclang", "-target-feature", "-Xclang", "-dot4-insts",
           "-Wno-unused-command-line-argument", "-I", os.path.join(ROOT, "include"), "-o", out]
    return cmd + [os.path.join(CSRC, s) for s in SOURCES]


def source_digest() -> str:
    """SHA-256 over the sources, the public header and the compile flags."""
    h = hashlib.sha256()
    paths = [os.path.join(CSRC, d) for d in DEPS] + [os.path.join(ROOT, "include", "mjgpu.h")]
    for p in paths:
        if not os.path.exists(p):
            continue
        h.update(os.path.relpath(p, ROOT).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(_command("OUT")[1:]).replace(ROOT, "ROOT").encode())
    return h.hexdigest()


def check() -> bool:
    """True when libmjgpu.so exists and was built from the current sources."""
    if not os.path.exists(LIB) or not os.path.exists(STAMP):
        return False
    with open(STAMP) as f:
        return f.read().strip() == source_digest()


CLIENT = os.path.join(PKG, "mjg_client")
CLIENT_STAMP = CLIENT + ".sha256"
CLIENT_SRC = os.path.join(CSRC, "mjg_client.c")


def _client_command(out: str):
    return [os.environ.get("CC", "gcc"), "-O2", "-Wall", "-o", out, CLIENT_SRC]


def client_digest() -> str:
    h = hashlib.sha256()
    with open(CLIENT_SRC, "rb") as f:
        h.update(f.read())
    h.update(" ".join(_client_command("OUT")[1:]).replace(ROOT, "ROOT").encode())
    return h.hexdigest()


def client_check() -> bool:
    """True when the mjg_client binary exists and was built from the current source."""
    if not os.path.exists(CLIENT) or not os.path.exists(CLIENT_STAMP):
        return False
    with open(CLIENT_STAMP) as f:
        return f.read().strip() == client_digest()


def build_client(force: bool = False, verbose: bool = False) -> str:
    """The native per-segment client of the resident encoder (csrc/mjg_client.c)."""
    if not force and client_check():
        return CLIENT
    tmp = f"{CLIENT}.tmp{os.getpid()}"
    cmd = _client_command(tmp)
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, CLIENT)
    with open(f"{CLIENT_STAMP}.tmp{os.getpid()}", "w") as f:
        f.write(client_digest() + "\n")
    os.replace(f"{CLIENT_STAMP}.tmp{os.getpid()}", CLIENT_STAMP)
    return CLIENT


def build(force: bool = False, verbose: bool = False) -> str:
    if shutil.which(_client_command("x")[0]) and (force or not client_check()):
        build_client(force, verbose)
    if not force and check():
        return LIB
    # per-process temporaries and atomic renames: ranks of one node that find the library
    # stale at the same time each build a complete copy, and none loads a partial file
    tmp = f"{LIB}.tmp{os.getpid()}"
    cmd = _command(tmp)
    if not shutil.which(cmd[0]) and not os.path.exists(cmd[0]):
        raise RuntimeError(f"{LIB} is missing or stale (sources changed) and {cmd[0]} is absent")
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(tmp, LIB)
    with open(f"{STAMP}.tmp{os.getpid()}", "w") as f:
        f.write(source_digest() + "\n")
    os.replace(f"{STAMP}.tmp{os.getpid()}", STAMP)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
