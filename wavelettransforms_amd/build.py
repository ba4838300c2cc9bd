"""Build libwtprune.so (HIP, gfx950) in-tree: wavelettransforms_amd/_lib/libwtprune.so.

hipcc cross-compiles for gfx950 without a GPU.  -ffp-contract=off is part of the parity
contract: PyWavelets' float32 filter bank uses separate multiplies and adds, so the
compiler must not fuse them into FMAs.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "_lib")
LIB = os.path.join(OUT_DIR, "libwtprune.so")
SOURCES = ["kernels.hip", "filterbank.hip", "small.hip", "api.hip"]
DEPS = SOURCES + ["wtp_internal.h", "wt_dwt_core.h", "wt_synth.h", "wt_perm.h", "wt_filters.inc", "small_geom.h", "fb_index.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("WTP_OFFLOAD_ARCH", "gfx950")

FLAGS = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
         "-Wall", "-Wno-unused-function", "-I" + CSRC, "-I" + os.path.join(os.path.dirname(HERE), "include")]


def stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, d) for d in DEPS] + [os.path.join(os.path.dirname(HERE), "include", "wtprune.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False):
    if not force and not stale():
        return LIB
    os.makedirs(OUT_DIR, exist_ok=True)
    tmp = LIB + ".tmp"
    cmd = [HIPCC] + FLAGS + ["-o", tmp] + [os.path.join(CSRC, s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
