"""Build libpss_hip.so in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = [os.path.join(HERE, "csrc", "pss_pipeline.hip"), os.path.join(HERE, "csrc", "pss_host.cpp")]
DEPS = SRC + [os.path.join(HERE, "csrc", f) for f in ("pss_device.hpp", "pss_fft.hpp")] + \
    [os.path.join(ROOT, "include", "pss_hip.h")]
OUT = os.path.join(HERE, "libpss_hip.so")
ARCH = os.environ.get("PSS_OFFLOAD_ARCH", "gfx950")


def stale():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(d) > t for d in DEPS)


def build(force=False, verbose=True):
    if not force and not stale():
        return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    # -fno-slp-vectorize: packed f32 (v_pk_*) issues at half rate on gfx950 and
    # costs register-pair moves; scalar f32 is cheaper here.
    cmd = [hipcc, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-shared", "-fno-slp-vectorize",
           "-I" + os.path.join(ROOT, "include"), "-o", OUT + ".tmp"] + SRC
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
