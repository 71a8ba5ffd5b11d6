"""Build libpss_hip.so in-tree for gfx950 (hipcc cross-compiles without a GPU).

The library embeds the sha256 of its sources (``pss_build_hash``); build()
recompiles whenever that hash differs from the sources in the tree (content,
not mtimes: a checkout or a copy to the GPU box can leave a stale binary
newer than its sources), and ``_lib.load`` refuses a library whose hash does
not match the sources next to it.
"""
import hashlib
import os
import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
# launch units: one translation unit each (the kernel templates are
# instantiated per unit), compiled in parallel and linked with the host code
UNITS = ["pss_pipeline.hip", "pss_fourstep.hip", "pss_fourstep_b.hip", "pss_smooth.hip", "pss_smooth_b.hip",
         "pss_smooth_c.hip", "pss_single.hip", "pss_fallback.hip"]
SRC = [os.path.join(HERE, "csrc", u) for u in UNITS] + [os.path.join(HERE, "csrc", "pss_host.cpp")]
DEPS = SRC + [os.path.join(HERE, "csrc", f) for f in ("pss_engine.hpp", "pss_device.hpp", "pss_fft.hpp")] + \
    [os.path.join(ROOT, "include", "pss_hip.h")]
OUT = os.path.join(HERE, "libpss_hip.so")
OUT_DEBUG = os.path.join(HERE, "libpss_hip_debug.so")
ARCH = os.environ.get("PSS_OFFLOAD_ARCH", "gfx950")
# -fno-slp-vectorize: packed f32 (v_pk_*) issues at half rate on gfx950 and
# costs register-pair moves; scalar f32 is cheaper here.
# -target-feature -packed-fp32-ops (device): without it the backend still
# forms v_pk_add_f32 from complex adds of 64-bit loaded pairs (34 in pass A,
# 50 in the row pass); measured 7.65 cycles per wave-instruction at 4 waves
# per SIMD against 2.54 for v_add_f32 (tools/probe_rates.hip,
# profiles/r06/probe_rates.txt): row pass -0.23 ms at C3 (same-box A/B,
# profiles/r06/ab_pk.txt).  The host compile ignores the feature (a warning).
# -ffp-contract=on: a multiply-add fuses only within one source expression,
# never across statements, so a value's rounding does not depend on the code
# around it (HIP's default fuses e.g. the wave pass A's profile x draw
# product into the first butterfly, which the LDS-staged kernels cannot: the
# fast and generic kernels would differ by an ulp; ~1 % of pass A's VALU).
FLAGS = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-shared", "-fno-slp-vectorize",
         "-ffp-contract=on", "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]


def source_hash(extra=()):
    """sha256 over the library's sources and compile flags."""
    h = hashlib.sha256()
    for d in DEPS:
        with open(d, "rb") as f:
            h.update(os.path.basename(d).encode() + b"\0" + f.read() + b"\0")
    h.update(" ".join(list(FLAGS) + list(extra)).encode())
    return h.hexdigest()


def embedded_hash(path=OUT):
    """The hash string compiled into a built library (read from its bytes,
    without loading it), or None."""
    try:
        with open(path, "rb") as f:
            m = re.search(rb"PSS_BUILD_HASH=([0-9a-f]{64})", f.read())
    except OSError:
        return None
    return m.group(1).decode() if m else None


def stale():
    return embedded_hash() != source_hash()


def build(force=False, verbose=True, debug=False, variant=None, variant_flags=()):
    """Build the product library, or with ``debug=True`` the device-assert
    build ``libpss_hip_debug.so`` (PSS_DEBUG=1: bounds asserts on generic and
    buffer accesses; load it with PSS_LIB_PATH, tools/debug_gpu.sh)."""
    extra = ["-DPSS_DEBUG=1"] if debug else []
    out = OUT_DEBUG if debug else OUT
    if variant:
        # an A/B build (tools/r3_abn.sh loads it through PSS_LIB_PATH): the
        # product sources with extra compile flags, e.g. -D switches
        extra = list(variant_flags)
        out = os.path.join(HERE, "libpss_hip_%s.so" % variant)
    if not force and embedded_hash(out) == source_hash(extra):
        return out
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    objdir = os.path.join(HERE, "build", variant or ("debug" if debug else "release"))
    os.makedirs(objdir, exist_ok=True)
    defs = extra + ['-DPSS_BUILD_HASH="%s"' % source_hash(extra), "-I" + os.path.join(ROOT, "include")]
    cflags = [f for f in FLAGS if f != "-shared"]
    jobs = []
    for src in SRC[:-1]:
        obj = os.path.join(objdir, os.path.basename(src).replace(".hip", ".o"))
        jobs.append(([hipcc] + cflags + defs + ["-c", "-o", obj, src], obj))
    if verbose:
        print("compiling %d units in parallel: %s" % (len(jobs), " ".join(jobs[0][0][:-3])), file=sys.stderr)
    workers = max(1, min(len(jobs), os.cpu_count() or 4, 16))
    with ThreadPoolExecutor(workers) as ex:
        results = list(ex.map(lambda j: subprocess.run(j[0], capture_output=True, text=True), jobs))
    for (cmd, _), r in zip(jobs, results):
        if r.returncode != 0:
            sys.stderr.write(r.stdout + r.stderr)
            raise subprocess.CalledProcessError(r.returncode, cmd)
    link = [hipcc] + FLAGS + defs + ["-o", out + ".tmp"] + [o for _, o in jobs] + [SRC[-1]]
    subprocess.run(link, check=True, capture_output=not verbose)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    # python -m psrsigsim_amd.build [--force] [--debug] [--variant NAME FLAG ...]
    if "--variant" in sys.argv:
        i = sys.argv.index("--variant")
        build(force=True, variant=sys.argv[i + 1], variant_flags=sys.argv[i + 2:])
    else:
        build(force="--force" in sys.argv, debug="--debug" in sys.argv)
