#!/bin/bash
# Ablation / layout-experiment study of the pair-mode kernels.
#   VARIANTS="tag:-DFLAG=v[,-DFLAG2=w] ..." tools/ablate.sh build   (here: builds
#       psrsigsim_amd/libpss_hip_abl<tag>.so; a bare number N means -DPSS_ABLATE=N)
#   VARIANTS=... tools/ablate.sh run TAG     (GPU box: kernel_lab per variant)
# PSS_ABLATE bits: 1 no RNG/source/epilogue, 2 no FFT stages, 4 no four-step
# twiddles, 8 no ramps.  Layout switches: PSS_XCD_MAP (XCD-aware column-block
# order, default 1), PSS_SPLIT4K (1024 x 4096 split for N = 2^22, default 0).
VARIANTS=${VARIANTS:-"1 2 4 8"}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
tag_of() { echo "${1%%:*}"; }
flags_of() {
  case "$1" in
    *:*) echo "${1#*:}" | tr ',' ' ' ;;
    *) echo "-DPSS_ABLATE=$1" ;;
  esac
}
if [ "$1" = build ]; then
  for v in $VARIANTS; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -fno-slp-vectorize $(flags_of "$v") \
      -I$R/include -o $R/psrsigsim_amd/libpss_hip_abl$(tag_of "$v").so $R/psrsigsim_amd/csrc/pss_pipeline.hip $R/psrsigsim_amd/csrc/pss_host.cpp 2>/dev/null &
  done
  wait
  ls -la $R/psrsigsim_amd/libpss_hip_abl*.so
  exit 0
fi
TAG=${2:-abl}
OUT=$R/gpurun_out
for v in base $VARIANTS; do
  t=$(tag_of "$v")
  lib=$R/psrsigsim_amd/libpss_hip_abl$t.so
  [ "$v" = base ] && lib=$R/psrsigsim_amd/libpss_hip.so
  echo "== variant $v"
  for fl in ${LAB_FLAGS:-0}; do
  PSS_LIB_PATH=$lib timeout -k 10 300 python $R/tools/kernel_lab.py --no-fill --reps 2 --flags $fl ${LAB_VARIANTS:-full nonull_nonoise} \
      > $OUT/${TAG}_${t}_f$fl.log 2>&1 || { echo "variant $v failed"; tail -5 $OUT/${TAG}_${t}_f$fl.log; exit 1; }
  echo "flags $fl"; grep -v negative $OUT/${TAG}_${t}_f$fl.log | grep wall
  done
done
