#!/bin/bash
# Ablation study of the pair-mode kernels.
#   tools/ablate.sh build          (here: builds psrsigsim_amd/libpss_hip_abl<N>.so)
#   tools/ablate.sh run TAG        (GPU box: kernel_lab per variant)
# PSS_ABLATE bits: 1 no RNG/source/epilogue, 2 no FFT stages, 4 no four-step
# twiddles, 8 no ramps (see pss_pipeline.hip).
VARIANTS=${VARIANTS:-"1 2 4 8"}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
if [ "$1" = build ]; then
  for v in $VARIANTS; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DPSS_ABLATE=$v \
      -I$R/include -o $R/psrsigsim_amd/libpss_hip_abl$v.so $R/psrsigsim_amd/csrc/pss_pipeline.hip 2>/dev/null &
  done
  wait
  ls -la $R/psrsigsim_amd/libpss_hip_abl*.so
  exit 0
fi
TAG=${2:-abl}
OUT=$R/gpurun_out
for v in 0 $VARIANTS; do
  lib=$R/psrsigsim_amd/libpss_hip_abl$v.so
  [ $v = 0 ] && lib=$R/psrsigsim_amd/libpss_hip.so
  echo "== PSS_ABLATE=$v"
  PSS_LIB_PATH=$lib timeout -k 10 300 python $R/tools/kernel_lab.py --no-fill --reps 2 full nonull_nonoise \
      > $OUT/${TAG}_$v.log 2>&1 || { echo "variant $v failed"; tail -5 $OUT/${TAG}_$v.log; exit 1; }
  grep -v negative $OUT/${TAG}_$v.log | grep wall
done
