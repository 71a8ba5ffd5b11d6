#!/bin/bash
# GPU parity tests against the device-assert build (PSS_DEBUG=1; built here
# with `python -m psrsigsim_amd.build --debug`, shipped in-tree like the product
# library).  An assert that fires aborts the kernel and fails its test.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
PSS_LIB_PATH=$R/psrsigsim_amd/libpss_hip_debug.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider ${@} > $OUT/debug_tests.log 2>&1
rc=$?; echo "debug-build GPU tests rc=$rc"; tail -3 $OUT/debug_tests.log; exit $rc
