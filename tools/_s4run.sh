set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s4_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s4_tests.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="${VARIANTS:-1 16 2}" LAB_VARIANTS="full" timeout -k 10 600 bash tools/ablate.sh run ${TAG:-s4b}
