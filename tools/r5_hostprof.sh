set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 200 python tools/host_first.py 2048 > gpurun_out/r05/host_first2048.txt 2>&1 || exit $?
timeout -k 10 200 python tools/host_first.py 256 > gpurun_out/r05/host_first256.txt 2>&1 || exit $?
