set -o pipefail
mkdir -p gpurun_out/r05
# the microbenchmark is built from its source here (no binary in git)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o tools/l3_spill tools/l3_spill.hip || exit $?
timeout -k 10 300 ./tools/l3_spill 8 > gpurun_out/r05/l3_spill.txt 2>&1 || exit $?
for n in 8 16 32 64 128 2048; do
  timeout -k 10 180 python bench.py --nchan $n --steps 10 --warmup 2 --no-cpu > gpurun_out/r05/bench_n$n.json 2> gpurun_out/r05/bench_n$n.err || exit $?
done
