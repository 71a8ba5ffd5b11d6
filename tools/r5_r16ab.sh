set -o pipefail
mkdir -p gpurun_out/r05/r16
for i in 1 2; do
for v in prod t512; do
  if [ $v = t512 ]; then export PSS_LIB_PATH=$PWD/psrsigsim_amd/libpss_hip_r16t512.so; else unset PSS_LIB_PATH; fi
  timeout -k 10 300 python bench.py --workload c5 --no-cpu --steps 10 > gpurun_out/r05/r16/c5_${v}_$i.json 2> gpurun_out/r05/r16/c5_${v}_$i.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/r05/r16/c5_${v}_$i.json')); print('$v', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
done
done
unset PSS_LIB_PATH
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "c5 or fullgrid or bitwise" > gpurun_out/r05/r16/tests.log 2>&1; echo tests rc=$?; tail -2 gpurun_out/r05/r16/tests.log
