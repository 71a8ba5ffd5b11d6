for v in "64 16" "64 32" "64 64" "128 64" "32 64"; do
  set -- $v
  PSS_LIB_PATH=psrsigsim_amd/libpss_hip_nf.so PSS_PASSA=0 PSS_DBG_GF=$1 PSS_DBG_CH=$2 bash tools/r4_prof.sh l_$1_$2 > gpurun_out/nfexp_l_$1_$2.txt 2>&1 || exit 1
  echo "gf=$1 ch=$2: $(grep -E 'k_null_fix|k_pairC_fast' gpurun_out/nfexp_l_$1_$2.txt | awk '{print $1, $NF}' | tr '\n' ' ')"
done
