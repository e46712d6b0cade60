set -o pipefail
mkdir -p gpurun_out
L=gym-ctr-reach_amd/ctr_reach_amd/lib
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_modes.py tests/test_gpu_configs.py tests/test_gpu_parity.py -k "rk4 or modes or configs or invariance" > gpurun_out/pair_t.log 2>&1; echo "tests rc=$?"; tail -5 gpurun_out/pair_t.log
for rep in 1 2; do
  for v in ${LIBS:-libctr_reach_amd.so libab_onelane.so}; do
    echo "== $v $rep" >> gpurun_out/pair_ab.log
    CTR_REACH_AMD_LIB=$L/$v timeout -k 10 200 python tools/time_step_modes.py 65536 c5 >> gpurun_out/pair_ab.log 2>&1 || exit 1
    CTR_REACH_AMD_LIB=$L/$v timeout -k 10 200 python bench.py --config 5 --steps 20 --warmup 5 --no-cpu-baseline >> gpurun_out/pair_ab.log 2>&1 || exit 1
  done
done
echo done
