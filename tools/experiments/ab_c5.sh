# configs[4] A/B: RK4 tests on the working tree's library, then k_step (tools/time_step_modes.py c5)
# and the bench line, interleaved, against libab_head.so (tools/experiments/build_rev.sh HEAD head)
set -e
mkdir -p gpurun_out
L=gym-ctr-reach_amd/ctr_reach_amd/lib
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_modes.py tests/test_gpu_configs.py tests/test_gpu_parity.py -k "rk4 or modes or configs or invariance" > gpurun_out/pf_t.log 2>&1
for rep in 1 2; do
  for v in libctr_reach_amd.so libab_head.so; do
    echo "== $v $rep" >> gpurun_out/pf_ab.log
    CTR_REACH_AMD_LIB=$L/$v timeout -k 10 200 python tools/time_step_modes.py 65536 c5 >> gpurun_out/pf_ab.log 2>&1
    CTR_REACH_AMD_LIB=$L/$v timeout -k 10 200 python bench.py --config 5 --no-cpu-baseline >> gpurun_out/pf_ab.log 2>&1
  done
done
