# configs[1] group-sort A/B: GPU mode tests, then k_step timing (rigid, 4096 envs) for the
# rank-based seg_build_group (default library) and the per-lane network (libab_net.so)
set -o pipefail
mkdir -p gpurun_out
L=$PWD/gym-ctr-reach_amd/ctr_reach_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_modes.py -x -v --timeout 120 --timeout-method thread > gpurun_out/modes.log 2>&1; rc=$?
tail -15 gpurun_out/modes.log; [ $rc -eq 0 ] || exit $rc
for v in libctr_reach_amd.so libab_net.so libctr_reach_amd.so libab_net.so; do
  echo "== $v"; CTR_REACH_AMD_LIB=$L/$v timeout -k 10 120 python tools/time_step_modes.py 4096 rigid || exit 1
done
timeout -k 10 300 python bench.py --config 2 --steps 20 --warmup 5 --cpu-seconds 2 > gpurun_out/bench_c2.log 2>&1 || exit 1
tail -1 gpurun_out/bench_c2.log | cut -c1-400
