# The refill-queue entries reserved when the wave knows its done envs (refill_reserve) against
# (the reserve variant was a working-tree change, reverted after this measurement: profiles/r06_pool_tail_ab.txt)
# HEAD's append at the wave's end (libab_head.so: tools/experiments/build_rev.sh HEAD head):
# the pool / sweep / HER / graph tests on the working tree, then k_step auto-reset off / pooled
# and the bench line, interleaved (headline, 65 536 envs).
set -o pipefail
mkdir -p gpurun_out
L=gym-ctr-reach_amd/ctr_reach_amd/lib
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_graph.py \
  tests/test_gpu_her.py tests/test_gpu_modes.py > gpurun_out/reserve_t.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/reserve_t.log
for rep in 1 2 3; do
  for v in libctr_reach_amd.so libab_head.so; do
    echo "== $v $rep" >> gpurun_out/reserve_ab.log
    CTR_REACH_AMD_LIB=$PWD/$L/$v timeout -k 10 200 python tools/time_step_modes.py 65536 >> gpurun_out/reserve_ab.log 2>&1 || exit 1
    CTR_REACH_AMD_LIB=$PWD/$L/$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/reserve_tmp.log 2>&1 || exit 1
    grep -o '"ms_per_step": [0-9.]*' gpurun_out/reserve_tmp.log >> gpurun_out/reserve_ab.log
  done
done
grep -v amdgpu.ids gpurun_out/reserve_ab.log
