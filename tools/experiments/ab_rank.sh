# seg_build by stable ranks (working tree) against HEAD's sorting network (libab_head.so:
# (the rank seg_build was a working-tree change, reverted after this measurement: profiles/r06_segbuild_rank_ab.txt)
# tools/experiments/build_rev.sh HEAD head): the FK / step parity tests on the working tree, then
# k_step for the headline and configs[4] and both bench lines, interleaved.
set -o pipefail
mkdir -p gpurun_out
L=gym-ctr-reach_amd/ctr_reach_amd/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/rank_t.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/rank_t.log
for rep in 1 2; do
  for v in libctr_reach_amd.so libab_head.so; do
    echo "== $v $rep" >> gpurun_out/rank_ab.log
    CTR_REACH_AMD_LIB=$PWD/$L/$v timeout -k 10 200 python tools/time_step_modes.py 65536 >> gpurun_out/rank_ab.log 2>&1 || exit 1
    CTR_REACH_AMD_LIB=$PWD/$L/$v timeout -k 10 200 python tools/time_step_modes.py 65536 c5 >> gpurun_out/rank_ab.log 2>&1 || exit 1
    CTR_REACH_AMD_LIB=$PWD/$L/$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/rank_tmp.log 2>&1 || exit 1
    grep -o '"ms_per_step": [0-9.]*' gpurun_out/rank_tmp.log >> gpurun_out/rank_ab.log
    CTR_REACH_AMD_LIB=$PWD/$L/$v timeout -k 10 200 python bench.py --config 5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/rank_tmp.log 2>&1 || exit 1
    grep -o '"ms_per_step": [0-9.]*' gpurun_out/rank_tmp.log >> gpurun_out/rank_ab.log
  done
done
grep -v amdgpu.ids gpurun_out/rank_ab.log
