# configs[4]: level-2 RK4 pair steps with the stages' sincos shared by the pair (working tree,
# (the shared-sincos variant was a working-tree change, reverted after this measurement: profiles/r06_lv2_share_ab.txt)
# CTR_PAIR_LV2_SHARE) against HEAD (libab_head.so: tools/experiments/build_rev.sh HEAD head):
# the configs[4] GPU tests, then k_step<2> and the configs[4] bench line, interleaved.
set -o pipefail
mkdir -p gpurun_out
L=gym-ctr-reach_amd/ctr_reach_amd/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_modes.py tests/test_gpu_configs.py \
  tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_gpu_her.py > gpurun_out/lv2_t.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/lv2_t.log
for rep in 1 2 3; do
  for v in libctr_reach_amd.so libab_head.so; do
    echo "== $v $rep" >> gpurun_out/lv2_ab.log
    CTR_REACH_AMD_LIB=$PWD/$L/$v timeout -k 10 200 python tools/time_step_modes.py 65536 c5 >> gpurun_out/lv2_ab.log 2>&1 || exit 1
    CTR_REACH_AMD_LIB=$PWD/$L/$v timeout -k 10 200 python bench.py --config 5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/lv2_tmp.log 2>&1 || exit 1
    grep -o '"ms_per_step": [0-9.]*' gpurun_out/lv2_tmp.log >> gpurun_out/lv2_ab.log
  done
done
grep -v amdgpu.ids gpurun_out/lv2_ab.log | paste - - - - -
