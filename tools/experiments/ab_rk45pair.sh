# the headline (scipy RK45, compliant) with one env per lane PAIR
# (libab_rk45pair.so: -DCTR_RK45_PAIR=1) against the product library (one env per lane):
# the step-path parity tests on the pair build, then k_step and the bench line, interleaved.
# Build first (CPU container): make -C gym-ctr-reach_amd LIB=ctr_reach_amd/lib/libab_rk45pair.so \
#   EXTRA=-DCTR_RK45_PAIR=1 ctr_reach_amd/lib/libab_rk45pair.so
# (tools/experiments/ab_rk45pair_key.sh: libab_rk45pair2.so adds -DCTR_RK45_KEY_NSEG)
set -o pipefail
mkdir -p gpurun_out
L=gym-ctr-reach_amd/ctr_reach_amd/lib
CTR_REACH_AMD_LIB=$PWD/$L/libab_rk45pair.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_gpu_her.py \
  -k "step_matches or ragged or full_size or facade_step or shard_invariance or reset_pool or graph or her" \
  > gpurun_out/rk45pair_t.log 2>&1; echo "tests rc=$?"; tail -5 gpurun_out/rk45pair_t.log
for rep in 1 2; do
  for v in libctr_reach_amd.so libab_rk45pair.so; do
    echo "== $v $rep" >> gpurun_out/rk45pair_ab.log
    CTR_REACH_AMD_LIB=$PWD/$L/$v timeout -k 10 200 python tools/time_step_modes.py 65536 >> gpurun_out/rk45pair_ab.log 2>&1 || exit 1
    CTR_REACH_AMD_LIB=$PWD/$L/$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/rk45pair_tmp.log 2>&1 || exit 1
    grep -o '"ms_per_step": [0-9.]*' gpurun_out/rk45pair_tmp.log >> gpurun_out/rk45pair_ab.log
  done
done
cat gpurun_out/rk45pair_ab.log
echo done
