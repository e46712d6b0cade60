# the RK45 pair with the segment-count deal key (libab_rk45pair2.so) vs the extension key
# (libab_rk45pair.so) vs one env per lane: k_step and the bench line, interleaved
set -o pipefail
mkdir -p gpurun_out
L=gym-ctr-reach_amd/ctr_reach_amd/lib
CTR_REACH_AMD_LIB=$PWD/$L/libab_rk45pair2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py -k "step_matches or ragged or full_size or shard_invariance" > gpurun_out/rk45pair2_t.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/rk45pair2_t.log
for rep in 1 2; do
  for v in libctr_reach_amd.so libab_rk45pair.so libab_rk45pair2.so; do
    echo "== $v $rep" >> gpurun_out/rk45pair_key.log
    CTR_REACH_AMD_LIB=$PWD/$L/$v timeout -k 10 200 python tools/time_step_modes.py 65536 >> gpurun_out/rk45pair_key.log 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/rk45pair_key.log
echo done
