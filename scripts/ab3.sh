# three-way A/B: working tree vs libab_stg.so vs libab_prev.so (k_step timing, interleaved), after a suite subset
set -o pipefail
mkdir -p gpurun_out
L=$PWD/gym-ctr-reach_amd/ctr_reach_amd/lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "parity or graph or modes or her" > gpurun_out/pytest_ab.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for v in libctr_reach_amd.so libab_stg.so libab_prev.so; do
  echo "== $v"
  CTR_REACH_AMD_LIB=$L/$v timeout -k 10 120 python tools/time_step_modes.py || exit 1
  CTR_REACH_AMD_LIB=$L/$v timeout -k 10 120 python tools/time_step_modes.py 4096 rigid || exit 1
done
done
