# A/B of k_refill (timed alone, tools/time_refill_budget.py) between the working tree's library and
# libab_prev.so, interleaved, after the GPU suite; then the refill's clock stamps of the new tree
set -o pipefail
mkdir -p gpurun_out
L=$PWD/gym-ctr-reach_amd/ctr_reach_amd/lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
for v in libctr_reach_amd.so libab_prev.so libctr_reach_amd.so libab_prev.so libctr_reach_amd.so libab_prev.so; do
  echo -n "$v: "
  CTR_REACH_AMD_LIB=$L/$v timeout -k 10 200 python tools/time_refill_budget.py 65536 6 2>&1 | grep budget || exit 1
done
CTR_REACH_AMD_LIB=$L/libab_diag.so timeout -k 10 200 python tools/diag_refill.py 6 2>&1 | grep -v amdgpu.ids | head -8
