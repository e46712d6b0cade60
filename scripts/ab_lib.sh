# A/B of the default library against gym-ctr-reach_amd/ctr_reach_amd/lib/libab_prev.so:
# the GPU suite on the default library, then k_step timing (headline and configs[1]) for both,
# interleaved.  usage: bash scripts/ab_lib.sh [pytest args]
set -o pipefail
mkdir -p gpurun_out
L=$PWD/gym-ctr-reach_amd/ctr_reach_amd/lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "$@" > gpurun_out/pytest_ab.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
for v in libctr_reach_amd.so libab_prev.so libctr_reach_amd.so libab_prev.so; do
  echo "== $v"
  CTR_REACH_AMD_LIB=$L/$v timeout -k 10 120 python tools/time_step_modes.py || exit 1
  CTR_REACH_AMD_LIB=$L/$v timeout -k 10 120 python tools/time_step_modes.py 4096 rigid || exit 1
done
