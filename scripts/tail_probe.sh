# k_step with extra spinning workgroups in its tail (tools/tail_probe.py); each combination in its own process
set -o pipefail
mkdir -p gpurun_out
L=$PWD/gym-ctr-reach_amd/ctr_reach_amd/lib/libab_tail.so
for c in "0 0" "64 3000" "128 3000" "256 3000" "64 6000" "128 6000" "256 6000" "0 0" "512 3000" "128 10000"; do
  set -- $c
  CTR_REACH_AMD_LIB=$L CTR_TAIL_WG=$1 CTR_TAIL_NS=$2 timeout -k 10 120 python tools/tail_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done
