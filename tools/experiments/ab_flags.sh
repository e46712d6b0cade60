# k_step under extra LLVM codegen options on top of the product flags (libab_f_<tag>.so):
#   trk  -amdgpu-use-amdgpu-trackers       noaa   -amdgpu-use-aa-in-codegen=0
#   nocl -misched-cluster=0                nopost -enable-post-misched=0
#   prera -amdgpu-enable-pre-ra-optimizations=0
# headline and configs[4] k_step, interleaved, two repetitions.
set -o pipefail
mkdir -p gpurun_out
L=gym-ctr-reach_amd/ctr_reach_amd/lib
for rep in 1 2; do
  for v in libctr_reach_amd.so libab_f_trk.so libab_f_noaa.so libab_f_nocl.so libab_f_nopost.so libab_f_prera.so; do
    echo "== $v $rep" >> gpurun_out/flags_ab.log
    CTR_REACH_AMD_LIB=$PWD/$L/$v timeout -k 10 200 python tools/time_step_modes.py 65536 >> gpurun_out/flags_ab.log 2>&1 || exit 1
    CTR_REACH_AMD_LIB=$PWD/$L/$v timeout -k 10 200 python tools/time_step_modes.py 65536 c5 >> gpurun_out/flags_ab.log 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/flags_ab.log | grep -v "FK operator" | paste - - - - - 
