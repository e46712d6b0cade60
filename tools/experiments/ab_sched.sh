# k_step under other AMDGPU scheduler strategies (libab_s_<strategy>.so, built with
# -mllvm -amdgpu-sched-strategy=<strategy>, or none for the default) against the product build
# (max-ilp): headline and configs[4] k_step, interleaved, two repetitions.
set -o pipefail
mkdir -p gpurun_out
L=gym-ctr-reach_amd/ctr_reach_amd/lib
for rep in 1 2; do
  for v in libctr_reach_amd.so libab_s_default.so libab_s_iterative-ilp.so libab_s_iterative-minreg.so libab_s_max-memory-clause.so; do
    echo "== $v $rep" >> gpurun_out/sched_ab.log
    CTR_REACH_AMD_LIB=$PWD/$L/$v timeout -k 10 200 python tools/time_step_modes.py 65536 >> gpurun_out/sched_ab.log 2>&1 || exit 1
    CTR_REACH_AMD_LIB=$PWD/$L/$v timeout -k 10 200 python tools/time_step_modes.py 65536 c5 >> gpurun_out/sched_ab.log 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/sched_ab.log
