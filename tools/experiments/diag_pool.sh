# Diagnostic: where the pooled k_step's extra ~1 us goes (headline, 65 536 envs): the product library vs
# libab_pfall.so (every env's next pool slot prefetched before the FK, not only the time-limit ones) vs
# libab_noq.so (no refill-queue append at the wave's end; the pool is not refilled, so the run drains it).
# The two variants were built from a temporary edit of ctr_kernels.hip (CTR_DIAG_PREFETCH_ALL / CTR_DIAG_NOREFILLQ).
set -o pipefail
mkdir -p gpurun_out
L=gym-ctr-reach_amd/ctr_reach_amd/lib
for rep in 1 2; do
  for v in libctr_reach_amd.so libab_pfall.so libab_noq.so; do
    echo "== $v $rep" >> gpurun_out/diag_pool.log
    CTR_REACH_AMD_LIB=$PWD/$L/$v timeout -k 10 200 python tools/time_step_modes.py 65536 >> gpurun_out/diag_pool.log 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/diag_pool.log
