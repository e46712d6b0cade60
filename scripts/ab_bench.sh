# A/B of the working tree's library against libab_prev.so (tools/experiments/build_rev.sh): the GPU
# suite on the new library, then the headline bench (k_step events + window) and configs[1],
# interleaved.  usage: bash scripts/ab_bench.sh
set -o pipefail
mkdir -p gpurun_out
L=$PWD/gym-ctr-reach_amd/ctr_reach_amd/lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
for v in libctr_reach_amd.so libab_prev.so libctr_reach_amd.so libab_prev.so libctr_reach_amd.so libab_prev.so; do
  for c in 3 2; do
    CTR_REACH_AMD_LIB=$L/$v timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/abb.log 2>&1 || { tail -5 gpurun_out/abb.log; exit 1; }
    python -c "import json; d=json.loads([l for l in open('gpurun_out/abb.log') if l.startswith('{')][-1]); print('$v cfg $c', round(d['ms_per_step']*1e3, 2), 'us/step  k_step', round(d['roofline']['kernel_ms']*1e3, 2))"
  done
done
