set -o pipefail
for v in ${VARIANTS:-libab_prev.so libctr_reach_amd.so}; do
  CTR_REACH_AMD_LIB=$PWD/gym-ctr-reach_amd/ctr_reach_amd/lib/$v timeout -k 10 120 python bench.py --config 2 --steps 64 --warmup 10 --cpu-seconds 1 > gpurun_out/ab_c2_$v.log 2>&1 || exit 1
  python -c "
import json,sys; d=[json.loads(l) for l in open('gpurun_out/ab_c2_$v.log') if l.startswith('{')][-1]
print('$v', '%.3g env-steps/s  k_step %.1f us  tip L2 max %.2g' % (d['value'], d['roofline']['kernel_ms']*1e3, d['parity']['tip_l2_max_m']))"
done
