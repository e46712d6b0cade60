# A/B timing of library variants: bash scripts/ab.sh lib1.so lib2.so ...  (paths relative to
# gym-ctr-reach_amd/ctr_reach_amd/lib).  Prints env-steps/s and k_step ms per variant.
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
    CTR_REACH_AMD_LIB=$PWD/gym-ctr-reach_amd/ctr_reach_amd/lib/$v timeout -k 10 120 \
        python bench.py --steps 128 --warmup 10 --cpu-seconds 0.5 > gpurun_out/ab_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ab_$v.log; exit 1; }
    python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
line = [l for l in open("gpurun_out/ab_%s.log" % v) if l.startswith("{")][-1]
d = json.loads(line)
print("%-34s %8.1f M env-steps/s   k_step %.1f us   tip L2 max %.2g m  reached agree %.6f" % (v, d["value"] / 1e6, d["roofline"]["kernel_ms"] * 1e3, d["parity"]["tip_l2_max_m"], d["parity"]["reached_flag_agreement"]))
PY
done
