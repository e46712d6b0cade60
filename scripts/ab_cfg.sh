# A/B of full library variants on one BASELINE config: bash scripts/ab_cfg.sh <config> <steps> lib1.so lib2.so ...
set -o pipefail
mkdir -p gpurun_out
C=$1; S=$2; shift 2
for v in "$@"; do
    CTR_REACH_AMD_LIB=$PWD/gym-ctr-reach_amd/ctr_reach_amd/lib/$v timeout -k 10 150 \
        python bench.py --config $C --steps $S --warmup 10 --cpu-seconds 0.5 > gpurun_out/abc_${C}_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/abc_${C}_$v.log; exit 1; }
    python - "$v" "$C" <<'PY'
import json, sys
v, c = sys.argv[1], sys.argv[2]
d = json.loads([l for l in open("gpurun_out/abc_%s_%s.log" % (c, v)) if l.startswith("{")][-1])
print("config %s %-22s %8.1f M env-steps/s  %.1f us/step  k_step %.2f us  tip L2 max %.2g m" % (c, v, d["value"] / 1e6, d["ms_per_step"] * 1e3, d["roofline"]["kernel_ms"] * 1e3, d["parity"]["tip_l2_max_m"]))
PY
done
