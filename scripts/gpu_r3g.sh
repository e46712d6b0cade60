# refill queue built by a scan (no appends in k_step) + rigid-group prefetch: suite, A/B, refill timing, benches
set -o pipefail
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -${TAILN:-6} "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abnormal exit, stopping"; exit $rc; fi
}
L=$PWD/gym-ctr-reach_amd/ctr_reach_amd/lib
TAILN=4 run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
for v in libctr_reach_amd.so libab_base.so libctr_reach_amd.so libab_base.so; do
  CTR_REACH_AMD_LIB=$L/$v run ab_$v 120 python tools/time_step_modes.py
  CTR_REACH_AMD_LIB=$L/$v run abr_$v 120 python tools/time_step_modes.py 4096 rigid
done
run time_refill 120 python tools/time_refill.py
run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
run bench_c2 300 python bench.py --config 2 --steps 20 --warmup 5 --no-cpu-baseline
