set -o pipefail
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -${TAILN:-2} "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abnormal exit, stopping"; exit $rc; fi
}
L=$PWD/gym-ctr-reach_amd/ctr_reach_amd/lib
TAILN=3 run pytest_modes 600 python -u -m pytest tests/test_gpu_modes.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread
for rep in 1 2; do
for v in libab_vc.so libctr_reach_amd.so; do
  CTR_REACH_AMD_LIB=$L/$v run abr_${v}_$rep 120 python tools/time_step_modes.py 4096 rigid
  CTR_REACH_AMD_LIB=$L/$v run ab_${v}_$rep 120 python tools/time_step_modes.py
done
done
run refill_rigid 120 python tools/time_refill.py 4096 rigid
run refill 120 python tools/time_refill.py
run bench_c2 300 python bench.py --config 2 --steps 20 --warmup 5 --no-cpu-baseline
