# Round 3 consolidated pass: suite, refill split, benches (all configs), profile r03 (trace + PMC)
set -o pipefail
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -${TAILN:-2} "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abnormal exit, stopping"; exit $rc; fi
}
TAILN=3 run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run refill_parts_rigid 120 python tools/time_refill_parts.py 4096 rigid
run refill_parts 120 python tools/time_refill_parts.py 65536
run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
run bench_128 300 python bench.py --steps 128 --warmup 5 --no-cpu-baseline
run bench_obs64 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --obs-dtype float64
run bench_c2 300 python bench.py --config 2 --steps 20 --warmup 5 --cpu-seconds 5
run bench_c5 300 python bench.py --config 5 --steps 20 --warmup 5 --cpu-seconds 5
run bench_mixed 300 python bench.py --systems 0,1,2,3 --steps 20 --warmup 5 --cpu-seconds 5
run profile 1200 bash scripts/profile.sh r03
