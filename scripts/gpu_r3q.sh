# window overhead: host window vs GPU time, graph vs eager; bench --graph on/off interleaved
set -o pipefail
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -${TAILN:-2} "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abnormal exit, stopping"; exit $rc; fi
}
TAILN=6 run window 180 python tools/window_overhead.py 5
for i in 1 2 3; do
  run bench_gon_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --graph on
  run bench_goff_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --graph off
done
