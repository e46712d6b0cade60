# refill budget 5-8 timed alone, then the headline window with budget 6 vs 7 (interleaved)
mkdir -p gpurun_out
timeout -k 10 300 python tools/time_refill_budget.py 65536 5,6,7,8 > gpurun_out/trb.log 2>&1 || exit 1
grep budget gpurun_out/trb.log
for b in 6 7 6 7; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --refill-budget $b > gpurun_out/bb_$b.log 2>&1 || exit 1
    python -c "import json; d=json.loads([l for l in open('gpurun_out/bb_$b.log') if l.startswith('{')][-1]); print($b, round(d['ms_per_step']*1e3, 2))"
done
