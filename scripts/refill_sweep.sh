set -o pipefail
mkdir -p gpurun_out
for ri in 32 64 128 32 64 128; do
  timeout -k 10 200 python bench.py --steps 256 --warmup 20 --no-cpu-baseline --refill-interval $ri > gpurun_out/ri_$ri.log 2>&1 || exit 1
  python -c "import json; d=json.loads([l for l in open('gpurun_out/ri_$ri.log') if l.startswith('{')][-1]); print($ri, round(d['value']/1e6,1), round(d['ms_per_step']*1e3,1))"
done
