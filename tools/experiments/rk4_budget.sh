set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for b in 16 24 32 48; do
  echo "== budget $b rep $rep" >> gpurun_out/rk4_budget.log
  timeout -k 10 200 python bench.py --config 5 --steps 20 --warmup 5 --no-cpu-baseline --refill-budget $b > gpurun_out/rb_tmp.log 2>&1 || exit 1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/rb_tmp.log >> gpurun_out/rk4_budget.log
done; done
echo done
