# the 128-step window with the default pool (P = 152, budget 6 / 32) against --refill-budget 0
# (P = 64, every refill runs its FKs to the end), interleaved; then the pool parity tests and soak
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "pool or carried" > gpurun_out/deep_t.log 2>&1
timeout -k 10 300 python -u tools/soak_pool.py > gpurun_out/deep_soak.log 2>&1
for rep in 1 2 3; do
  for b in default 0; do
    if [ $b = default ]; then BA=""; else BA="--refill-budget 0"; fi
    echo "== $b $rep" >> gpurun_out/deep_ab.log
    timeout -k 10 200 python bench.py --no-cpu-baseline $BA >> gpurun_out/deep_ab.log 2>&1
  done
done
echo "== c5 default" >> gpurun_out/deep_ab.log
timeout -k 10 200 python bench.py --config 5 --no-cpu-baseline >> gpurun_out/deep_ab.log 2>&1
echo "== c5 0" >> gpurun_out/deep_ab.log
timeout -k 10 200 python bench.py --config 5 --no-cpu-baseline --refill-budget 0 >> gpurun_out/deep_ab.log 2>&1
