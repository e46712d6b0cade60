# refill-interval / pool-depth / refill-budget sweep of the bench (one GPU box call)
set -e
mkdir -p gpurun_out
run() { timeout -k 10 150 python bench.py --no-cpu-baseline "$@" >> gpurun_out/sweep.log 2>&1; echo "ARGS $*" >> gpurun_out/sweep.log; }
run --config 3 --steps 128
run --config 3 --steps 128 --refill-interval 16 --refill-budget 6
run --config 3 --steps 128 --refill-interval 16 --refill-budget 3
run --config 3 --steps 128 --refill-interval 16 --refill-budget 0
run --config 3 --steps 128 --refill-interval 32 --refill-budget 0
run --config 5 --steps 128
run --config 5 --steps 128 --refill-interval 16 --refill-budget 32
run --config 5 --steps 128 --refill-interval 32 --refill-budget 0
run --config 2 --steps 128
run --config 2 --steps 128 --refill-interval 16
