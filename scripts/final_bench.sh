# Three runs of the driver's bench command, then the rocprof trace + PMC passes (profile.sh).
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_final_$i.log 2>&1 || exit 1
done
bash scripts/profile.sh r02
