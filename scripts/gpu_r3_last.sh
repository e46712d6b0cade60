# last evidence of the round on the final tree: suite, smoke, benches, then the reset-pool soak
set -o pipefail
bash scripts/gpu_r3_final.sh || exit $?
timeout -k 10 600 python tools/soak_pool.py > gpurun_out/soak_pool.log 2>&1; rc=$?
tail -2 gpurun_out/soak_pool.log; exit $rc
