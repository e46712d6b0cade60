set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench/launch_cost > gpurun_out/launch_cost.log 2>&1 || exit 1
cat gpurun_out/launch_cost.log
echo "== HIP_FORCE_DEV_KERNARG=0"
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 120 ./tools/ubench/launch_cost > gpurun_out/launch_cost_hostka.log 2>&1 || exit 2
cat gpurun_out/launch_cost_hostka.log
