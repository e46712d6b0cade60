# in-stream k_refill durations per budget (kernel trace of tools/time_refill_budget.py)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_budget -o run -- python3 tools/time_refill_budget.py 65536 0,2,4,6,8,12,20 > gpurun_out/trace_budget.log 2>&1
echo "rc=$?"; grep budget gpurun_out/trace_budget.log
