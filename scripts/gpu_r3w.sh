# kernel trace of the configs[1] bench (graph replays)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_c2 -o run -- python3 bench.py --config 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/trace_c2.log 2>&1
echo "rc=$?"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/trace_c2.log
