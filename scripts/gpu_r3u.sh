# kernel trace of graph replays vs eager (window_overhead), to find the gaps inside a window
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_window -o run -- python3 tools/window_overhead.py 3 > gpurun_out/trace_window.log 2>&1
echo "rc=$?"; tail -4 gpurun_out/trace_window.log | cut -c1-250
