# quick check of the current tree: the GPU suite, then one headline bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit 1
python -c "import json; d=json.loads([l for l in open('gpurun_out/bench.log') if l.startswith('{')][-1]); print(round(d['ms_per_step']*1e3, 2), 'us/step, k_step', round(d['roofline']['kernel_ms']*1e3, 2))"
