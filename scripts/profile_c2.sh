# rocprofv3 kernel trace of configs[1] (4 096 envs, rigid, RK4) at the driver's window and at 128 steps.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/prof_c2
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t20 -o run -- \
    python3 bench.py --config 2 --steps 20 --warmup 5 --no-cpu-baseline > $O/b20.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t128 -o run -- \
    python3 bench.py --config 2 --steps 128 --warmup 5 --no-cpu-baseline > $O/b128.log 2>&1 || exit 2
timeout -k 10 200 python3 bench.py --config 2 --steps 128 --warmup 5 --no-cpu-baseline > $O/plain128.log 2>&1 || exit 3
echo done
