#!/bin/bash
# rocprofv3 kernel-trace stats + PMC passes for bench.py (run on the GPU box).
# usage: [BENCH_ARGS="--config 5"] bash scripts/profile.sh <tag>
#   BENCH_ARGS  extra bench.py arguments for every pass (default: the headline, configs[2])
set -o pipefail
TAG=${1:-r01}
BA=${BENCH_ARGS:-}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline $BA > $OUT/bench_under_trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
    python3 bench.py --steps 10 --warmup 2 --profile-only $BA > $OUT/pmc1.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
    python3 bench.py --steps 10 --warmup 2 --profile-only $BA > $OUT/pmc2.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_valu -o run -- \
    python3 bench.py --steps 10 --warmup 2 --profile-only $BA > $OUT/pmc3.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_THREAD_CYCLES_VALU --output-format csv -d $OUT/pmc_f64 -o run -- \
    python3 bench.py --steps 10 --warmup 2 --profile-only $BA > $OUT/pmc4.log 2>&1 || echo "pmc4 failed (counter names?)"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS --output-format csv -d $OUT/pmc_mix -o run -- \
    python3 bench.py --steps 10 --warmup 2 --profile-only $BA > $OUT/pmc5.log 2>&1 || echo "pmc5 failed (counter names?)"
# FETCH_SIZE / WRITE_SIZE calibration for k_step's access shapes (tools/traffic_probe.hip)
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/probe_fetch -o run -- \
    ./tools/traffic_probe > $OUT/probe1.log 2>&1 || exit 6
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/probe_write -o run -- \
    ./tools/traffic_probe > $OUT/probe2.log 2>&1 || exit 7
find $OUT -name "*.csv" | head -50
