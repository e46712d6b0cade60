#!/bin/bash
# SQ stall breakdown for k_step (separate --pmc passes).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_sq
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $OUT/a -o run -- python3 bench.py --steps 10 --warmup 2 --profile-only > $OUT/a.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INST_CYCLES_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d $OUT/b -o run -- python3 bench.py --steps 10 --warmup 2 --profile-only > $OUT/b.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT --output-format csv -d $OUT/c -o run -- python3 bench.py --steps 10 --warmup 2 --profile-only > $OUT/c.log 2>&1 || exit 3
