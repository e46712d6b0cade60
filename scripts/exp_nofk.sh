#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/exp_nofk
mkdir -p $OUT
CTR_REACH_AMD_LIB=$PWD/gym-ctr-reach_amd/ctr_reach_amd/lib/libctr_reach_amd_nofk.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t -o run -- python3 bench.py --steps 20 --warmup 2 --profile-only > $OUT/t.log 2>&1 || exit 1
CTR_REACH_AMD_LIB=$PWD/gym-ctr-reach_amd/ctr_reach_amd/lib/libctr_reach_amd_nofk.so timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY --output-format csv -d $OUT/a -o run -- python3 bench.py --steps 10 --warmup 2 --profile-only > $OUT/a.log 2>&1 || exit 2
