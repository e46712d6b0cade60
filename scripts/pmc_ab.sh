# PMC passes of bench.py --profile-only per library variant (A/B of kernel designs).
# usage: [BENCH_ARGS="--config 5"] bash scripts/pmc_ab.sh tag lib1.so lib2.so ...   -> gpurun_out/pmcab_<tag>/<lib>/<pass>/
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
P1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS"
P2="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE"
for v in "$@"; do
    O=gpurun_out/pmcab_$TAG/$v
    mkdir -p $O
    i=0
    for P in "$P1" "$P2"; do
        i=$((i+1))
        CTR_REACH_AMD_LIB=$PWD/gym-ctr-reach_amd/ctr_reach_amd/lib/$v timeout -s KILL 120 rocprofv3 --pmc $P \
            --output-format csv -d $O/p$i -o run -- python3 bench.py --steps 10 --warmup 2 --profile-only ${BENCH_ARGS:-} \
            > $O/p$i.log 2>&1 || { echo "$v pass $i failed"; tail -5 $O/p$i.log; exit 1; }
    done
done
echo pmc_ab done
