#!/bin/bash
# Every GPU call of this repository, as phases (run through gpurun from the repo root):
#   bash scripts/gpu.sh <phase> [<phase> ...]
#   suite     the GPU test suite + smoke
#   bench     headline bench x2 (+ CPU baseline once) and the two-rank gloo rehearsals on one GPU
#             (headline and configs[4]: the push gather's pre-window check, calibration and
#             post-window check)
#   evidence  every bench line: headline x2, 128 steps, float64 observations, configs[1] x2,
#             configs[4] (20 and 128 steps), mixed systems 0-3
#   soak      reset-pool soak (tools/soak_pool.py: pooled vs synchronous resets, bit-equal)
#   pushsoak  fused-push flow-control soak: $WORLD free-running ranks on one GPU (tools/push_soak.py)
#   interf    fused push into 8 blocks on one GPU: per-step cost with and without the fused wait
#   profile   scripts/profile.sh $TAG (kernel trace + PMC passes; tools/summarize_profile.py $TAG here)
#   traffic   k_step / k_refill FETCH_SIZE and WRITE_SIZE at the bench's --steps 20, with the
#             default refill budget and with --refill-budget 0
#   tattrib   k_step reads by source: FETCH_SIZE / WRITE_SIZE passes of tools/traffic_attrib.py
#   fake      RCCL-footprint stand-in (tools/fake_gather.hip, built here into tools/libfake_gather.so)
#             at 2-32 workgroups, durations from a per-channel bandwidth model
#   refill    k_refill timed alone per refill budget (tools/time_refill_budget.py)
#   ab        A/B of the default library against the libraries named in $AB (file names under
#             gym-ctr-reach_amd/ctr_reach_amd/lib, e.g. built by tools/experiments/build_rev.sh):
#             bit-equality of the bench workload, then k_step timing and the headline, interleaved
#   abt       k_step timing only, default library and each of $AB (diagnostic builds)
#   wavet     per-wave k_step durations (libab_wavet.so, -DCTR_DIAG_WAVETIME; tools/wave_times.py)
#   pmcab     PMC passes per library in $AB and the default one (scripts/pmc_ab.sh $TAG ...)
#   tailprobe k_step with extra spinning workgroups (libab_tail.so, tools/experiments/tail_probe.sh)
# Every GPU step runs under its own time limit; the first failing step ends the call.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -${TAILN:-2} "gpurun_out/$name.log" | cut -c1-900
    if [ $rc -ne 0 ]; then echo "step failed, stopping"; exit $rc; fi
}
pmc() {   # pmc <dir> <counter> <bench args...>
    local d=$1 c=$2; shift 2
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/$d -o run -- \
        python3 bench.py "$@" > gpurun_out/$d.log 2>&1
    local rc=$?
    echo "$d rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/$d.log; exit $rc; fi
}
LIBDIR=$PWD/gym-ctr-reach_amd/ctr_reach_amd/lib
for phase in "$@"; do
case "$phase" in
suite)
    TAILN=6 run pytest_gpu 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
    run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
    ;;
bench)
    run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
    run bench_2 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
    TAILN=3 run bench_n2_gloo 300 env CTR_BENCH_BACKEND=gloo CTR_BENCH_SAME_DEVICE=1 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline
    TAILN=3 run bench_c5_n2_gloo 300 env CTR_BENCH_BACKEND=gloo CTR_BENCH_SAME_DEVICE=1 python bench.py --gpus 2 --config 5 --steps 20 --warmup 5 --no-cpu-baseline
    ;;
evidence)
    run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
    run bench_2 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
    run bench_128 300 python bench.py --steps 128 --warmup 5 --no-cpu-baseline
    run bench_obs64 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --obs-dtype float64
    run bench_c2 300 python bench.py --config 2 --steps 20 --warmup 5 --cpu-seconds 5
    run bench_c2b 300 python bench.py --config 2 --steps 20 --warmup 5 --no-cpu-baseline
    run bench_c5 300 python bench.py --config 5 --steps 20 --warmup 5 --cpu-seconds 5
    run bench_c5_128 300 python bench.py --config 5 --warmup 5 --no-cpu-baseline
    run bench_mixed 300 python bench.py --systems 0,1,2,3 --steps 20 --warmup 5 --cpu-seconds 5
    ;;
soak)
    run soak_pool 600 python tools/soak_pool.py
    ;;
pushsoak)
    TAILN=12 run push_soak 600 python tools/push_soak.py ${WORLD:-8} ${STEPS:-200}
    ;;
interf)
    run interf_fused8 200 python tools/gather_interference.py fused 8
    run interf_fused8_wait 200 python tools/gather_interference.py fused 8 wait
    ;;
profile)
    bash scripts/profile.sh ${TAG:-r04} > gpurun_out/profile_${TAG:-r04}.log 2>&1 || { tail -5 gpurun_out/profile_${TAG:-r04}.log; exit 1; }
    tail -3 gpurun_out/profile_${TAG:-r04}.log
    ;;
traffic)
    run bench_base 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
    pmc r4t_fetch_b6 FETCH_SIZE --steps 20 --warmup 5 --profile-only
    pmc r4t_write_b6 WRITE_SIZE --steps 20 --warmup 5 --profile-only
    pmc r4t_fetch_b0 FETCH_SIZE --steps 20 --warmup 5 --profile-only --refill-budget 0
    pmc r4t_write_b0 WRITE_SIZE --steps 20 --warmup 5 --profile-only --refill-budget 0
    ;;
tattrib)
    # k_step reads by source (tools/traffic_attrib.py): one FETCH_SIZE and one WRITE_SIZE pass
    timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/tra_fetch -o run -- \
        python3 tools/traffic_attrib.py run > gpurun_out/tra_fetch.log 2>&1 || { echo "tra_fetch failed"; tail -5 gpurun_out/tra_fetch.log; exit 1; }
    timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/tra_write -o run -- \
        python3 tools/traffic_attrib.py run > gpurun_out/tra_write.log 2>&1 || { echo "tra_write failed"; tail -5 gpurun_out/tra_write.log; exit 1; }
    echo "tattrib ok"
    ;;
fake)
    # 7.3 MB received per GPU and step (7 x 65 536 x 16 B) at ~40 GB/s per channel
    for wd in "2 92" "4 46" "8 23" "16 12" "32 6"; do
        set -- $wd
        run fake_$1 200 python tools/gather_interference.py fake $2 $1
    done
    ;;
refill)
    run time_refill_budget 300 python tools/time_refill_budget.py 65536 ${BUDGETS:-5,6,7,8}
    ;;
ab)
    # (the arrays go to /tmp on the box: gpurun merges at most 64 MiB of gpurun_out back)
    run abits_base 300 python tools/ab_bits.py run /tmp/abits_base.npz
    for v in $AB; do
        run abits_$v 300 env CTR_REACH_AMD_LIB=$LIBDIR/$v python tools/ab_bits.py run /tmp/abits_$v.npz
        TAILN=30 run abits_cmp_$v 60 python tools/ab_bits.py cmp /tmp/abits_base.npz /tmp/abits_$v.npz
    done
    for rep in 1 2; do
        for v in libctr_reach_amd.so $AB; do
            TAILN=3 run steps_${v}_$rep 200 env CTR_REACH_AMD_LIB=$LIBDIR/$v python tools/time_step_modes.py
            run bench_${v}_$rep 300 env CTR_REACH_AMD_LIB=$LIBDIR/$v python bench.py --steps 20 --warmup 5 --no-cpu-baseline
        done
    done
    ;;
abt)
    # timing only (diagnostic builds whose results differ, e.g. -DCTR_DIAG_NOFK): k_step per library
    for v in libctr_reach_amd.so $AB; do
        TAILN=3 run steps_${v} 200 env CTR_REACH_AMD_LIB=$LIBDIR/$v python tools/time_step_modes.py
    done
    ;;
wavet)
    # per-wave durations of k_step (libab_wavet.so, built with -DCTR_DIAG_WAVETIME; tools/wave_times.py)
    TAILN=20 run wave_times 200 env CTR_REACH_AMD_LIB=$LIBDIR/libab_wavet.so python tools/wave_times.py
    ;;
pmcab)
    bash scripts/pmc_ab.sh ${TAG:-ab} libctr_reach_amd.so $AB || exit 1
    ;;
tailprobe)
    for c in "0 0" "64 3000" "128 3000" "256 3000" "64 6000" "128 6000" "256 6000" "0 0" "512 3000" "128 10000"; do
        set -- $c
        run tail_$1_$2 120 env CTR_REACH_AMD_LIB=$LIBDIR/libab_tail.so CTR_TAIL_WG=$1 CTR_TAIL_NS=$2 python tools/tail_probe.py
    done
    ;;
*)
    echo "usage: bash scripts/gpu.sh suite|bench|evidence|soak|pushsoak|interf|profile|traffic|tattrib|fake|refill|ab|abt|wavet|pmcab|tailprobe ..."
    exit 2 ;;
esac
done
