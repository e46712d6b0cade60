#!/bin/bash
# Round-4 GPU calls (run through gpurun from the repo root): bash scripts/r4.sh <phase> [<phase> ...]
#   suite    GPU test suite + smoke
#   bench    headline bench x2 (+ CPU baseline once) and the two-rank gloo rehearsal on one GPU
#            (exercises the push gather's pre-window check, calibration and post-window check)
#   interf   fused push into 8 blocks on one GPU: its per-step cost with and without the fused
#            consumer wait
#   profile  scripts/profile.sh r04 (kernel trace + PMC passes; tools/summarize_profile.py r04 here)
#   traffic  k_step / k_refill FETCH_SIZE and WRITE_SIZE at the bench's --steps 20, with the
#            default refill budget and with --refill-budget 0
#   ab       A/B of the default library against the libraries named in $AB (lib/ file names)
#   fake     RCCL-footprint stand-in at 2-32 workgroups (channel caps), durations from a per-channel
#            bandwidth model; needs tools/libfake_gather.so (built here)
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
    ;;
interf)
    run interf_fused8 200 python tools/gather_interference.py fused 8
    run interf_fused8_wait 200 python tools/gather_interference.py fused 8 wait
    ;;
profile)
    bash scripts/profile.sh r04 > gpurun_out/profile_r04.log 2>&1 || { tail -5 gpurun_out/profile_r04.log; exit 1; }
    tail -3 gpurun_out/profile_r04.log
    ;;
traffic)
    run bench_base 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
    pmc r4t_fetch_b6 FETCH_SIZE --steps 20 --warmup 5 --profile-only
    pmc r4t_write_b6 WRITE_SIZE --steps 20 --warmup 5 --profile-only
    pmc r4t_fetch_b0 FETCH_SIZE --steps 20 --warmup 5 --profile-only --refill-budget 0
    pmc r4t_write_b0 WRITE_SIZE --steps 20 --warmup 5 --profile-only --refill-budget 0
    ;;
fake)
    # 7.3 MB received per GPU and step (7 x 65 536 x 16 B) at ~40 GB/s per channel
    for wd in "2 92" "4 46" "8 23" "16 12" "32 6"; do
        set -- $wd
        run fake_$1 200 python tools/gather_interference.py fake $2 $1
    done
    ;;
ab)
    # A/B of the default library against $AB (lib/ names, space-separated): bit-equality of the
    # bench workload (40 steps + one FK with counters), then k_step timing, interleaved twice
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
*)
    echo "usage: bash scripts/r4.sh suite|bench|interf|profile|traffic|fake|ab ..."; exit 2 ;;
esac
done
