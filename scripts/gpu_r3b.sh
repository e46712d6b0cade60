# Round 3, second GPU pass: push-kernel gather (tests, interference), evaluation-info tests,
# k_step A/B against the round-2 library, two-rank push rehearsal, then the whole suite.
set -o pipefail
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -${TAILN:-6} "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abnormal exit, stopping"; exit $rc; fi
}
L=$PWD/gym-ctr-reach_amd/ctr_reach_amd/lib
TAILN=8 run pytest_new 300 python -u -m pytest tests/test_gpu_gather.py tests/test_gpu_eval.py -x -v --timeout 120 --timeout-method thread
run interf_push8 240 python tools/gather_interference.py push 8 128
run interf_push8_32 240 python tools/gather_interference.py push 8 32
run interf_push8_512 240 python tools/gather_interference.py push 8 512
for v in libctr_reach_amd.so libab_r2.so libctr_reach_amd.so libab_r2.so; do
  CTR_REACH_AMD_ALLOW_ABI=10 CTR_REACH_AMD_LIB=$L/$v run ab_$v 120 python tools/time_step_modes.py
done
run bench_n2_push 300 env CTR_BENCH_BACKEND=gloo CTR_BENCH_SAME_DEVICE=1 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline
run bench_n2_rccl_gloo 300 env CTR_BENCH_BACKEND=gloo CTR_BENCH_SAME_DEVICE=1 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline --gather-backend rccl
TAILN=12 run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
