# push-kernel interference: stream priorities
set -o pipefail
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -${TAILN:-6} "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abnormal exit, stopping"; exit $rc; fi
}
run interf_push8_32p 240 python tools/gather_interference.py push 8 32
run interf_push8_128p 240 python tools/gather_interference.py push 8 128
run interf_push8_32sp 240 env SIDE_PRIO=-1 python tools/gather_interference.py push 8 32
run interf_fake 240 python tools/gather_interference.py fake 20 128
