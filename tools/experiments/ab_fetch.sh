# A/B of k_step FETCH_SIZE / WRITE_SIZE per library ($AB, plus the default one): one PMC pass per
# counter and library on the headline bench (--profile-only), then tools/pmc_ab_summary.py-style
# averages; and the usual bit-equality / timing A/B (scripts/gpu.sh ab)
set -o pipefail
export TMPDIR=/tmp
L=$PWD/gym-ctr-reach_amd/ctr_reach_amd/lib
for v in libctr_reach_amd.so $AB; do
  for c in FETCH_SIZE WRITE_SIZE; do
    O=gpurun_out/abf_$v/$c
    mkdir -p $O
    CTR_REACH_AMD_LIB=$L/$v timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O -o run -- \
        python3 bench.py --steps 10 --warmup 2 --profile-only ${BENCH_ARGS:-} > $O.log 2>&1 || { echo "$v $c failed"; tail -3 $O.log; exit 1; }
  done
done
echo fetch done
