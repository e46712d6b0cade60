# Diagnostic: is k_step's fixed per-launch read (~89 KB per XCD) its whole code object?  FETCH_SIZE
# passes of tools/traffic_attrib.py for the product library and libab_nocareful.so (the same
# source with fk_dispatch_d's CAREFUL instantiation compiled out: a smaller k_step, the executed
# code unchanged).  Summaries: python tools/traffic_attrib.py summarize <fetch dir> <write dir> <tag>
set -o pipefail
export TMPDIR=/tmp
L=$PWD/gym-ctr-reach_amd/ctr_reach_amd/lib
for v in libctr_reach_amd.so libab_nocareful.so; do
  for c in FETCH_SIZE WRITE_SIZE; do
    CTR_REACH_AMD_LIB=$L/$v timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/cf_${v%.so}_$c -o run -- \
      python3 tools/traffic_attrib.py run > gpurun_out/cf_${v%.so}_$c.log 2>&1 || { echo "$v $c failed"; tail -5 gpurun_out/cf_${v%.so}_$c.log; exit 1; }
  done
done
echo done
