# configs[4] pair kernel: k_step timing per deal variant (tools/time_step_modes.py c5), then the
# configs[4] rocprof profile of the default library (scripts/profile.sh r06_c5)
set -o pipefail
mkdir -p gpurun_out
L=gym-ctr-reach_amd/ctr_reach_amd/lib
for rep in 1 2; do
  for v in libctr_reach_amd.so libab_nosort.so libab_adj.so libab_onelane.so; do
    echo "== $v $rep" >> gpurun_out/deal_ab.log
    CTR_REACH_AMD_LIB=$L/$v timeout -k 10 200 python tools/time_step_modes.py 65536 c5 >> gpurun_out/deal_ab.log 2>&1 || exit 1
  done
done
echo timing done
BENCH_ARGS="--config 5" bash scripts/profile.sh r06_c5 > gpurun_out/profile_r06_c5.log 2>&1 || { tail -5 gpurun_out/profile_r06_c5.log; exit 1; }
echo profile done
