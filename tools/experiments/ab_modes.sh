# k_step timing for configs[1] (rigid) and configs[4] (c5) plus their bench lines, default library
# against each of $AB, interleaved (tools/time_step_modes.py)
set -o pipefail
mkdir -p gpurun_out
L=gym-ctr-reach_amd/ctr_reach_amd/lib
for rep in 1 2; do
  for v in libctr_reach_amd.so $AB; do
    for m in "4096 rigid 2" "65536 c5 5"; do
      set -- $m
      echo "== $v $2 $rep" >> gpurun_out/ab_modes.log
      CTR_REACH_AMD_LIB=$L/$v timeout -k 10 200 python tools/time_step_modes.py $1 $2 >> gpurun_out/ab_modes.log 2>&1 || exit 1
      CTR_REACH_AMD_LIB=$L/$v timeout -k 10 200 python bench.py --config $3 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_modes_tmp.log 2>&1 || exit 1
      grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_modes_tmp.log >> gpurun_out/ab_modes.log
    done
  done
done
echo done
