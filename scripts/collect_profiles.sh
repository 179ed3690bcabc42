#!/bin/bash
# Copy a gpu_check/pmc/sq run's outputs (gpurun_out/) into the tracked profiles/.
# usage: scripts/collect_profiles.sh <round tag, e.g. r02>   (only what the run produced is copied)
set -eu
cd "$(dirname "$0")/.."
R=${1:-r02}
for w in rt rast c4 c5 c5yaw yaw f256; do
  [ -f gpurun_out/prof_$w/${w}_kernel_stats.csv ] && cp gpurun_out/prof_$w/${w}_kernel_stats.csv profiles/${R}_${w}_kernel_stats.csv
  [ -f gpurun_out/bench_$w.log ] && tail -n 1 gpurun_out/bench_$w.log > profiles/${R}_bench_$w.json
done
[ -f gpurun_out/pytest_gpu.log ] && tail -n 3 gpurun_out/pytest_gpu.log > profiles/${R}_pytest_gpu_tail.log
[ -f gpurun_out/bal_rt16.log ] && cp gpurun_out/bal_rt16.log profiles/${R}_shard_balance_rt_k16.json
pmc=0
for w in rt rast c4 c5 c5yaw yaw f256; do
  for c in FETCH_SIZE WRITE_SIZE; do
    if [ -f gpurun_out/pmc_${w}_$c/pmc_counter_collection.csv ]; then
      cp gpurun_out/pmc_${w}_$c/pmc_counter_collection.csv profiles/${R}_pmc_${w}_$c.csv
      pmc=1
    fi
  done
done
[ $pmc = 1 ] && CG_PMC_RT_FRAMES=32 python3 scripts/pmc_summary.py $R > /dev/null
echo collected
