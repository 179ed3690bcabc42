#!/bin/bash
# Copy a gpu_check/pmc/sq run's outputs (gpurun_out/) into the tracked profiles/ (round r01).
set -eu
cd "$(dirname "$0")/.."
for w in rt rast c4 c5; do
  cp gpurun_out/prof_$w/${w}_kernel_stats.csv profiles/r01_${w}_kernel_stats.csv
  tail -n 1 gpurun_out/bench_$w.log > profiles/r01_bench_$w.json
done
[ -f gpurun_out/bal_rt16.log ] && cp gpurun_out/bal_rt16.log profiles/r01_shard_balance_rt_k16.json
[ -f gpurun_out/bench_gloo4.log ] && cp gpurun_out/bench_gloo4.log profiles/r01_bench_rt_gloo4_rehearsal.log
for i in 1 2 3; do cp gpurun_out/sq_$i/sq_counter_collection.csv profiles/r01_sq/lattice_sq_$i.csv; done
for c in FETCH_SIZE WRITE_SIZE; do
  cp gpurun_out/pmc_rt_$c/pmc_counter_collection.csv profiles/r01_pmc_rt_$c.csv
  cp gpurun_out/pmc_rast_$c/pmc_counter_collection.csv profiles/r01_pmc_rast_$c.csv
done
CG_PMC_RT_FRAMES=32 python3 scripts/pmc_summary.py r01 > /dev/null
python3 scripts/sq_summary.py rt_lattice_kernel > /dev/null
echo collected
