#!/bin/bash
# SQ counters of the RT pixel kernel (one pass per group; no tracing domains).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
cd /tmp
rocprofv3 -L > "$ROOT/gpurun_out/counters_list.txt" 2>&1 || true
i=0
for grp in ${SQ_GROUPS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" \
           "SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE GRBM_COUNT"}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$ROOT/gpurun_out/${SQ_PREFIX:-sq}_$i" -o sq -- \
      python3 "$ROOT/bench.py" ${BENCH_ARGS:-} --steps 32 --warmup 32 --no-cpu-baseline > "$ROOT/gpurun_out/${SQ_PREFIX:-sq}_$i.log" 2>&1 \
      || echo "group $i failed: $(tail -3 $ROOT/gpurun_out/${SQ_PREFIX:-sq}_$i.log)"
done
echo sq done
