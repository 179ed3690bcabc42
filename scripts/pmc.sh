#!/bin/bash
# HBM traffic per kernel from rocprofv3 PMC counters, one counter group per pass
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; MI355X_MICROARCH.md).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
cd /tmp
for wl in rt rast; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$ROOT/gpurun_out/pmc_${wl}_$ctr" -o pmc -- \
        python3 "$ROOT/bench.py" --workload $wl --steps 64 --warmup 32 --no-cpu-baseline \
        > "$ROOT/gpurun_out/pmc_${wl}_$ctr.log" 2>&1 || { echo "pmc $wl $ctr failed"; exit 1; }
  done
done
echo pmc done
