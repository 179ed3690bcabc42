#!/bin/bash
# C3 throughput after the C2 loop: which earlier stream set-up serialises the rasteriser's lanes?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"
run() { local n=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > "$OUT/diag_$n.log" 2>&1; local rc=$?; echo "== $n rc=$rc"; [ $rc -le 1 ] || exit $rc; }
run rast_alone 150 python bench.py --workload rast --no-cpu-baseline
run c2c3 200 python bench.py --steps 20 --warmup 5 --sub-frames '' --no-cpu-baseline
run c2c3_noprio 200 env CG_AUX_PRIO=0 python bench.py --steps 20 --warmup 5 --sub-frames '' --no-cpu-baseline
run c2c3_nodraw 200 python bench.py --steps 20 --warmup 5 --sub-frames '' --no-cpu-baseline --no-draw
run c2c3_nodraw_noprio 200 env CG_AUX_PRIO=0 python bench.py --steps 20 --warmup 5 --sub-frames '' --no-cpu-baseline --no-draw
echo diag done
