#!/bin/bash
# A/B session: each step under its own time limit, stop at the first crash or
# timeout (rc not 0/1).  Outputs under gpurun_out/ab_*.  The B side loads
# computer-graphics_amd/_build_ab/libcgamd.so (the same sources built with the
# variant's -D flag).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"; export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $OUT/ab_steps.log
  timeout -k 10 "$to" "$@" > "$OUT/ab_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/ab_steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 "$OUT/ab_$name.log"; exit $rc; fi
}
step tests 300 python -u -m pytest tests/test_rt_big_gpu.py tests/test_dist_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
for i in 1 2; do
  for n in 1 2 3 4; do
    step c5_slots${n}_$i 150 env CG_BIG_SLOTS=$n python bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline
  done
done
step c5yaw_slots1 150 env CG_BIG_SLOTS=1 python bench.py --workload c5yaw --steps 20 --warmup 3 --no-cpu-baseline
step c5yaw_slots2 150 env CG_BIG_SLOTS=2 python bench.py --workload c5yaw --steps 20 --warmup 3 --no-cpu-baseline
step c5yaw_slots3 150 env CG_BIG_SLOTS=3 python bench.py --workload c5yaw --steps 20 --warmup 3 --no-cpu-baseline
echo ab done
