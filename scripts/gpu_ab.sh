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
step tests 300 python -u -m pytest tests/test_rt_gpu.py tests/test_dist_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
B="python bench.py --steps 20 --warmup 5 --no-sub --no-draw --no-cpu-baseline"
for i in 1 2 3; do
  step c2_head2_$i 120 $B
  step c2_old_$i 120 env CG_COLD_HEAD=0 CG_AUX_PRIO=0 $B
  step c2_head4_$i 120 env CG_COLD_HEAD=4 $B
  step c2_prio_$i 120 env CG_COLD_HEAD=0 $B
done
step c2long_new 150 python bench.py --steps 800 --warmup 32 --no-sub --no-draw --no-cpu-baseline --no-steady
step c2long_old 150 env CG_COLD_HEAD=0 CG_AUX_PRIO=0 python bench.py --steps 800 --warmup 32 --no-sub --no-draw --no-cpu-baseline --no-steady
step band_head2 200 python scripts/band_balanced.py 15 fixed
step band_old 200 env CG_COLD_HEAD=0 CG_AUX_PRIO=0 python scripts/band_balanced.py 15 fixed
echo ab done
