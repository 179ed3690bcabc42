#!/bin/bash
# A/B session: each step under its own time limit, stop at the first crash or
# timeout (rc not 0/1).  Outputs under gpurun_out/ab_*.  Steps: $AB_STEPS.
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
step tests 300 python -u -m pytest tests/test_rt_gpu.py tests/test_dist_gpu.py tests/test_rt_big_gpu.py tests/test_rast_gpu.py tests/test_rast_screenshot.py tests/test_rast_tex_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
for i in 1 2; do
  step c2_fused_$i 120 python bench.py --steps 20 --warmup 5 --no-sub --no-draw --no-cpu-baseline --no-steady
  step c2_split_$i 120 env CG_CERT_FUSED=0 python bench.py --steps 20 --warmup 5 --no-sub --no-draw --no-cpu-baseline --no-steady
done
step c4_fused 120 python bench.py --workload c4 --steps 32 --warmup 3 --no-cpu-baseline
step c4_split 120 env CG_CERT_FUSED=0 python bench.py --workload c4 --steps 32 --warmup 3 --no-cpu-baseline
step band_fused 200 python scripts/band_balanced.py 15 fixed
step band_split 200 env CG_CERT_FUSED=0 python scripts/band_balanced.py 15 fixed
step band_fused_moving 200 python scripts/band_balanced.py 15 moving
for i in 1 2; do
  step c5_two_$i 150 python bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline
  step c5_one_$i 150 env CG_BIG_SLOTS=1 python bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline
done
step dist_c5 200 python scripts/dist_probe.py c5 20
cd /tmp
for i in 1 2; do
  step rastlat_new_$i 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rastlat_new_$i -o rast -- python3 $ROOT/scripts/rast_lat.py 300
  step rastlat_old_$i 120 env CGAMD_LIB=$ROOT/computer-graphics_amd/_build_ab/libcgamd.so rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rastlat_old_$i -o rast -- python3 $ROOT/scripts/rast_lat.py 300
done
step trace_band 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_band -o band -- python3 $ROOT/scripts/band_balanced.py 5 fixed
echo ab done
