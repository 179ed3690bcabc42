#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/timeout (rc not 0/1) stops the
# script before any further GPU work.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
MODE=${1:-all}
rocminfo 2>/dev/null | grep -m3 -E "Marketing|gfx" > "$OUT/device.txt" || true
nproc > "$OUT/nproc.txt"; lscpu | grep -E "Model name|^CPU\(s\)" >> "$OUT/nproc.txt" || true
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  step pytest_gpu 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench_rt 600 python bench.py
  step bench_rast 300 python bench.py --workload rast
  step bench_c4 300 python bench.py --workload c4 --steps 30 --warmup 3
  step bench_c5 300 python bench.py --workload c5 --steps 20 --warmup 2
  step bench_yaw 300 python bench.py --workload yaw
  step bench_f256 300 python bench.py --workload f256
  step bench_c5yaw 300 python bench.py --workload c5yaw --steps 20 --warmup 2
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  cd /tmp
  step rocprof_rt 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rt" -o rt -- \
      python3 "$ROOT/bench.py" --no-cpu-baseline
  step rocprof_rast 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rast" -o rast -- \
      python3 "$ROOT/bench.py" --workload rast --no-cpu-baseline
  step rocprof_c4 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c4" -o c4 -- \
      python3 "$ROOT/bench.py" --workload c4 --steps 10 --warmup 2 --no-cpu-baseline
  step rocprof_c5 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c5" -o c5 -- \
      python3 "$ROOT/bench.py" --workload c5 --steps 10 --warmup 2 --no-cpu-baseline
  cd "$ROOT"
fi
echo done
