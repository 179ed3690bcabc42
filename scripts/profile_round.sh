#!/bin/bash
# One GPU session collecting the round's profiles (kernel stats, PMC HBM
# traffic, SQ executed-work counters) for every bench workload; each step has
# its own time limit and a failure stops the script (WLS="rt rast ..." limits
# the workloads).  Then on the CPU:
#   scripts/collect_profiles.sh rNN ; python3 scripts/sq_summary.py ... (see below)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$OUT/$name.log"; exit $rc; }
}
B="python3 $ROOT/bench.py --no-cpu-baseline --no-draw --no-steady"
# the machine code these counters describe (bench.py nulls roofline.frac for other code)
python3 -c "import json, sys; sys.path.insert(0, '$ROOT/computer-graphics_amd'); import codeobj; \
json.dump({k: codeobj.kernel_sha256(k) for k in codeobj.kernel_names()}, open('$OUT/code_sha256.json', 'w'), indent=1)"
WLS=${WLS:-rt rast c4 c5 c5yaw yaw f256}
has() { case " $WLS " in *" $1 "*) return 0;; esac; return 1; }
# every launch of a profiled kernel carries the same frames (the --stats mean is per launch)
for w in $WLS; do
  case $w in c4|yaw|f256) P="--steps 32 --warmup 32";; *) P="";; esac
  run prof_$w 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$w" -o $w -- $B --workload $w --no-sub $P
done
for wl in rt rast c4 c5 c5yaw yaw f256; do
  has $wl || continue
  case $wl in rt|rast) S="--steps 64 --warmup 32";; c4|yaw|f256) S="--steps 32 --warmup 32";; *) S="--steps 4 --warmup 2";; esac
  for ctr in FETCH_SIZE WRITE_SIZE; do
    run pmc_${wl}_$ctr 180 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc_${wl}_$ctr" -o pmc -- $B --workload $wl $S --no-sub
  done
done
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
G2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
G3="SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_TRANS_F SQ_INSTS_VALU_CVT SQ_INST_LEVEL_SMEM"
for w in rt c4 c5 c5yaw yaw f256 rast; do
  has $w || continue
  case $w in rt|c4|yaw|f256) S="--steps 32 --warmup 32";; rast) S="--steps 64 --warmup 64";; *) S="--steps 4 --warmup 2";; esac
  i=0
  for g in "$G1" "$G2" "$G3"; do
    i=$((i+1))
    run sq_${w}_$i 180 rocprofv3 --pmc $g --output-format csv -d "$OUT/sq_${w}_$i" -o sq -- $B --workload $w $S --no-sub
  done
done
echo profiles done
