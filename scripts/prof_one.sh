#!/bin/bash
# usage: scripts/prof_one.sh <tag> <bench args...>  -> gpurun_out/prof_<tag>/*_kernel_stats.csv
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_$TAG" -o "$TAG" -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline "$@" > "$ROOT/gpurun_out/prof_$TAG.log" 2>&1
rc=$?
tail -1 "$ROOT/gpurun_out/prof_$TAG.log" | cut -c1-300
python3 "$ROOT/scripts/kstats.py" "$ROOT/gpurun_out/prof_$TAG/${TAG}_kernel_stats.csv"
exit $rc
