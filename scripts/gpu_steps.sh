#!/bin/bash
# A GPU session: each line of the steps file is "name timeout command...", run in order, each
# under its own time limit; stops at the first crash or timeout (rc not 0/1).  Logs under
# gpurun_out/steps_<name>.log.  Usage: bash scripts/gpu_steps.sh STEPS_FILE
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
while read -r name to cmd; do
  [ -z "$name" ] || [ "${name:0:1}" = "#" ] && continue
  echo "== $name"
  timeout -k 10 "$to" bash -c "$cmd" > "$OUT/steps_$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"; tail -3 "$OUT/steps_$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done < "$1"
echo steps done
