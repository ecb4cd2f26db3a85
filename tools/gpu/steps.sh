#!/bin/bash
# Step runner for gpurun calls: `step <name> <timeout_s> <cmd...>` runs one GPU step under its own
# time limit, logs to gpurun_out/$OUT/<name>.log and records the status.  A step that FAILS
# (exit 1-2: test failures) lets the next step run; a step that times out, is killed, aborts or
# segfaults (124 / 137 / 134 / 139 / >128) ends the whole call — nothing more touches the GPU.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-run}
mkdir -p "gpurun_out/$OUT"
export MP4X_TEST_PROGRESS="$PWD/gpurun_out/$OUT/progress.log"
STATUS=0
step() {
  local name=$1 t=$2
  shift 2
  echo "$(date +%T) step $name (limit ${t}s)" | tee -a "gpurun_out/$OUT/progress.log"
  timeout -k 10 "$t" "$@" > "gpurun_out/$OUT/$name.log" 2>&1
  local rc=$?
  echo "$(date +%T) step $name rc=$rc" | tee -a "gpurun_out/$OUT/progress.log"
  tail -3 "gpurun_out/$OUT/$name.log"
  if [ $rc -ne 0 ]; then STATUS=1; fi
  if [ $rc -gt 2 ]; then
    echo "step $name ended abnormally (rc=$rc): no further GPU steps" | tee -a "gpurun_out/$OUT/progress.log"
    exit $rc
  fi
  return 0
}
