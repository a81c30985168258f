#!/bin/bash
# Run a GPU step under its own time limit; abort the whole script on a
# timeout / crash / signal (never start more GPU work after one).
# usage: gpu_step <timeout_s> <log> <cmd...>
gpu_step() {
  local t=$1; shift
  local log=$1; shift
  timeout -k 10 "$t" "$@" > "$log" 2>&1
  local rc=$?
  echo "step '$*' rc=$rc $(date +%T)" >> "$GRAFT_REPO_ROOT/gpurun_out/progress.txt"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -ge 128 ]; then
    echo "fatal rc=$rc in: $*" >> "$GRAFT_REPO_ROOT/gpurun_out/progress.txt"
    exit $rc
  fi
  return 0
}
