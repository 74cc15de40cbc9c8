#!/bin/bash
# Runs GPU steps in order; each step has its own time limit.  Stops at the first
# step that times out, aborts or segfaults (never retries a GPU step).
# usage: scripts/gpu_session.sh "<limit_s>:<name>:<command>" ...
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  limit="${spec%%:*}"; rest="${spec#*:}"; name="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] (limit ${limit}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$limit" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 25 "gpurun_out/$name.log"
  case $rc in
    0) ;;
    *) echo "=== stopping: $name ended with $rc"; exit $rc;;
  esac
done
