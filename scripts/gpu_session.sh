#!/bin/bash
# Runs GPU steps in order; each step has its own time limit.  Stops at the first
# step that times out, aborts or segfaults (never retries a GPU step).
# usage: scripts/gpu_session.sh "<limit_s>:<name>:<command>" ...
# Each call writes its logs under gpurun_out/<stamp>/ (stamp = UTC start time, or
# $SESSION_TAG), so a failed run's logs are never overwritten by the next call.
cd "$(dirname "$0")/.." || exit 1
stamp="${SESSION_TAG:-$(date -u +%Y%m%dT%H%M%S)}"
dir="gpurun_out/$stamp"
mkdir -p "$dir"
export TMPDIR=/tmp
export PYTHONFAULTHANDLER=1
echo "=== session $stamp: logs in $dir/"
for spec in "$@"; do
  limit="${spec%%:*}"; rest="${spec#*:}"; name="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] (limit ${limit}s): $cmd"
  echo "$cmd" > "$dir/$name.cmd"
  start=$(date +%s)
  timeout -k 10 "$limit" bash -c "$cmd" > "$dir/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 25 "$dir/$name.log"
  case $rc in
    0) ;;
    *) echo "=== stopping: $name ended with $rc (full log: $dir/$name.log)"; exit $rc;;
  esac
done
