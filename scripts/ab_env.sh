#!/bin/bash
# A/B of environment settings on the headline's host entry (scripts/e2e_profile.py, 1M
# metric strings): median ms per call of each setting, settings alternating per round so
# clock drift hits all of them.
# usage: scripts/ab_env.sh <rounds> "<name>:<VAR=VAL ...>" ... [-- extra e2e_profile args]
cd "$(dirname "$0")/.." || exit 1
rounds=$1; shift
specs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do specs+=("$1"); shift; done
[ "$1" = "--" ] && shift
for r in $(seq 1 "$rounds"); do
  for spec in "${specs[@]}"; do
    name="${spec%%:*}"; vars="${spec#*:}"
    env $vars timeout -k 10 100 python -u scripts/e2e_profile.py 1048576 "$@" \
      > "gpurun_out/abv_$name.$r.log" 2>&1 || exit 1
    echo "$name $r $(grep '"call"' "gpurun_out/abv_$name.$r.log" | tail -5 | python3 -c \
      'import sys, json, statistics; print(statistics.median(json.loads(l)["ms"] for l in sys.stdin))')"
  done
done
