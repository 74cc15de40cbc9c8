#!/bin/bash
# A/B of band-replay settings: "<name>:<variant>:<VAR=VAL ...>" specs, strings/s each,
# alternating per round.  usage: scripts/ab_band_env.sh <rounds> <n> <spec> ...
cd "$(dirname "$0")/.." || exit 1
rounds=$1; n=$2; shift 2
for r in $(seq 1 "$rounds"); do
  for spec in "$@"; do
    name="${spec%%:*}"; rest="${spec#*:}"; v="${rest%%:*}"; vars="${rest#*:}"
    env FSTAMD_ROUTE_LOG=1 LIBFST_AMD_LIB=libfst_amd/variants/$v.so $vars timeout -k 10 120 python -u scripts/band_profile.py --n "$n" \
      > "gpurun_out/abe_$name.$r.log" 2>&1 || exit 1
    echo "$name $r $(tail -1 gpurun_out/abe_$name.$r.log)"
    sleep 2
  done
done
