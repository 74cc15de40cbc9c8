#!/bin/bash
# A/B of band-replay builds (config 3's kernel, scripts/band_profile.py): strings/s of each
# variant library, variants alternating per round so clock drift hits all of them.
# usage: scripts/ab_band.sh <rounds> <n> <variant> ...   (variant = libfst_amd/variants/<v>.so)
cd "$(dirname "$0")/.." || exit 1
rounds=$1; n=$2; shift 2
for r in $(seq 1 "$rounds"); do
  for v in "$@"; do
    FSTAMD_ROUTE_LOG=1 LIBFST_AMD_LIB=libfst_amd/variants/$v.so timeout -k 10 120 python -u scripts/band_profile.py --n "$n" \
      > "gpurun_out/abb_$v.$r.log" 2>&1 || exit 1
    echo "$v $r $(grep "band plan" gpurun_out/abb_$v.$r.log | tail -1 | cut -c1-120) $(tail -1 gpurun_out/abb_$v.$r.log)"
    sleep 2
  done
done
