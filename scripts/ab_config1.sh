#!/bin/bash
# A/B of engine builds on config 1 (fst_compose_frozen of 1^96 vs eps-dense T=4096 B=12:
# the 781 K-state lattice): kernel and call ms per variant, alternating per round.
# usage: scripts/ab_config1.sh <rounds> <variant> ...   (variant = libfst_amd/variants/<v>.so)
cd "$(dirname "$0")/.." || exit 1
rounds=$1; shift
for r in $(seq 1 "$rounds"); do
  for v in "$@"; do
    LIBFST_AMD_LIB=libfst_amd/variants/$v.so timeout -k 10 200 python -u scripts/bench_configs.py --configs 1 \
      > "gpurun_out/abc1_$v.$r.log" 2>&1 || exit 1
    echo "$v $r $(grep '"config": 1' gpurun_out/abc1_$v.$r.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["gpu_kernel_ms"], d["gpu_call_ms"])')"
  done
done
