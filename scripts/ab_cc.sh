#!/bin/bash
# A/B of library builds on concurrent single calls (WeText-scale tagger stand-in, the tool
# libfst_amd/concurrent_calls; its RUNPATH lets LD_LIBRARY_PATH pick the build).
# usage: scripts/ab_cc.sh <rounds> <threads> <dir> ...   (dir holds a libfst_amd.so)
cd "$(dirname "$0")/.." || exit 1
rounds=$1; th=$2; shift 2
for r in $(seq 1 "$rounds"); do
  for d in "$@"; do
    LD_LIBRARY_PATH=$d timeout -k 10 200 python -u scripts/concurrent_calls_bench.py --wetext \
      --threads "$th" --calls 500 --cpu-seconds 0.1 > "gpurun_out/abcc_$(basename $d).$r.log" 2>&1 || exit 1
    echo "$(basename $d) $r $(grep calls_per_s gpurun_out/abcc_$(basename $d).$r.log | head -3 | tr '\n' ' ')"
  done
done
