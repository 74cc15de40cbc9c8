#!/bin/bash
# Lane utilisation and LDS conflict counters of the metric's pull kernels (tier P and the
# lazy pull) at 64K strings, one rocprofv3 pass per semantics.
# usage: scripts/profile_lanes.sh [outdir]   (outdir under gpurun_out/)
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
out=${1:-gpurun_out/prof_lanes}
mkdir -p "$out"
export TMPDIR=/tmp
C="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS_ATOMIC SQ_WAVE_CYCLES SQ_INSTS_LDS"
E="bench.py --steps 2 --warmup 1 --no-cpu --lazy-batch 0 --no-varied --no-e2e --no-f64 --global-batch 65536"
scripts/gpu_session.sh \
  "200:lanes_eager:rocprofv3 --pmc $C --output-format csv -d $out/eager -o e -- python3 $E" \
  "200:lanes_lazy:rocprofv3 --pmc $C --output-format csv -d $out/lazy -o l -- python3 $E --semantics lazy"
