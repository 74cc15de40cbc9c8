#!/bin/bash
# The two SQ instruction-mix passes of the metric bench (eager tier P and lazy pull) at
# 64K strings, each in its own rocprofv3 run.  usage: scripts/profile_sq.sh [outdir]
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
out=${1:-gpurun_out/prof_sq}
mkdir -p "$out"
export TMPDIR=/tmp
S="bench.py --steps 2 --warmup 1 --no-cpu --lazy-batch 0 --no-varied --no-e2e --no-f64 --global-batch 65536"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM"
scripts/gpu_session.sh \
  "200:sq1:rocprofv3 --pmc $P1 --output-format csv -d $out/sq1 -o p1 -- python3 $S" \
  "200:sq2:rocprofv3 --pmc $P2 --output-format csv -d $out/sq2 -o p2 -- python3 $S"
