#!/bin/bash
# SQ counter passes (wave cycles, stalls, instruction mix) for the eager metric kernel.
# usage: scripts/sq_counters.sh <outdir> [bench args...]
cd "$(dirname "$0")/.." || exit 1
out=${1:-gpurun_out/sq}; shift
mkdir -p "$out"
export TMPDIR=/tmp
B="bench.py --steps 2 --warmup 1 --no-cpu --lazy-batch 0 --no-varied --no-e2e --no-f64 --scaling weak --batch 65536 $*"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH"
scripts/gpu_session.sh \
  "120:sq_list:rocprofv3 -L > $out/counters.txt 2>&1" \
  "200:sq_p1:rocprofv3 --pmc $P1 --output-format csv -d $out/p1 -o p1 -- python3 $B" \
  "200:sq_p2:rocprofv3 --pmc $P2 --output-format csv -d $out/p2 -o p2 -- python3 $B"
