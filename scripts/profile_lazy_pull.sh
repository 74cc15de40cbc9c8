#!/bin/bash
# Profile of the lazy pull (tier LP, kernels/lazy_pull.hpp) on the metric shape: the
# rocprofv3 kernel trace at 1M strings and two SQ instruction-mix passes at 64K strings.
# usage: scripts/profile_lazy_pull.sh [outdir]   (outdir under gpurun_out/)
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
out=${1:-gpurun_out/prof_lp}
mkdir -p "$out"
export TMPDIR=/tmp
B="bench.py --semantics lazy --steps 5 --warmup 2 --no-cpu --lazy-batch 0 --no-varied --no-e2e --no-f64"
S="bench.py --semantics lazy --steps 2 --warmup 1 --no-cpu --lazy-batch 0 --no-varied --no-e2e --no-f64 --global-batch 65536"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM"
scripts/gpu_session.sh \
  "300:lkt:rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o kt -- python3 $B" \
  "200:lsq1:rocprofv3 --pmc $P1 --output-format csv -d $out/sq1 -o p1 -- python3 $S" \
  "200:lsq2:rocprofv3 --pmc $P2 --output-format csv -d $out/sq2 -o p2 -- python3 $S"
