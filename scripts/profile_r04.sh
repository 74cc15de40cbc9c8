#!/bin/bash
# Round-4 profile of the benched build (run on the GPU box via gpurun): the rocprofv3
# kernel trace of bench.py's timed region, the HBM traffic passes (FETCH_SIZE, WRITE_SIZE:
# separate passes) at 1M strings, and the SQ instruction-mix passes at 64K strings.
# usage: scripts/profile_r04.sh [outdir]   (outdir under gpurun_out/)
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
out=${1:-gpurun_out/prof_r04}
mkdir -p "$out"
export TMPDIR=/tmp
B="bench.py --steps 20 --warmup 2 --no-cpu --lazy-batch 0 --no-varied --no-e2e --no-f64"
S="bench.py --steps 2 --warmup 1 --no-cpu --lazy-batch 0 --no-varied --no-e2e --no-f64 --global-batch 65536"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH"
scripts/gpu_session.sh \
  "300:kt:rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o kt -- python3 $B" \
  "300:fetch:rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o fetch -- python3 $B" \
  "300:write:rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o write -- python3 $B" \
  "200:sq1:rocprofv3 --pmc $P1 --output-format csv -d $out/sq1 -o p1 -- python3 $S" \
  "200:sq2:rocprofv3 --pmc $P2 --output-format csv -d $out/sq2 -o p2 -- python3 $S"
