#!/bin/bash
# Round-5 profile of the benched build (run on the GPU box via gpurun), each step under its
# own limit, stopping at the first failure (scripts/gpu_session.sh):
#   * eager tier P and the lazy pull, kernel-resident at 1M metric strings: the rocprofv3
#     kernel trace (--stats) and the HBM passes (FETCH_SIZE, WRITE_SIZE: separate passes);
#   * the SQ instruction-mix passes at 64K strings (two passes of <= 8 SQ counters);
#   * the host entry (the headline): kernel + memory-copy trace of scripts/e2e_profile.py.
# usage: scripts/profile_r05.sh [outdir]   (outdir under gpurun_out/)
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
out=${1:-gpurun_out/prof_r05}
mkdir -p "$out"
export TMPDIR=/tmp
C="--no-cpu --lazy-batch 0 --no-varied --no-e2e --no-f64"
BE="bench.py --steps 20 --warmup 2 $C"
BL="bench.py --semantics lazy --steps 20 --warmup 2 $C"
SE="bench.py --steps 2 --warmup 1 $C --batch 65536"
SL="bench.py --semantics lazy --steps 2 --warmup 1 $C --batch 65536"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH"
R="rocprofv3 --output-format csv"
scripts/gpu_session.sh \
  "300:kt_e:$R --kernel-trace --stats -d $out/kt_e -o kt -- python3 $BE" \
  "200:fetch_e:timeout -s KILL 180 $R --pmc FETCH_SIZE -d $out/fetch_e -o fetch -- python3 $BE" \
  "200:write_e:timeout -s KILL 180 $R --pmc WRITE_SIZE -d $out/write_e -o write -- python3 $BE" \
  "150:sq1_e:timeout -s KILL 120 $R --pmc $P1 -d $out/sq1_e -o p1 -- python3 $SE" \
  "150:sq2_e:timeout -s KILL 120 $R --pmc $P2 -d $out/sq2_e -o p2 -- python3 $SE" \
  "300:kt_l:$R --kernel-trace --stats -d $out/kt_l -o kt -- python3 $BL" \
  "200:fetch_l:timeout -s KILL 180 $R --pmc FETCH_SIZE -d $out/fetch_l -o fetch -- python3 $BL" \
  "200:write_l:timeout -s KILL 180 $R --pmc WRITE_SIZE -d $out/write_l -o write -- python3 $BL" \
  "150:sq1_l:timeout -s KILL 120 $R --pmc $P1 -d $out/sq1_l -o p1 -- python3 $SL" \
  "150:sq2_l:timeout -s KILL 120 $R --pmc $P2 -d $out/sq2_l -o p2 -- python3 $SL" \
  "200:e2e_trace:$R --kernel-trace --memory-copy-trace --stats -d $out/e2e -o e2e -- python3 scripts/e2e_profile.py"
