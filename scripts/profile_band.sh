#!/bin/bash
# Profile of the band replay (config 3, kernels/lazy_band.hpp) on the GPU box: the
# rocprofv3 kernel trace, the HBM traffic passes (FETCH_SIZE, WRITE_SIZE: separate passes)
# and two SQ instruction-mix passes, on N (default 8,192) strings of config 3's length
# distribution against the eps-dense rhs at T (default the full 65,536).
# usage: scripts/profile_band.sh [outdir]   (outdir under gpurun_out/)
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
out=${1:-gpurun_out/prof_band}
mkdir -p "$out"
export TMPDIR=/tmp FSTAMD_LAZY_TINY=0
C="scripts/config3_scaling.py --ts ${T:-65536} --n ${N:-8192} --cpu-max-t 0"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM"
scripts/gpu_session.sh \
  "200:bkt:rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o kt -- python3 $C" \
  "200:bfetch:rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o fetch -- python3 $C" \
  "200:bwrite:rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o write -- python3 $C" \
  "200:bsq1:rocprofv3 --pmc $P1 --output-format csv -d $out/sq1 -o p1 -- python3 $C" \
  "200:bsq2:rocprofv3 --pmc $P2 --output-format csv -d $out/sq2 -o p2 -- python3 $C"
