#!/bin/bash
# SQ instruction counts of one band-replay build (scripts/band_profile.py, n strings):
# VALU / SALU / LDS / VMEM instructions and wave cycles, one rocprofv3 pass.
# usage: scripts/sq_band_variant.sh <variant> <n> <outdir>
cd "$(dirname "$0")/.." || exit 1
v=$1; n=$2; out=$3
mkdir -p "$out"
export TMPDIR=/tmp
LIBFST_AMD_LIB=libfst_amd/variants/$v.so timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY \
  --output-format csv -d "$out/$v" -o sq -- python3 scripts/band_profile.py --n "$n"
