#!/bin/bash
# Round-6 profiles (run on the GPU box via gpurun), each step under its own limit, stopping
# at the first failure (scripts/gpu_session.sh).  Steps by name: kt_e fetch_e write_e sq1_e
# sq2_e (eager tier P, 1M / 64K metric strings), kt_l fetch_l write_l sq1_l sq2_l (the lazy
# pull), sq1_lf sq2_lf kt_lf (the lazy pull with f64 cells, FSTAMD_LP_F64=1), e2e (host
# entry: kernel + memory-copy trace).
# usage: scripts/profile_r06.sh <outdir under gpurun_out/> <step> ...
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
out=$1; shift
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
specs=()
for s in "$@"; do
  case $s in
    kt_e) specs+=("300:kt_e:$R --kernel-trace --stats -d $out/kt_e -o kt -- python3 $BE");;
    fetch_e) specs+=("200:fetch_e:timeout -s KILL 180 $R --pmc FETCH_SIZE -d $out/fetch_e -o fetch -- python3 $BE");;
    write_e) specs+=("200:write_e:timeout -s KILL 180 $R --pmc WRITE_SIZE -d $out/write_e -o write -- python3 $BE");;
    sq1_e) specs+=("150:sq1_e:timeout -s KILL 120 $R --pmc $P1 -d $out/sq1_e -o p1 -- python3 $SE");;
    sq2_e) specs+=("150:sq2_e:timeout -s KILL 120 $R --pmc $P2 -d $out/sq2_e -o p2 -- python3 $SE");;
    kt_l) specs+=("300:kt_l:$R --kernel-trace --stats -d $out/kt_l -o kt -- python3 $BL");;
    fetch_l) specs+=("200:fetch_l:timeout -s KILL 180 $R --pmc FETCH_SIZE -d $out/fetch_l -o fetch -- python3 $BL");;
    write_l) specs+=("200:write_l:timeout -s KILL 180 $R --pmc WRITE_SIZE -d $out/write_l -o write -- python3 $BL");;
    sq1_l) specs+=("150:sq1_l:timeout -s KILL 120 $R --pmc $P1 -d $out/sq1_l -o p1 -- python3 $SL");;
    sq2_l) specs+=("150:sq2_l:timeout -s KILL 120 $R --pmc $P2 -d $out/sq2_l -o p2 -- python3 $SL");;
    kt_lf) specs+=("300:kt_lf:FSTAMD_LP_F64=1 $R --kernel-trace --stats -d $out/kt_lf -o kt -- python3 $BL");;
    sq1_lf) specs+=("150:sq1_lf:FSTAMD_LP_F64=1 timeout -s KILL 120 $R --pmc $P1 -d $out/sq1_lf -o p1 -- python3 $SL");;
    sq2_lf) specs+=("150:sq2_lf:FSTAMD_LP_F64=1 timeout -s KILL 120 $R --pmc $P2 -d $out/sq2_lf -o p2 -- python3 $SL");;
    e2e) specs+=("200:e2e:$R --kernel-trace --memory-copy-trace --stats -d $out/e2e -o e2e -- python3 scripts/e2e_profile.py");;
    *) echo "unknown step $s"; exit 2;;
  esac
done
scripts/gpu_session.sh "${specs[@]}"
