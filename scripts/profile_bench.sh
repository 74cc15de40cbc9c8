#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box via gpurun):
#   1) kernel trace + stats (average kernel durations, compared with bench.py's HIP events)
#   2) FETCH_SIZE pass, 3) WRITE_SIZE pass (separate: they do not fit one TCC pass).
# usage: scripts/profile_bench.sh <outdir-under-gpurun_out>
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
out=${1:-gpurun_out/prof}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
B="bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu --lazy-batch 0 --no-varied --no-e2e --no-f64"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o kt -- python3 $B > "$out/kt.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o fetch -- python3 $B > "$out/fetch.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o write -- python3 $B > "$out/write.log" 2>&1
