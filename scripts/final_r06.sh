#!/bin/bash
# Round-6 final-build GPU session: suite, smoke, bench line, configs 1/3m/4/4w/5, and the
# band replay's kernel trace and HBM passes.  Logs under gpurun_out/<stamp>/ (gpu_session.sh).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/final
mkdir -p $o
B="python3 scripts/band_profile.py --n 32768"
scripts/gpu_session.sh \
  "700:suite:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --durations=25" \
  "120:smoke:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "240:bench:python bench.py" \
  "600:configs:python -u scripts/bench_configs.py --configs 1,3m,4,4w,5 --out $o/configs.jsonl" \
  "200:band_kt:rocprofv3 --kernel-trace --stats --output-format csv -d $o/band_kt -o kt -- $B" \
  "200:band_fetch:rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/band_fetch -o fetch -- $B" \
  "200:band_write:rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/band_write -o write -- $B"
