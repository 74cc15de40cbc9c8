#!/bin/bash
# A/B of library builds on the per-utterance paths (LDS replays): single-call latency sweep
# and config 4 / 4w, alternating builds so clock drift hits both.
# usage: scripts/ab_calls.sh <rounds> <name=lib.so> ...   (run on the GPU box)
cd "$(dirname "$0")/.." || exit 1
rounds=$1; shift
for r in $(seq 1 "$rounds"); do
  for spec in "$@"; do
    name="${spec%%=*}"; lib="${spec#*=}"
    export LIBFST_AMD_LIB="$lib"
    s=$(timeout -k 10 120 python -u scripts/single_call_profile.py --calls 100 --sweep 32 2>/dev/null \
        | grep -o '"mean_us": [0-9.]*' | grep -o '[0-9.]*$') || exit 1
    c=$(timeout -k 10 150 python -u scripts/bench_configs.py --configs 4,4w 2>/dev/null \
        | python3 -c 'import sys, json
print(" ".join("%.3g" % d["strings_per_s"] for d in map(json.loads, (l for l in sys.stdin if l.startswith("{"))) if "lazy" in d.get("workload", "")))') || exit 1
    echo "{\"build\": \"$name\", \"round\": $r, \"sweep_mean_us\": $s, \"cfg4_4w_lazy\": \"$c\"}"
  done
done
