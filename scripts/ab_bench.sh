#!/bin/bash
# A/B of library builds on the metric bench (eager tier P + lazy pull), alternating builds
# so clock drift hits both: scripts/ab_bench.sh <rounds> <name=lib.so> ...
# ("default" = libfst_amd/libfst_amd.so).  One JSON summary line per run.
cd "$(dirname "$0")/.." || exit 1
rounds=$1; shift
for r in $(seq 1 "$rounds"); do
  for spec in "$@"; do
    name="${spec%%=*}"; lib="${spec#*=}"
    [ "$lib" = default ] && lib=""
    LIBFST_AMD_LIB="$lib" timeout -k 10 150 python -u bench.py --no-cpu --no-e2e --no-varied \
      --no-f64 --steps 10 --warmup 2 > gpurun_out/ab_$name.$r.json 2> gpurun_out/ab_$name.$r.err
    rc=$?
    python3 - "$name" "$r" "$rc" <<'PY'
import json, sys
name, r, rc = sys.argv[1:]
try:
    d = json.loads(open(f"gpurun_out/ab_{name}.{r}.json").read().strip().splitlines()[-1])
    print(json.dumps({"build": name, "round": int(r), "eager": d["value"],
                      "eager_kernel_ms": d["roofline"]["kernel_ms"], "lazy": d["lazy"]["value"],
                      "lazy_kernel_ms": d["lazy"]["kernel_ms"]}), flush=True)
except Exception as e:
    print(json.dumps({"build": name, "round": int(r), "rc": int(rc), "error": repr(e)}), flush=True)
PY
    case $rc in 124|137|134|139) exit $rc;; esac
  done
done
