"""Calls/s of the drop-in single-string entry under concurrency, beside the CPU port.

Runs libfst_amd/concurrent_calls (N host threads, each calling fst_compile_string ->
fst_compose_frozen_shortest_path -> result readback, every result checked) for several N,
and the CPU port (oracle/fst_oracle.c -O3, lazy composeShortestPath per string) on all
nproc threads over the same strings.  One JSON line per configuration.

usage: python scripts/concurrent_calls_bench.py [--threads 1,8,32,128] [--calls 500]
       [--len 64] [--transducer-len 4096]
"""
import argparse
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import bench  # noqa: E402
import libfst_amd as F  # noqa: E402
from libfst_amd import dist as D  # noqa: E402
import oracle_ffi as O  # noqa: E402  (CPU baseline only)

TOOL = os.path.join(REPO, "libfst_amd", "concurrent_calls")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="1,8,32,128")
    ap.add_argument("--calls", type=int, default=500)
    ap.add_argument("--len", type=int, default=64)
    ap.add_argument("--transducer-len", type=int, default=4096)
    ap.add_argument("--rhs", default="ambiguous")
    ap.add_argument("--cpu-seconds", type=float, default=5.0)
    ap.add_argument("--light-check", action="store_true",
                    help="--wetext: check the state count only (no per-arc API reads)")
    ap.add_argument("--stderr-to", default="",
                    help="--wetext: keep the tool's stderr (FSTAMD_HOST_PROF / ROUTE_LOG lines)")
    ap.add_argument("--wetext", action="store_true",
                    help="the WeText-scale tagger stand-in and 4,096 of its utterances "
                         "(libfst_amd/wetext_standin.py) instead of a bench rhs")
    a = ap.parse_args()
    if a.wetext:
        return wetext(a)
    for t in [int(x) for x in a.threads.split(",")]:
        r = subprocess.run([TOOL, "--threads", str(t), "--calls", str(a.calls), "--len", str(a.len),
                            "--transducer-len", str(a.transducer_len), "--rhs", a.rhs],
                           capture_output=True, text=True, timeout=600)
        line = json.loads(r.stdout.strip().splitlines()[-1])
        line["rc"] = r.returncode
        print(json.dumps(line), flush=True)
    nth = bench.nproc()
    kind = F.BENCH_EPS_DENSE if a.rhs == "eps_dense" else F.BENCH_AMBIGUOUS
    blob = D.blob_bytes(F.Fst.bench_transducer(kind, a.transducer_len, 12))
    L = a.len

    def run(n, th):
        secs, _ = O.batch_time(blob, np.ones(n * L, np.uint32),
                               np.arange(n + 1, dtype=np.uint64) * L, 0, th)
        return secs
    n0 = nth * 4
    rate0 = n0 / run(n0, nth)
    n = max(n0, int(rate0 * a.cpu_seconds))
    rate = n / run(n, nth)
    print(json.dumps({"cpu_port_calls_per_s": rate, "threads": nth, "strings": n, "len": L,
                      "rhs": a.rhs, "transducer_len": a.transducer_len,
                      "kind": "port (oracle/fst_oracle.c -O3, lazy composeShortestPath per "
                              "string, no C-ABI handle overhead)"}), flush=True)


def wetext(a):
    """Concurrent single calls on realistic utterances: the WeText-scale tagger stand-in
    (0.43 M states) and its utterances, every result checked against the batch entry; the
    CPU port on nproc threads over the same utterances beside it."""
    import tempfile
    from libfst_amd import wetext_standin as W
    tag = W.tagger()
    blob = W.freeze_blob(tag)
    labels, offsets = W.utterances(np.random.default_rng(11), 4096, tag)
    d = tempfile.mkdtemp()
    bpath, spath = os.path.join(d, "tagger.fst"), os.path.join(d, "utt.bin")
    open(bpath, "wb").write(blob)
    with open(spath, "wb") as f:
        f.write(np.uint32(len(offsets) - 1).tobytes())
        f.write(offsets.astype(np.uint64).tobytes())
        f.write(labels.astype(np.uint32).tobytes())
    for t in [int(x) for x in a.threads.split(",")]:
        r = subprocess.run([TOOL, "--threads", str(t), "--calls", str(a.calls), "--rhs-file", bpath,
                            "--strings-file", spath] + (["--light-check"] if a.light_check else []),
                           capture_output=True, text=True, timeout=600)
        if a.stderr_to:
            with open(f"{a.stderr_to}.{t}", "w") as f:
                f.write(r.stderr)
        line = json.loads(r.stdout.strip().splitlines()[-1])
        line["rc"] = r.returncode
        line["rhs"] = "WeText-scale tagger stand-in (0.43 M states), 4,096 utterances"
        print(json.dumps(line), flush=True)
    nth = bench.nproc()
    secs, _ = O.batch_time(blob, labels, offsets, 0, nth)
    print(json.dumps({"cpu_port_calls_per_s": (len(offsets) - 1) / secs, "threads": nth,
                      "strings": len(offsets) - 1, "rhs": "WeText-scale tagger stand-in",
                      "kind": "port (oracle/fst_oracle.c -O3, lazy composeShortestPath per "
                              "utterance, no C-ABI handle overhead)"}), flush=True)


if __name__ == "__main__":
    main()
