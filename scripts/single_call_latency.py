"""Per-call latency of the single-string C ABI entries (the drop-in path a per-utterance
caller uses): fst_compose_frozen_shortest_path, and fst_compose_frozen + fst_shortest_path,
on config 4's tagger stand-in (one utterance) and on the metric rhs (1^64 vs the ambiguous
T=4096 chain).  Beside it: the CPU port's compute time per string (oracle/fst_oracle.c,
one thread, batch loop: no per-call handle overhead).  Prints one JSON line per case.

usage: python scripts/single_call_latency.py [--calls N]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import libfst_amd as F  # noqa: E402
import libfst_amd.synthetic as SY  # noqa: E402
from libfst_amd import dist as D  # noqa: E402
import oracle_ffi as O  # noqa: E402  (CPU baseline only)


def median_us(fn, calls):
    fn()  # warm-up (device mirror, pools)
    ts = []
    for _ in range(calls):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=200)
    args = ap.parse_args()
    tagger = SY.to_mutable(SY.tagger()).freeze()
    amb = F.Fst.bench_transducer(F.BENCH_AMBIGUOUS, 4096, 12)
    utt = SY.utterances(np.random.default_rng(3), 1, 22, 22)[0].encode()
    cases = [("tagger, one 22-char utterance", tagger, utt),
             ("ambiguous T=4096, 1^64", amb, bytes([0] * 64))]  # byte 0 -> label 1
    for name, rhs, text in cases:
        a = F.MutableFst.compile_string(text)
        lazy = median_us(lambda: F.compose_frozen_shortest_path(a, rhs, 1), args.calls)
        eager = median_us(lambda: F.shortest_path(F.compose_frozen(a, rhs), 1), args.calls)
        blob = D.blob_bytes(rhs)
        labels = np.frombuffer(text, np.uint8).astype(np.uint32) + 1
        reps = 256
        lab = np.tile(labels, reps).astype(np.uint32)
        offs = (np.arange(reps + 1, dtype=np.uint64) * len(labels))
        cpu = {}
        for sem, key in ((0, "lazy"), (1, "eager")):
            secs, _ = O.batch_time(blob, lab, offs, sem, 1)
            cpu[key] = secs / reps * 1e6
        print(json.dumps({"case": name, "gpu_call_us": {"lazy": lazy, "eager": eager},
                          "cpu_port_us_per_string": cpu, "calls": args.calls}), flush=True)


if __name__ == "__main__":
    main()
