"""Where one drop-in fst_compose_frozen_shortest_path call spends its time:
the WeText-scale tagger stand-in (libfst_amd/wetext_standin.py) and one of its utterances,
compiled with fst_compile_string exactly as the OnType caller does.  Prints the median call
latency over --calls calls, then one call with FSTAMD_HOST_PROF=1 (host phases on stderr).
Run it under rocprofv3 --kernel-trace --hip-runtime-trace for the API / kernel breakdown.

usage: python scripts/single_call_profile.py [--calls N] [--utt I] [--eager]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import libfst_amd as F  # noqa: E402
from libfst_amd import wetext_standin as W  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--utt", type=int, default=0)
    ap.add_argument("--eager", action="store_true")
    ap.add_argument("--sweep", type=int, default=0,
                    help="also time the first N utterances (20 calls each): length vs latency")
    a = ap.parse_args()
    tag = W.tagger()
    rhs = F.Fst.from_bytes(W.freeze_blob(tag))
    labels, offsets = W.utterances(np.random.default_rng(11), 64, tag)
    lab = labels[int(offsets[a.utt]):int(offsets[a.utt + 1])]
    text = bytes((lab - 1).astype(np.uint8).tolist())  # compileString: label = byte + 1
    lhs = F.MutableFst.compile_string(text)

    def call():
        if a.eager:
            return F.shortest_path(F.compose_frozen(lhs, rhs), 1)
        return F.compose_frozen_shortest_path(lhs, rhs, 1)
    r = call()  # warm-up: device mirror, pools, engines
    assert r is not None
    ts = []
    for _ in range(a.calls):
        t0 = time.perf_counter()
        call()
        ts.append(time.perf_counter() - t0)
    print(json.dumps({"utterance_labels": int(len(lab)), "calls": a.calls,
                      "semantics": "eager" if a.eager else "lazy",
                      "median_us": float(np.median(ts)) * 1e6,
                      "p10_us": float(np.percentile(ts, 10)) * 1e6,
                      "p90_us": float(np.percentile(ts, 90)) * 1e6}), flush=True)
    if a.sweep:
        rows = []
        for u in range(a.sweep):
            lb = labels[int(offsets[u]):int(offsets[u + 1])]
            x = F.MutableFst.compile_string(bytes((lb - 1).astype(np.uint8).tolist()))
            F.compose_frozen_shortest_path(x, rhs, 1)
            tt = []
            for _ in range(20):
                t0 = time.perf_counter()
                F.compose_frozen_shortest_path(x, rhs, 1)
                tt.append(time.perf_counter() - t0)
            rows.append((int(len(lb)), float(np.median(tt)) * 1e6, F.last_launch_stats().kernel_ms))
        rows.sort()
        lens = np.array([r[0] for r in rows])
        us = np.array([r[1] for r in rows])
        print(json.dumps({"sweep": a.sweep, "mean_len": float(lens.mean()),
                          "mean_us": float(us.mean()), "median_us": float(np.median(us)),
                          "by_len": [[r[0], round(r[1], 1), round(r[2] * 1e3, 1)] for r in rows]}),
              flush=True)
    os.environ["FSTAMD_HOST_PROF"] = "1"
    call()


if __name__ == "__main__":
    main()
