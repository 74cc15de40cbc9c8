"""Where the host batch entry's time goes on the metric batch.

Runs fst_compose_frozen_shortest_path_batch on 1M 1^64 strings vs the ambiguous rhs a few
times (FSTAMD_HOST_PROF=1 prints the host phases to stderr) and measures the box's PCIe
copy rates with plain torch copies (pinned and pageable, both directions), so the
end-to-end figure can be set against its transfer floor.  One JSON line per measurement.
"""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import libfst_amd as F  # noqa: E402


def bw(label, nbytes, fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / reps
    print(json.dumps({"copy": label, "bytes": nbytes, "ms": el * 1e3, "GBps": nbytes / el / 1e9}),
          flush=True)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    sem = F.FST_SEM_LAZY if "lazy" in sys.argv[2:] else F.FST_SEM_EAGER
    torch.cuda.set_device(0)
    gib = 1 << 30
    d = torch.empty(gib, dtype=torch.uint8, device="cuda")
    hp = torch.empty(gib, dtype=torch.uint8).pin_memory()
    hq = torch.empty(gib, dtype=torch.uint8)
    hq.fill_(1)
    bw("d2h_pinned_1GiB", gib, lambda: hp.copy_(d, non_blocking=True))
    bw("h2d_pinned_1GiB", gib, lambda: d.copy_(hp, non_blocking=True))
    bw("d2h_pageable_1GiB", gib, lambda: hq.copy_(d))
    bw("h2d_pageable_256MiB", gib // 4, lambda: d[: gib // 4].copy_(hq[: gib // 4]))
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def duplex():
        with torch.cuda.stream(s1):
            hp.copy_(d, non_blocking=True)
        with torch.cuda.stream(s2):
            d[: gib // 4].copy_(hq[: gib // 4])
    bw("duplex_d2h_1GiB_pinned+h2d_256MiB_pageable", gib + gib // 4, duplex, reps=3)
    del d, hp, hq
    torch.cuda.empty_cache()

    rhs = F.Fst.bench_transducer(F.BENCH_AMBIGUOUS, 4096, 12)
    L = 64
    labels = np.ones(n * L, np.uint32)
    offsets = np.arange(n + 1, dtype=np.uint64) * L
    if "--ab" in sys.argv:  # streamed-batch A/B knobs (FSTAMD_STREAM_AB), timing only
        for ab in ("0", "1", "0", "1"):
            os.environ["FSTAMD_STREAM_AB"] = ab
            ts, ks = [], []
            for i in range(6):
                t0 = time.perf_counter()
                r = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem, 0)
                ts.append(time.perf_counter() - t0)
                ks.append(F.last_launch_stats().kernel_ms)
                assert r.status[0] == F.FST_PATH_OK
                del r
                if i == 5 and ab == "0":  # where the host time goes (stderr)
                    os.environ["FSTAMD_HOST_PROF"] = "1"
                    F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem, 0)
                    os.environ.pop("FSTAMD_HOST_PROF")
            print(json.dumps({"ab": ab, "ms": float(np.median(ts[1:]) * 1e3),
                              "kernel_ms": float(np.median(ks[1:]))}), flush=True)
        os.environ.pop("FSTAMD_STREAM_AB")
    if "--cuts" in sys.argv:  # streamed-batch part cuts (FSTAMD_STREAM_CUTS), timing only
        for cuts in os.environ.get("E2E_CUTS", "167;23,163;125;200;167;100,400").split(";"):
            os.environ["FSTAMD_STREAM_CUTS"] = cuts
            ts = []
            for i in range(6):
                t0 = time.perf_counter()
                r = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem, 0)
                ts.append(time.perf_counter() - t0)
                assert r.status[0] == F.FST_PATH_OK
                del r
            print(json.dumps({"cuts": cuts, "ms": float(np.median(ts[1:]) * 1e3)}), flush=True)
        os.environ.pop("FSTAMD_STREAM_CUTS")
    for i in range(6):
        t0 = time.perf_counter()
        r = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem, 0)
        el = time.perf_counter() - t0
        st = F.last_launch_stats()
        assert r.status[0] == F.FST_PATH_OK and int(r.offsets[-1]) == n * L
        print(json.dumps({"call": i, "strings": n, "ms": el * 1e3, "strings_per_s": n / el,
                          "kernel_ms_sum": st.kernel_ms, "launches": st.launches}), flush=True)
        del r


if __name__ == "__main__":
    main()
