"""Probe: tier P with its labels and/or path arena in pinned host memory (zero-copy over
PCIe) instead of HBM, on the metric batch.  Kernel ms per variant, results checked equal to
the all-device run.  One JSON line per variant."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import libfst_amd as F  # noqa: E402
from libfst_amd import fst as FF  # noqa: E402


def run(rhs, labels, offsets, n, L, arena, reps=5):
    il, ol, w = arena
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    pl = torch.empty(n, dtype=torch.int32, device="cuda")
    po = torch.empty(n, dtype=torch.int64, device="cuda")
    fin = torch.empty(n, dtype=torch.float64, device="cuda")
    cur = torch.zeros(1, dtype=torch.int64, device="cuda")
    desc = FF.FstDeviceBatch(st.data_ptr(), pl.data_ptr(), po.data_ptr(), fin.data_ptr(),
                             il.data_ptr(), ol.data_ptr(), w.data_ptr(), il.numel(),
                             cur.data_ptr(), 0)
    opts = FF.FstBatchOptions(0, F.FST_SEM_EAGER, 0)
    s = torch.cuda.current_stream().cuda_stream
    ms = []
    for i in range(reps + 1):
        rc = F.lib().fst_device_compose_shortest_path(
            rhs.h, C.c_void_p(labels.data_ptr()), C.c_void_p(offsets.data_ptr()), n, L, 1,
            C.byref(opts), C.byref(desc), C.c_void_p(s))
        assert rc == 0
        torch.cuda.synchronize()
        if i:
            ms.append(F.last_launch_stats().kernel_ms)
    assert bool((st == 0).all())
    order = torch.argsort(po.cpu())
    return float(np.median(ms)), ol.cpu()[: n * L].reshape(n, L)[order.numpy()].numpy(), \
        w.cpu()[: n * L].reshape(n, L)[order.numpy()].numpy()


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    L = 64
    torch.cuda.set_device(0)
    rhs = F.Fst.bench_transducer(F.BENCH_AMBIGUOUS, 4096, 12)
    lab_d = torch.ones(n * L, dtype=torch.int32, device="cuda")
    lab_h = torch.ones(n * L, dtype=torch.int32).pin_memory()
    off_d = (torch.arange(n + 1, dtype=torch.int64) * L).cuda()
    cap = n * L + 64

    def arena(host):
        if host:
            return (torch.empty(cap, dtype=torch.int32).pin_memory(),
                    torch.empty(cap, dtype=torch.int32).pin_memory(),
                    torch.empty(cap, dtype=torch.float64).pin_memory())
        return (torch.empty(cap, dtype=torch.int32, device="cuda"),
                torch.empty(cap, dtype=torch.int32, device="cuda"),
                torch.empty(cap, dtype=torch.float64, device="cuda"))
    base = None
    for name, lab, host_out in (("device", lab_d, False), ("host_labels", lab_h, False),
                                ("host_arena", lab_d, True), ("host_both", lab_h, True)):
        ms, ol, w = run(rhs, lab, off_d, n, L, arena(host_out))
        same = None
        if base is None:
            base = (ol, w)
        else:
            same = bool(np.array_equal(ol, base[0]) and np.array_equal(w, base[1]))
        print(json.dumps({"variant": name, "strings": n, "kernel_ms": ms, "same": same}),
              flush=True)


if __name__ == "__main__":
    main()
