"""Debug helper: run tiny lazy cases on the GPU and print per-string status and
work counters next to the oracle's (tuples X, relaxations R)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import libfst_amd as F  # noqa: E402
import oracle_ffi as O  # noqa: E402
from bench import DeviceBatch  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(0)
for (T, B, lens) in [(8, 12, [0, 1, 2, 3, 5]), (64, 12, [8, 16]), (4096, 12, [64])]:
    rhs = F.Fst.bench_transducer(F.BENCH_AMBIGUOUS, T, B)
    blob = O.freeze(O.gen("ambiguous", T, B))
    for sem in (F.FST_SEM_LAZY, F.FST_SEM_EAGER):
        b = DeviceBatch(np.array(lens), lambda t: torch.ones(t, dtype=torch.int32), dev)
        st = b.run(rhs, sem, 0, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        lab = np.ones(sum(lens), np.uint32)
        offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        ref = O.batch_run(blob, lab, offs, 0 if sem == F.FST_SEM_LAZY else 1)
        print(f"T={T} sem={sem} kernel_ms={st.kernel_ms:.3f}", flush=True)
        print("  status", b.status.cpu().numpy(), "plen", b.plen.cpu().numpy(),
              "poff", b.poff.cpu().numpy(), flush=True)
        print("  work  ", b.work.cpu().numpy().reshape(-1, 2).tolist(), flush=True)
        print("  oracle X,R", list(zip(ref.tuples.tolist(), ref.relaxations.tolist())), flush=True)
