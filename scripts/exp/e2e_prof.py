"""Host batch entry timing (fst_compose_frozen_shortest_path_batch) on the metric batch,
streamed vs not, pageable vs pinned inputs; FSTAMD_HOST_PROF=1 prints the phases."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import libfst_amd as F

torch.cuda.set_device(0)
rhs = F.Fst.bench_transducer(F.BENCH_AMBIGUOUS, 4096, 12)
B, L = 1 << 20, 64
lab_pg = np.ones(B * L, np.uint32)
off = np.arange(B + 1, dtype=np.uint64) * L
lab_pin = torch.ones(B * L, dtype=torch.int32).pin_memory().numpy().view(np.uint32)
for name, lab in (("pageable", lab_pg), ("pinned", lab_pin)):
    for stream in ("1", ""):
        if stream:
            os.environ.pop("FSTAMD_NO_STREAM", None)
        else:
            os.environ["FSTAMD_NO_STREAM"] = "1"
        r = F.compose_frozen_shortest_path_batch(rhs, lab, off, 1, F.FST_SEM_EAGER)
        del r
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            r = F.compose_frozen_shortest_path_batch(rhs, lab, off, 1, F.FST_SEM_EAGER)
            ts.append(time.perf_counter() - t0)
            del r
        print(f"{name} stream={bool(stream)}: {min(ts)*1e3:.1f} ms (median {sorted(ts)[1]*1e3:.1f})",
              flush=True)
