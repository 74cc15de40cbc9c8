"""Runs the eager device path on a few metric strings and prints status + work counters
(debug aid: with FSTAMD_WATCHDOG_MS set, a stuck wave reports INTERNAL with the layer it
was in: tuples = 0x10000 | layer, relax = tuples in that layer)."""
import sys
import os
import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import libfst_amd as F  # noqa: E402
from libfst_amd import dist as D  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
L = int(sys.argv[2]) if len(sys.argv) > 2 else 64
dev = torch.device("cuda:0")
blob = D.blob_bytes(F.Fst.bench_transducer(F.BENCH_AMBIGUOUS, 4096, 12))
rhs = D.adopt_on_device(torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev), 0)
b = bench.DeviceBatch(np.full(n, L, np.int64), lambda t: torch.ones(t, dtype=torch.int32), dev)
st = b.run(rhs, F.FST_SEM_EAGER, 0, torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
status = b.status.cpu().numpy()
work = b.work.cpu().numpy()
print("kernel_ms", st.kernel_ms, "grid", st.grid, "launches", st.launches)
print("status", np.unique(status, return_counts=True))
for i in range(min(n, 8)):
    print(i, status[i], hex(int(work[2 * i]) & 0xFFFFFFFF), int(work[2 * i + 1]))
