"""Three host batch calls on the metric batch (streamed unless FSTAMD_NO_STREAM), for traces."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import libfst_amd as F

torch.cuda.set_device(0)
rhs = F.Fst.bench_transducer(F.BENCH_AMBIGUOUS, 4096, 12)
B, L = 1 << 20, 64
lab = np.ones(B * L, np.uint32)
off = np.arange(B + 1, dtype=np.uint64) * L
for _ in range(3):
    r = F.compose_frozen_shortest_path_batch(rhs, lab, off, 1, F.FST_SEM_EAGER)
    del r
print("done")
