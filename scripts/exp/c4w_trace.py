"""The WeText-scale tagger stage (lazy, then eager) three times each, for kernel traces."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import libfst_amd as F
from libfst_amd import wetext_standin as W

torch.cuda.set_device(0)
tag = F.Fst.from_bytes(W.freeze_blob(W.tagger()))
labels, offsets = W.utterances(np.random.default_rng(44), 65536)
for sem in (F.FST_SEM_LAZY, F.FST_SEM_EAGER):
    for _ in range(3):
        r = F.compose_frozen_shortest_path_batch(tag, labels, offsets, 1, sem)
        del r
print("done")
