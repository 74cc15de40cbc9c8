"""Debug helper for the band replay (kernels/lazy_band.hpp): the metric-shape case of
tests/test_gpu_lazy_rounds.py and a few config-3 strings, with FSTAMD_LAZY_ENGINE=dense
(band first), the route log and FSTAMD_BFS_PROF (per-wave overflow / INTERNAL sites).
usage: python scripts/debug_band.py"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
os.environ.setdefault("FSTAMD_LAZY_ENGINE", "dense")
os.environ.setdefault("FSTAMD_BFS_PROF", "1")
os.environ.setdefault("FSTAMD_ROUTE_LOG", "1")

import libfst_amd as F  # noqa: E402
import oracle_ffi as O  # noqa: E402
from test_gpu_parity import csr, expected_status, load_blob  # noqa: E402

cases = [("ambiguous", 4096, [[1] * 64] * 6 + [[1] * L for L in (0, 1, 2, 17, 63, 128)] + [[1, 2, 1]]),
         ("eps_dense", 1024, [[1] * L for L in (87, 44, 176, 249)]),
         ("eps_dense", 256, [[1] * L for L in (11, 24, 40)])]
for kind, T, seqs in cases:
    blob = O.freeze(O.gen(kind, T, 12))
    labels, offsets = csr(seqs)
    got = F.compose_frozen_shortest_path_batch(load_blob(blob), labels, offsets, 1, F.FST_SEM_LAZY)
    ref = O.batch_run(blob, labels, offsets, 0, 1, 8)
    exp = expected_status(ref)
    bad = np.nonzero(got.status != exp)[0]
    print(kind, T, "mismatch", len(bad), [(int(i), len(seqs[i]), int(got.status[i])) for i in bad],
          flush=True)
