"""Debug helper for the dense lazy replay (kernels/lazy_dense.hpp): runs the random
tie-heavy case of tests/test_gpu_lazy_rounds.py with FSTAMD_LAZY_ENGINE=dense and prints
per-string status against the oracle (INTERNAL strings: path_len = pops, path_off = site).
usage: FSTAMD_WATCHDOG_MS=3000 python scripts/debug_dense.py [seed ...]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
os.environ.setdefault("FSTAMD_LAZY_ENGINE", "dense")

import libfst_amd as F  # noqa: E402
import oracle_ffi as O  # noqa: E402
from test_gpu_parity import csr, expected_status, load_blob, random_rhs  # noqa: E402

for seed in [int(x) for x in sys.argv[1:]] or [0]:
    rng = np.random.default_rng(31000 + seed)
    f = random_rhs(rng, int(rng.integers(2, 30)), int(rng.integers(4, 120)), 3,
                   eps=seed % 4 != 3, wmax=2, frac=seed % 3 == 0)
    blob = O.freeze(f)
    seqs = [[int(x) for x in rng.integers(0, 4, int(rng.integers(0, 10)))] for _ in range(48)]
    if os.environ.get("NO_LABEL0"):
        seqs = [[x if x else 1 for x in q] for q in seqs]
    if os.environ.get("ONE"):
        seqs = seqs[:1]
    if os.environ.get("EACH"):  # one call per string: the first hang names its string
        rhs = load_blob(blob)
        for i, q in enumerate(seqs):
            print("  call", i, q, flush=True)
            lab1, off1 = csr([q])
            g1 = F.compose_frozen_shortest_path_batch(rhs, lab1, off1, 1, F.FST_SEM_LAZY)
            print("   ->", g1.status[0], flush=True)
    labels, offsets = csr(seqs)
    rhs = load_blob(blob)
    got = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, F.FST_SEM_LAZY)
    ref = O.batch_run(blob, labels, offsets, 0, 1)
    exp = expected_status(ref)
    bad = np.nonzero(got.status != exp)[0]
    print("seed", seed, "engine", F.last_launch_stats().engine, "mismatch", len(bad), flush=True)
    for i in bad[:8]:
        print("  string", i, seqs[i], "got", got.status[i], "exp", exp[i], flush=True)
