"""Phase profile of the general engine (kernels/eager_bfs.hpp) on a few workloads:
FSTAMD_BFS_PROF=1 python scripts/prof_bfs.py  -> "[bfs prof]" lines on stderr."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import libfst_amd as F  # noqa: E402
from libfst_amd import synthetic as SY  # noqa: E402


def run(name, fz, seqs, sem):
    lens = [len(s) for s in seqs]
    labels = np.concatenate([np.asarray(s, np.uint32) for s in seqs])
    offsets = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    F.compose_frozen_shortest_path_batch(fz, labels[: int(offsets[8])], offsets[:9], 1, sem)
    t0 = time.perf_counter()
    r = F.compose_frozen_shortest_path_batch(fz, labels, offsets, 1, sem)
    dt = time.perf_counter() - t0
    print(f"{name}: {len(seqs)} strings {dt * 1e3:.1f} ms ({len(seqs) / dt:.0f}/s), "
          f"ok {(r.status == 0).sum()}", flush=True)


amb = F.Fst.bench_transducer(F.BENCH_AMBIGUOUS, 4096, 12)
run("metric lazy 8K", amb, [[1] * 64] * 8192, F.FST_SEM_LAZY)
run("metric lazy 64K", amb, [[1] * 64] * 65536, F.FST_SEM_LAZY)
eps = F.Fst.bench_transducer(F.BENCH_EPS_DENSE, 256, 12)
rng = np.random.default_rng(0x5EED)
run("eps-dense T=256 lazy", eps, [[1] * int(L) for L in rng.integers(11, 252, 256)], F.FST_SEM_LAZY)
tag = SY.to_mutable(SY.tagger()).freeze()
texts = SY.utterances(np.random.default_rng(44), 65536)
lab, off = SY.to_labels(texts)
seqs = [lab[int(off[i]):int(off[i + 1])].tolist() for i in range(len(texts))]
run("tagger lazy 64K", tag, seqs, F.FST_SEM_LAZY)
run("tagger eager 64K", tag, seqs, F.FST_SEM_EAGER)
