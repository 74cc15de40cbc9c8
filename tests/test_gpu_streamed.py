"""The streamed host batch (c_api.cpp run_streamed): a batch of >= 4 M labels and >= 32 K
strings on an rhs whose first tier is a pull tier runs as parts of growing size over two
engines, the pull tier alone per part (its statuses written twice by the kernel, its paths
copied into the pinned result by the kernel), then the later tiers once over the strings it
handed on, then the fix-up downloads and the in-place compaction of strings without a path.

The batch mixes what every stage must handle: metric strings (the pull tier), strings with
a label-0 arc (the pull tier hands them on as UNSUPPORTED: general engine), strings longer
than the pull window allows (OVERFLOW: the push tiers), labels without rhs arcs (EMPTY:
compacted out of the CSR result) and empty strings.  A sample of strings across every part
is bit-compared with the oracle, and the whole result with the non-streamed entry
(FSTAMD_STREAM=0), for both semantics and several part cuts.
"""
import numpy as np
import pytest

import libfst_amd as F
import oracle_ffi as O
from test_gpu_parity import EAGER, LAZY, bits, expected_status

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def metric():
    return F.Fst.bench_transducer(F.BENCH_AMBIGUOUS, 4096, 12), O.freeze(O.gen("ambiguous", 4096, 12))


def mixed_batch(rng, num=40000):
    lens = rng.integers(80, 130, num)
    seqs = []
    for i, L in enumerate(lens):
        q = np.where(rng.random(L) < 0.9, 1, 2).astype(np.uint32)
        kind = i % 97
        if kind == 5:
            q[int(rng.integers(0, L))] = 0           # label 0: UNSUPPORTED for the pull tier
        elif kind == 11:
            q[int(rng.integers(0, L))] = 3           # no rhs arc: EMPTY
        elif kind == 17:
            q = q[:0]                                # the empty string
        elif kind == 23:
            q = np.ones(900, np.uint32)              # long: beyond the pull tier's window
        seqs.append(q)
    offsets = np.concatenate([[0], np.cumsum([len(q) for q in seqs])]).astype(np.uint64)
    return np.concatenate(seqs).astype(np.uint32), offsets


def compare_sample(got, blob, labels, offsets, sem, idx):
    sub = [labels[int(offsets[i]):int(offsets[i + 1])] for i in idx]
    so = np.concatenate([[0], np.cumsum([len(q) for q in sub])]).astype(np.uint64)
    sl = np.concatenate(sub).astype(np.uint32) if len(sub) else np.zeros(0, np.uint32)
    ref = O.batch_run(blob, sl, so, 0 if sem == LAZY else 1, 1, 8)
    exp = expected_status(ref)
    assert np.array_equal(got.status[idx], exp)
    for j, i in enumerate(idx):
        if exp[j] != F.FST_PATH_OK:
            assert got.offsets[i + 1] == got.offsets[i]  # compacted out
            continue
        a0, a1 = int(got.offsets[i]), int(got.offsets[i + 1])
        b0, b1 = int(ref.offsets[j]), int(ref.offsets[j + 1])
        assert np.array_equal(got.ilabels[a0:a1], ref.ilabels[b0:b1]), i
        assert np.array_equal(got.olabels[a0:a1], ref.olabels[b0:b1]), i
        assert np.array_equal(bits(got.weights[a0:a1]), bits(ref.weights[b0:b1])), i
        assert bits(got.finals[i]) == bits(ref.finals[j]), i


@pytest.mark.parametrize("sem", [EAGER, LAZY])
@pytest.mark.parametrize("cuts", ["", "8,45,230"])
def test_streamed_batch(metric, sem, cuts, monkeypatch):
    rhs, blob = metric
    rng = np.random.default_rng(20260 + sem)
    labels, offsets = mixed_batch(rng)
    assert offsets[-1] >= (1 << 22)
    if cuts:
        monkeypatch.setenv("FSTAMD_STREAM_CUTS", cuts)
    got = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem)
    num = len(offsets) - 1
    # every kind of string, in every part (the parts cut the batch in order)
    special = [i for i in range(num) if i % 97 in (5, 11, 17, 23)]
    idx = np.unique(np.concatenate([rng.choice(num, 150, replace=False),
                                    np.asarray(special[::14]), [0, num - 1]])).astype(np.int64)
    compare_sample(got, blob, labels, offsets, sem, idx)
    # the whole result against the non-streamed entry
    monkeypatch.setenv("FSTAMD_STREAM", "0")
    ref = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem)
    assert np.array_equal(got.status, ref.status)
    assert np.array_equal(got.offsets, ref.offsets)
    assert np.array_equal(got.ilabels, ref.ilabels)
    assert np.array_equal(got.olabels, ref.olabels)
    assert np.array_equal(bits(got.weights), bits(ref.weights))
    assert np.array_equal(bits(got.finals), bits(ref.finals))
