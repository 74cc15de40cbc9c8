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


def mixed_batch(rng, num=40000, long=True):
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
        elif kind == 23 and long:
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


def handed_on_batch(rng, num=48000, every=5):
    """Metric strings with a label-0 arc in every `every`-th one (short, so the general
    engine finishes them quickly): > 4096 strings handed on by the pull tier."""
    seqs = []
    for i in range(num):
        if i % every == 0:
            L = int(rng.integers(8, 24))
            q = np.ones(L, np.uint32)
            q[int(rng.integers(0, L))] = 0
        else:
            L = int(rng.integers(100, 130))
            q = np.where(rng.random(L) < 0.9, 1, 2).astype(np.uint32)
        seqs.append(q)
    offsets = np.concatenate([[0], np.cumsum([len(q) for q in seqs])]).astype(np.uint64)
    return np.concatenate(seqs).astype(np.uint32), offsets


def same_result(a, b):
    assert np.array_equal(a.status, b.status)
    assert np.array_equal(a.offsets, b.offsets)
    assert np.array_equal(a.ilabels, b.ilabels)
    assert np.array_equal(a.olabels, b.olabels)
    assert np.array_equal(bits(a.weights), bits(b.weights))
    assert np.array_equal(bits(a.finals), bits(b.finals))


@pytest.mark.parametrize("sem", [EAGER, LAZY])
def test_streamed_bulk_fixup(metric, sem, monkeypatch):
    # more than 4096 strings handed on: the fix-up copies the whole device arena over the
    # paths the pull tier already wrote into the result
    rhs, blob = metric
    rng = np.random.default_rng(777 + sem)
    labels, offsets = handed_on_batch(rng)
    assert offsets[-1] >= (1 << 22)
    monkeypatch.setenv("FSTAMD_SHARD_LOG", "1")
    got = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem)
    num = len(offsets) - 1
    idx = np.unique(np.concatenate([rng.choice(num, 120, replace=False),
                                    np.arange(0, num, 997), [num - 1]])).astype(np.int64)
    compare_sample(got, blob, labels, offsets, sem, idx)
    monkeypatch.setenv("FSTAMD_STREAM", "0")
    same_result(got, F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem))
    # and the per-string fix-up on the same batch gives the same bytes
    monkeypatch.delenv("FSTAMD_STREAM")
    monkeypatch.setenv("FSTAMD_STREAM_FIX_FEW", "1000000")
    same_result(got, F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem))


@pytest.mark.parametrize("sem", [EAGER, LAZY])
def test_streamed_label_staging_modes(metric, sem, monkeypatch):
    # FSTAMD_STREAM_STAGE=1: the labels copied into the result's pinned ilabels chunk by
    # chunk and uploaded from there (one host-DRAM pass) -- the same result as the
    # runtime-staged upload
    rhs, blob = metric
    rng = np.random.default_rng(31337 + sem)
    labels, offsets = mixed_batch(rng, long=False)  # (test_streamed_batch has the long ones)
    monkeypatch.setenv("FSTAMD_STREAM_STAGE", "0")
    a = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem)
    monkeypatch.setenv("FSTAMD_STREAM_STAGE", "1")
    b = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem)
    same_result(a, b)
    num = len(offsets) - 1
    compare_sample(b, blob, labels, offsets, sem,
                   np.unique(np.concatenate([rng.choice(num, 80, replace=False), [0, num - 1]])))


@pytest.mark.parametrize("sem", [EAGER, LAZY])
@pytest.mark.parametrize("shards", [2, 3])
def test_streamed_shards_on_one_gpu(metric, sem, shards, monkeypatch, capfd):
    # FST_BATCH_DEVICES through the streamed entry: each shard streams into its own slice
    # of the one pinned result (fixed slots), strings without a path compacted out after
    # the last shard; 2 and 3 logical shards on device 0 equal the one-shard run and the
    # oracle bit for bit
    rhs, blob = metric
    rng = np.random.default_rng(4040 + 10 * shards + sem)
    labels, offsets = mixed_batch(rng, num=60000, long=False)
    one = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem)
    capfd.readouterr()
    monkeypatch.setenv("FSTAMD_SHARD_LOG", "1")
    many = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem, devices=[0],
                                                shards=shards)
    err = capfd.readouterr().err
    plan = [ln.split() for ln in err.splitlines() if ln.startswith("[libfst_amd shard]")]
    assert len(plan) == shards and all(p[-1] == "streamed" for p in plan), err[-2000:]
    spans = [tuple(int(x) for x in p[6].split("..")) for p in plan]
    num = len(offsets) - 1
    assert spans[0][0] == 0 and spans[-1][1] == num
    assert all(spans[j][1] == spans[j + 1][0] for j in range(shards - 1))
    costs = [float(p[8]) for p in plan]
    assert max(costs) / min(costs) < 1.2
    same_result(many, one)
    # strings on both sides of every shard boundary, against the oracle
    edges = np.asarray([s for sp in spans for s in (sp[0], sp[1] - 1)])
    idx = np.unique(np.concatenate([edges, rng.choice(num, 40, replace=False)])).astype(np.int64)
    compare_sample(many, blob, labels, offsets, sem, idx)
