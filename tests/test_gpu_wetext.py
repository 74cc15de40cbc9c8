"""Config 4 at WeText scale (libfst_amd/wetext_standin.py: 0.43 M-state / 1.03 M-arc
tagger, UTF-8 byte labels, scattered state ids, epsilon-output chains, multi-label states;
a markup-removing verbalizer), bit-exact against the oracle on the GPU:

* the tagger stage alone, both semantics (lazy: the LDS replay at 128 / 256 tuples, then the
  dense replay for what outgrows it; eager: the general engine's LDS tiny tiers, then HBM);
* the two-stage pipeline, both semantics (device projection between the stages);
* the same pipeline sharded (fake multi-GPU).
The real WeTextProcessing FSTs are unavailable offline: parity on them stays unpinned.
"""
import numpy as np
import pytest

import libfst_amd as F
import oracle_ffi as O
from libfst_amd import wetext_standin as W
from test_gpu_configs import DEAD
from test_gpu_parity import EAGER, LAZY, bits, check, expected_status

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def standin():
    tb, vb = W.freeze_blob(W.tagger()), W.freeze_blob(W.verbalizer())
    return tb, vb, F.Fst.from_bytes(tb), F.Fst.from_bytes(vb)


@pytest.mark.parametrize("sem", [LAZY, EAGER])
def test_tagger_stage(standin, sem):
    tb, _, tag, _ = standin
    labels, offsets = W.utterances(np.random.default_rng(31 + sem), 800)
    got, ref = check(tb, labels, offsets, sem, rhs=tag)
    assert (got.status == F.FST_PATH_OK).all()


@pytest.mark.parametrize("sem", [LAZY, EAGER])
@pytest.mark.parametrize("start", ["1", "2"])
def test_tagger_stage_tiny_start(standin, sem, start, monkeypatch):
    # the LDS tiny sizes start at 128 tuples, or at 256 on an rhs whose 128-tuple pass
    # handed on over a third of a batch (learnt per rhs; forced here both ways)
    monkeypatch.setenv("FSTAMD_LAZY_TINY_START", start)
    monkeypatch.setenv("FSTAMD_BFS_TINY_START", start)
    tb, _, _, _ = standin
    labels, offsets = W.utterances(np.random.default_rng(57 + sem), 1200)
    got, ref = check(tb, labels, offsets, sem)
    assert (got.status == F.FST_PATH_OK).all()


@pytest.mark.parametrize("ctiny", ["0", "1"])
@pytest.mark.parametrize("start", ["1", "2"])
def test_tagger_stage_eager_tables(standin, ctiny, start, monkeypatch):
    # eager, both LDS table layouts (the compact one of kernels/eager_tiny.hpp, the default,
    # and eager_bfs.hpp's kTiny ones), from either size: bit-exact against the oracle
    monkeypatch.setenv("FSTAMD_EAGER_CTINY", ctiny)
    monkeypatch.setenv("FSTAMD_BFS_TINY_START", start)
    tb, _, _, _ = standin
    labels, offsets = W.utterances(np.random.default_rng(91 + int(start)), 1000)
    got, ref = check(tb, labels, offsets, EAGER)
    assert (got.status == F.FST_PATH_OK).all()


def oracle_pipeline(blobs, labels, offsets, sem):
    num = len(offsets) - 1
    fail = np.full(num, F.FST_PATH_OK, np.int32)
    for k, blob in enumerate(blobs):
        ref = O.batch_run(blob, labels, offsets, 0 if sem == LAZY else 1, 1, 8)
        exp = expected_status(ref)
        if k == len(blobs) - 1:
            return ref, np.where(fail != F.FST_PATH_OK, fail, exp)
        seqs = []
        for i in range(num):
            nxt = [DEAD]
            if exp[i] == F.FST_PATH_OK:
                ol = [int(x) for x in ref.olabels[int(ref.offsets[i]):int(ref.offsets[i + 1])] if x]
                if any(x > 256 for x in ol):
                    fail[i] = F.FST_PATH_UNSUPPORTED if fail[i] == F.FST_PATH_OK else fail[i]
                else:
                    nxt = ol
            elif fail[i] == F.FST_PATH_OK:
                fail[i] = exp[i]
            seqs.append(nxt)
        lens = [len(s) for s in seqs]
        offsets = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        labels = np.concatenate([np.asarray(s, np.uint32) for s in seqs])


@pytest.mark.parametrize("sem", [LAZY, EAGER])
@pytest.mark.parametrize("shards", [0, 3])
def test_two_stage_pipeline(standin, sem, shards):
    tb, vb, tag, verb = standin
    labels, offsets = W.utterances(np.random.default_rng(41 + sem), 600)
    got = F.pipeline_batch([tag, verb], labels, offsets, 1, sem,
                           devices=[0] if shards else None, shards=shards)
    ref, exp = oracle_pipeline([tb, vb], labels, offsets, sem)
    assert np.array_equal(got.status, exp)
    ok = exp == F.FST_PATH_OK
    assert ok.sum() > 0.95 * len(ok)
    assert np.array_equal(np.diff(got.offsets)[ok], np.diff(ref.offsets)[ok])
    for i in np.nonzero(ok)[0]:
        a0, a1 = int(got.offsets[i]), int(got.offsets[i + 1])
        b0, b1 = int(ref.offsets[i]), int(ref.offsets[i + 1])
        assert np.array_equal(got.ilabels[a0:a1], ref.ilabels[b0:b1]), i
        assert np.array_equal(got.olabels[a0:a1], ref.olabels[b0:b1]), i
        assert np.array_equal(bits(got.weights[a0:a1]), bits(ref.weights[b0:b1])), i
    assert np.array_equal(bits(got.finals[ok]), bits(ref.finals[ok]))
    # the markup is gone after the verbalizer: only UTF-8 text remains
    i = int(np.nonzero(ok)[0][0])
    out = bytes(int(x) - 1 for x in got.olabels[int(got.offsets[i]):int(got.offsets[i + 1])] if x)
    out.decode("utf-8")
    assert b"w{" not in out and b"n{" not in out


@pytest.mark.parametrize("start", ["", "1", "2"])
def test_lds_replay_generation_wrap(standin, start, monkeypatch):
    # lazy_tiny_kernel's hash generation starts near its wrap (65536) and 8 waves take the
    # batch, so every wave clears its table mid-launch and reuses it; the direct 1024-tuple
    # size (no start forced) and the 128 / 256 sizes each
    monkeypatch.setenv("FSTAMD_TINY_GEN0", "65500")
    monkeypatch.setenv("FSTAMD_TINY_WAVES", "8")
    if start:
        monkeypatch.setenv("FSTAMD_LAZY_TINY_START", start)
    tb, _, tag, _ = standin
    labels, offsets = W.utterances(np.random.default_rng(77), 700)
    got, ref = check(tb, labels, offsets, LAZY, rhs=tag)
    assert (got.status == F.FST_PATH_OK).all()
