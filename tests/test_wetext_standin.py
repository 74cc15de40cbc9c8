"""The WeText-scale stand-in generator (libfst_amd/wetext_standin.py), CPU only: its blob
is Fst.fromMutable's byte for byte (the oracle's freeze of the same arcs), and it has the
structure the config-4 GPU tests rely on (size, byte labels, scattered ids, epsilon
outputs, multi-label states)."""
import numpy as np

import libfst_amd as F
import oracle_ffi as O
from libfst_amd import wetext_standin as W


def as_oracle(g):
    ns, start, fin, arcs = g.lists()
    return O.Fst(start=start, finals=fin, arcs=[list(a) for a in arcs])


def test_freeze_blob_is_from_mutable():
    for g in (W.tagger(n_chars=300, n_words=500), W.verbalizer(n_chars=300)):
        blob = W.freeze_blob(g)
        assert blob == O.freeze(as_oracle(g))
        # and the library accepts it unchanged
        f = F.Fst.from_bytes(blob)
        assert f.num_states == g.num_states and f.start == g.start


def test_full_size_structure():
    g = W.tagger()
    assert g.num_states >= 100_000 and len(g.src) >= 1_000_000
    assert int(g.il.max()) <= 256 and int(g.ol.max()) <= 256       # byte + 1 labels
    assert (g.il == 0).sum() > 100_000                              # epsilon-input outputs
    deg = np.bincount(g.src, minlength=g.num_states)
    assert deg.max() >= 16 and (deg >= 8).sum() > 10_000            # multi-label states
    # scattered ids: arcs jump far (no band a P / LP window could hold)
    jump = np.abs(g.dst.astype(np.int64) - g.src.astype(np.int64))
    assert np.median(jump) > 10_000
    labels, offsets = W.utterances(np.random.default_rng(0), 200)
    assert labels.max() <= 256 and len(offsets) == 201


def test_small_pipeline_matches_oracle_shapes():
    # the oracle's two stages on a small stand-in: every utterance gets a path
    tag, verb = W.tagger(n_chars=300, n_words=500), W.verbalizer(n_chars=300)
    tb, vb = W.freeze_blob(tag), W.freeze_blob(verb)
    labels, offsets = W.utterances(np.random.default_rng(2), 50, n_chars=300, n_words=500)
    r = O.batch_run(tb, labels, offsets, 0, 1)
    assert (r.status == 0).all() and (r.empty == 0).all()
