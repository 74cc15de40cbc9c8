"""GPU parity on the shapes of BASELINE.json's configs, at sizes the oracle finishes in
seconds (the full sizes are measured by scripts/bench_configs.py):

  config 1  single string, eager compose (fst_compose_frozen) vs epsilon-dense rhs
  config 3  lazy 1-best, mixed lengths, epsilon-dense rhs
  config 5  LogWeight blob (weight_type 1), mixed lengths + dead strings (divergence)
"""
import numpy as np
import pytest

import libfst_amd as F
import oracle_ffi as O
from test_gpu_eager_general import chain_of, compare_compose
from test_gpu_parity import EAGER, LAZY, check, csr

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("L", [24, 96])
def test_config1_eager_compose_epsilon_dense(L):
    compare_compose(chain_of([1] * L), O.freeze(O.gen("eps_dense", 256, 12)))


def test_config3_lazy_epsilon_dense_mixed_lengths():
    blob = O.freeze(O.gen("eps_dense", 512, 12))
    rng = np.random.default_rng(0x5EED)
    seqs = [[1] * int(L) for L in rng.integers(11, 41, 24)]
    check(blob, *csr(seqs), LAZY)


@pytest.mark.parametrize("sem", [EAGER, LAZY])
def test_config5_log_weight_divergence(sem):
    f = O.gen("ambiguous", 512, 12)
    blob_log = O.freeze(f, 1)
    rhs = F.Fst.from_bytes(blob_log)
    assert rhs.weight_type == 1
    rng = np.random.default_rng(55)
    n = 3000 if sem == EAGER else 300
    lens = rng.integers(1, 65, n)
    seqs = []
    for L in lens:
        s = [1] * int(L)
        if rng.random() < 0.1:          # dead strings: label 2 has no arc in the rhs
            s[int(rng.integers(0, L))] = 2
        seqs.append(s)
    # the oracle ignores the header weight type: Log times/compare == Tropical's
    check(blob_log, *csr(seqs), sem, rhs=rhs)


# ---------------------------------------------------------------------------------------
# config 4: two-stage tagger -> verbalizer (synthetic stand-ins, libfst_amd/synthetic.py)
# ---------------------------------------------------------------------------------------

from libfst_amd import synthetic as SY  # noqa: E402
from test_gpu_parity import bits, expected_status  # noqa: E402

DEAD = 0xFFFFFFFF


def oracle_fst(spec) -> O.Fst:
    ns, start, finals, arcs = spec
    f = O.Fst()
    for s in range(ns):
        f.add_state(finals[s])
    f.start = start
    for s, al in enumerate(arcs):
        for a in al:
            f.add_arc(s, *a)
    return f


def oracle_pipeline(blobs, labels, offsets, sem):
    """print_output_string -> compile_string between stages, on the oracle."""
    num = len(offsets) - 1
    fail = np.full(num, F.FST_PATH_OK, np.int32)
    for k, blob in enumerate(blobs):
        ref = O.batch_run(blob, labels, offsets, 0 if sem == LAZY else 1, 1)
        exp = expected_status(ref)
        if k == len(blobs) - 1:
            exp = np.where(fail != F.FST_PATH_OK, fail, exp)
            return ref, exp
        seqs = []
        for i in range(num):
            nxt = [DEAD]
            if exp[i] == F.FST_PATH_OK:
                ol = [int(x) for x in ref.olabels[int(ref.offsets[i]):int(ref.offsets[i + 1])]
                      if x != 0]
                if any(x > 256 for x in ol):
                    if fail[i] == F.FST_PATH_OK:
                        fail[i] = F.FST_PATH_UNSUPPORTED
                else:
                    nxt = ol
            elif fail[i] == F.FST_PATH_OK:
                fail[i] = exp[i]
            seqs.append(nxt)
        labels, offsets = csr(seqs)


@pytest.mark.parametrize("sem", [LAZY, EAGER])
def test_config4_tagger_verbalizer_pipeline(sem):
    tag, verb = SY.tagger(), SY.verbalizer()
    blobs = [O.freeze(oracle_fst(tag)), O.freeze(oracle_fst(verb))]
    rng = np.random.default_rng(4)
    texts = SY.utterances(rng, 300 if sem == LAZY else 1000) + ["", "a", "7", "##", "call 911"]
    labels, offsets = SY.to_labels(texts)
    stages = [F.Fst.from_bytes(b) for b in blobs]
    got = F.pipeline_batch(stages, labels, offsets, 1, sem)
    ref, exp = oracle_pipeline(blobs, labels, offsets, sem)
    assert np.array_equal(got.status, exp)
    ok = exp == F.FST_PATH_OK
    assert ok.sum() > 0.9 * len(texts) - 5
    for i in np.nonzero(ok)[0]:
        a0, a1 = int(got.offsets[i]), int(got.offsets[i + 1])
        b0, b1 = int(ref.offsets[i]), int(ref.offsets[i + 1])
        assert np.array_equal(got.ilabels[a0:a1], ref.ilabels[b0:b1]), i
        assert np.array_equal(got.olabels[a0:a1], ref.olabels[b0:b1]), i
        assert np.array_equal(bits(got.weights[a0:a1]), bits(ref.weights[b0:b1])), i
    assert np.array_equal(bits(got.finals[ok]), bits(ref.finals[ok]))
    # a readable spot check: "7" -> tagger picks "#h" (0.5 < 1.0) -> verbalizer "seven"
    i = texts.index("7")
    out = bytes(int(x) - 1 for x in got.olabels[int(got.offsets[i]):int(got.offsets[i + 1])] if x)
    assert out == b"seven"
