"""GPU: a host batch call that fails after its work is in flight hands nothing still in use
back to the pools (DESIGN §3.1 post-mortems).

FSTAMD_FAULT_INJECT=<site> makes the named error branch fire after the kernels (and, for
the small batches of per-utterance calls, the download) were queued.  The next calls reuse the same pooled device
block and pinned staging buffers; had the failed call returned before its stream drained,
its kernel or its download would still be writing them, and the next results would differ
from the oracle.
"""
import numpy as np
import pytest

import libfst_amd as F
import oracle_ffi as O
from test_gpu_parity import EAGER, LAZY, bits, compare_single, csr, expected_status

pytestmark = pytest.mark.gpu


def check(got, blob, labels, offsets, sem):
    ref = O.batch_run(blob, labels, offsets, 0 if sem == LAZY else 1, 1, 8)
    exp = expected_status(ref)
    assert np.array_equal(got.status, exp)
    ok = exp == F.FST_PATH_OK
    assert np.array_equal(np.diff(got.offsets.astype(np.int64))[ok],
                          np.diff(ref.offsets.astype(np.int64))[ok])
    assert np.array_equal(got.olabels, ref.olabels)
    assert np.array_equal(bits(got.weights), bits(ref.weights))
    assert np.array_equal(bits(got.finals[ok]), bits(ref.finals[ok]))


def test_single_call_failure_drains_its_stream(monkeypatch):
    # per-utterance calls (fst_compose_frozen_shortest_path) run as small batches
    # (c_api.cpp run_small_batch: one pooled device block, pinned staging in and out); a call
    # whose branch fails after the kernels and the download were queued must drain its
    # stream before those go back to the pools
    blob = O.freeze(O.gen("ambiguous", 512, 12))
    rng = np.random.default_rng(55)
    texts = [bytes(rng.choice([1, 1, 1, 2], int(rng.integers(20, 60))).tolist()) for _ in range(8)]
    for k, t in enumerate(texts):
        monkeypatch.setenv("FSTAMD_FAULT_INJECT", "small_after_launch")
        # (the failed chain batch hands the call to the general lazy engine: same answer)
        compare_single(O.compile_string(t), blob)
        monkeypatch.delenv("FSTAMD_FAULT_INJECT")
        compare_single(O.compile_string(texts[(k + 1) % len(texts)]), blob)


@pytest.mark.parametrize("sem", [EAGER, LAZY])
def test_streamed_failure_drains_its_streams(sem, monkeypatch):
    rhs = F.Fst.bench_transducer(F.BENCH_AMBIGUOUS, 4096, 12)
    blob = O.freeze(O.gen("ambiguous", 4096, 12))
    rng = np.random.default_rng(66 + sem)
    lab2d = np.where(rng.random((40000, 64)) < 0.95, 1, 2).astype(np.uint32)
    seqs = list(lab2d)
    labels, offsets = lab2d.ravel(), np.arange(0, 40001 * 64, 64, dtype=np.uint64)
    monkeypatch.setenv("FSTAMD_FAULT_INJECT", "stream_after_pull")
    with pytest.raises(RuntimeError):
        F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem)
    monkeypatch.delenv("FSTAMD_FAULT_INJECT")
    got = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem)
    sub = np.unique(np.concatenate([rng.choice(40000, 200, replace=False), [0, 39999]]))
    sl = [seqs[i] for i in sub]
    l2, o2 = csr(sl)
    part = F.compose_frozen_shortest_path_batch(rhs, l2, o2, 1, sem)
    check(part, blob, l2, o2, sem)
    # the big call's strings agree with the checked sub-batch
    for j, i in enumerate(sub):
        assert got.status[i] == part.status[j]
        a0, a1 = int(got.offsets[i]), int(got.offsets[i + 1])
        b0, b1 = int(part.offsets[j]), int(part.offsets[j + 1])
        assert np.array_equal(got.olabels[a0:a1], part.olabels[b0:b1])
        assert np.array_equal(bits(got.weights[a0:a1]), bits(part.weights[b0:b1]))
