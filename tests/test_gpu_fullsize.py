"""GPU parity at the full sizes of BASELINE.json configs 1 and 3 (bit-exact vs the oracle).

config 1  compose_frozen_epsilon_dense, len=96, transducer-len=4096, branches=12
          (bench/optimize-bench.zig:219-248, :357-361): the whole fst_compose_frozen lattice
          (781,313 states, 10,058,572 arcs) state by state and arc by arc, plus the eager
          1-best of the same string through the batch entry.
config 3  compose_frozen_lazy_shortest_path_epsilon_dense (:398-401), its hard corners:
          - (L=251, T=512), where the survey found eager != lazy (equal total, different
            epsilon placement and olabels): both semantics on the GPU
            equal their oracle, and differ from each other exactly as the oracle's do;
          - a mixed-length batch, L uniform in [11, 251] (seed 0x5EED), at T=4096;
          - strings at the full T=65,536 with L in {11, 87} (live oracle), and 8 strings of
            the config's lengths up to L=251 against the oracle's fixture
            (tests/golden/config3_T65536.npz, tests/golden/make_config3_golden.py).
The oracle runs on the host (threads for the larger batches); the GPU path goes through the
C ABI (fst_compose_frozen, fst_compose_frozen_shortest_path_batch).
"""
import numpy as np
import pytest

import libfst_amd as F
import oracle_ffi as O
from test_gpu_eager_general import chain_of
from test_gpu_parity import EAGER, LAZY, bits, csr, expected_status, load_blob, to_product

pytestmark = pytest.mark.gpu


def check_batch(blob, seqs, sem, rhs=None, threads=8):
    """Like test_gpu_parity.check, with a threaded oracle (large lattices)."""
    labels, offsets = csr(seqs)
    rhs = rhs or load_blob(blob)
    got = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem)
    ref = O.batch_run(blob, labels, offsets, 0 if sem == LAZY else 1, 1, threads)
    exp = expected_status(ref)
    assert np.array_equal(got.status, exp), (got.status, exp)
    ok = exp == F.FST_PATH_OK
    assert np.array_equal(got.offsets, ref.offsets) or np.array_equal(
        np.diff(got.offsets)[ok], np.diff(ref.offsets)[ok])
    for i in np.nonzero(ok)[0]:
        a0, a1 = int(got.offsets[i]), int(got.offsets[i + 1])
        b0, b1 = int(ref.offsets[i]), int(ref.offsets[i + 1])
        assert np.array_equal(got.ilabels[a0:a1], ref.ilabels[b0:b1]), i
        assert np.array_equal(got.olabels[a0:a1], ref.olabels[b0:b1]), i
        assert np.array_equal(bits(got.weights[a0:a1]), bits(ref.weights[b0:b1])), i
    assert np.array_equal(bits(got.finals[ok]), bits(ref.finals[ok]))
    return got, ref


def path_of(res, i):
    a, b = int(res.offsets[i]), int(res.offsets[i + 1])
    return (res.ilabels[a:b].tolist(), res.olabels[a:b].tolist(), bits(res.weights[a:b]).tolist())


# ---------------------------------------------------------------------------------------
# config 1 at full size
# ---------------------------------------------------------------------------------------

@pytest.fixture(scope="module")
def eps4096():
    blob = O.freeze(O.gen("eps_dense", 4096, 12))
    return blob, load_blob(blob)


def test_config1_full_compose_lattice(eps4096):
    blob, rhs = eps4096
    lhs = chain_of([1] * 96)
    rc, ref = O.compose_csr(lhs, blob)
    assert rc == O.OR_OK
    assert len(ref.finals) == 781_313 and len(ref.arcs) == 10_058_572
    got = F.compose_frozen(to_product(lhs), rhs)
    assert got is not None
    start, off, arcs, fin = got.to_arrays()
    assert start == ref.start == 0
    assert np.array_equal(off, ref.off)
    assert np.array_equal(bits(fin), bits(ref.finals))
    for f in ("il", "ol", "next"):
        assert np.array_equal(arcs[f], ref.arcs[f]), f
    assert np.array_equal(bits(arcs["w"]), bits(ref.arcs["w"]))


@pytest.mark.parametrize("sem", [EAGER, LAZY])
def test_config1_full_one_best(eps4096, sem):
    blob, rhs = eps4096
    got, ref = check_batch(blob, [[1] * 96], sem, rhs=rhs)
    assert got.status[0] == F.FST_PATH_OK
    # 96 arcs, olabels 1..96, weights 0, final 0 (both semantics agree)
    assert got.olabels.tolist() == list(range(1, 97))


# ---------------------------------------------------------------------------------------
# config 3 corners
# ---------------------------------------------------------------------------------------

def test_config3_eager_lazy_divergence_L251_T512():
    blob = O.freeze(O.gen("eps_dense", 512, 12))
    rhs = load_blob(blob)
    seqs = [[1] * 251]
    ge, re_ = check_batch(blob, seqs, EAGER, rhs=rhs)
    gl, rl = check_batch(blob, seqs, LAZY, rhs=rhs)
    # the oracle's two semantics differ here (equal totals); the GPU reproduces both
    assert path_of(re_, 0) != path_of(rl, 0)
    assert bits(re_.finals).tolist() == bits(rl.finals).tolist()
    assert path_of(ge, 0) == path_of(re_, 0) and path_of(gl, 0) == path_of(rl, 0)
    tot = lambda r: float(np.sum(r.weights) + r.finals[0])  # noqa: E731
    assert tot(re_) == tot(rl)


def test_config3_mixed_lengths_T4096_lazy(eps4096):
    blob, rhs = eps4096
    rng = np.random.default_rng(0x5EED)
    lens = [int(x) for x in rng.integers(11, 252, 12)] + [11, 251]
    got, _ = check_batch(blob, [[1] * L for L in lens], LAZY, rhs=rhs)
    assert np.all(got.status == F.FST_PATH_OK)


def test_config3_mixed_lengths_T4096_eager(eps4096):
    blob, rhs = eps4096
    rng = np.random.default_rng(0x5EED + 1)
    lens = [int(x) for x in rng.integers(11, 252, 5)] + [251]
    got, _ = check_batch(blob, [[1] * L for L in lens], EAGER, rhs=rhs)
    assert np.all(got.status == F.FST_PATH_OK)


def test_config3_full_T65536():
    blob = O.freeze(O.gen("eps_dense", 65536, 12))
    rhs = load_blob(blob)
    got, _ = check_batch(blob, [[1] * 11, [1] * 87, [1] * 11], LAZY, rhs=rhs, threads=3)
    assert np.all(got.status == F.FST_PATH_OK)


def test_config3_full_T65536_golden():
    # config 3's full rhs against strings of its length distribution, L up to 251 (33 M
    # product tuples in the reference's replay), bit-exact vs the oracle's fixture; the
    # GPU takes the band replay's exact early exit, the oracle replays
    # the whole product as the reference does
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "config3_T65536.npz"),
                allow_pickle=False)
    rhs = F.Fst.bench_transducer(1, int(z["T"]), int(z["B"]))
    lens = [int(x) for x in z["lengths"]]
    labels, offsets = csr([[1] * L for L in lens])
    got = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, LAZY)
    assert np.all(z["status"] == 0) and np.all(got.status == F.FST_PATH_OK), got.status
    assert np.array_equal(got.offsets, z["offsets"])
    assert np.array_equal(got.ilabels, z["ilabels"])
    assert np.array_equal(got.olabels, z["olabels"])
    assert np.array_equal(bits(got.weights), bits(z["weights"]))
    assert np.array_equal(bits(got.finals), bits(z["finals"]))
