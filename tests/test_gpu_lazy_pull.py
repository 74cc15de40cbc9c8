"""GPU parity of the lazy pull tier (kernels/lazy_pull.hpp), composeShortestPath semantics.

FSTAMD_LAZY_ONLY_FIRST=1 stops the lazy chain after the pull tier, so the strings it hands
on (OVERFLOW: an uncertified tuple, a hub state, a window wider than 320 states) stay
visible; everything it returns as OK / EMPTY must be bit-exact against the oracle's
sequential replay of compose-shortest-path.zig:26-401.  The model of the tier,
tests/lazy_pull_model.py, is checked against the same oracle on the CPU
(tests/test_lazy_pull_model.py); these tests check the kernel against the oracle and, on
the metric shape, that the tier takes every string by itself.
"""
import math

import numpy as np
import pytest

import libfst_amd as F
import oracle_ffi as O
from test_gpu_parity import bits, check, csr, expected_status, load_blob, random_rhs

pytestmark = pytest.mark.gpu

LAZY = F.FST_SEM_LAZY


@pytest.fixture(params=["direct", "indirect", "f64"])
def only_lp(request, monkeypatch):
    # f64: the f64-cell kernel (FSTAMD_LP_F64) on the direct layout -- 16-bit sort entries,
    # a 64-bin counting sort and the split sort on f64 bit patterns (round 6)
    monkeypatch.setenv("FSTAMD_LAZY_ONLY_FIRST", "1")
    monkeypatch.delenv("FSTAMD_LAZY_ENGINE", raising=False)
    if request.param == "indirect":
        monkeypatch.setenv("FSTAMD_PULL_INDIRECT", "1")
    else:
        monkeypatch.delenv("FSTAMD_PULL_INDIRECT", raising=False)
    if request.param == "f64":
        monkeypatch.setenv("FSTAMD_LP_F64", "1")
    else:
        monkeypatch.delenv("FSTAMD_LP_F64", raising=False)


def run_lp(blob, seqs, expect_all=True):
    labels, offsets = csr(seqs)
    rhs = load_blob(blob)
    got = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, LAZY)
    ref = O.batch_run(blob, labels, offsets, 0, 1)
    exp = expected_status(ref)
    took = (got.status == F.FST_PATH_OK) | (got.status == F.FST_PATH_EMPTY)
    if expect_all:
        assert took.all(), np.unique(got.status, return_counts=True)
    assert np.all((got.status[~took] == F.FST_PATH_OVERFLOW) |
                  (got.status[~took] == F.FST_PATH_UNSUPPORTED))
    assert np.array_equal(got.status[took], exp[took]), (
        np.nonzero(got.status[took] != exp[took])[0][:8])
    for i in np.nonzero(took & (exp == F.FST_PATH_OK))[0]:
        a0, a1 = int(got.offsets[i]), int(got.offsets[i + 1])
        b0, b1 = int(ref.offsets[i]), int(ref.offsets[i + 1])
        assert np.array_equal(got.ilabels[a0:a1], ref.ilabels[b0:b1]), i
        assert np.array_equal(got.olabels[a0:a1], ref.olabels[b0:b1]), (i, seqs[i])
        assert np.array_equal(bits(got.weights[a0:a1]), bits(ref.weights[b0:b1])), i
        assert bits(got.finals[i:i + 1])[0] == bits(ref.finals[i:i + 1])[0], i
    return got, took


def test_metric_shape_entirely_in_lazy_pull(only_lp):
    blob = O.freeze(O.gen("ambiguous", 4096, 12))
    seqs = [[1] * 64] * 24 + [[1] * L for L in (0, 1, 2, 5, 33, 63, 65, 79)]
    seqs += [[1] * 30 + [2] + [1] * 10]
    got, _ = run_lp(blob, seqs)
    assert list(got.olabels[:64]) == [1] * 64


@pytest.mark.parametrize("T", [64, 256])
def test_metric_shape_small_transducers(only_lp, T):
    # the chain reaches the transducer's last state (an in-arc group of 11 arcs: a hub
    # for blocks of 5, handed on) -- exact on what the tier keeps
    blob = O.freeze(O.gen("ambiguous", T, 12))
    seqs = [[1] * L for L in range(0, 70, 3)]
    run_lp(blob, seqs, expect_all=False)


@pytest.mark.parametrize("seed", range(8))
def test_random_tie_heavy_graphs(only_lp, seed):
    # integer weights in {0, 1, 2} (or all 0): many equal distances, 0-weight ties and
    # joiner candidates; the tier certifies most strings and hands on the rest
    rng = np.random.default_rng(7700 + seed)
    ns = int(rng.integers(2, 60))
    f = random_rhs(rng, ns, int(rng.integers(ns, 5 * ns)), 3, eps=False,
                   wmax=0 if seed % 4 == 0 else 2, frac=seed % 4 == 3)
    blob = O.freeze(f)
    seqs = [[int(x) for x in rng.integers(1, 4, int(rng.integers(0, 16)))] for _ in range(128)]
    got, took = run_lp(blob, seqs, expect_all=False)
    assert took.mean() > 0.5, took.mean()


@pytest.mark.parametrize("seed", range(4))
def test_full_chain_random(seed, monkeypatch):
    # the whole lazy chain (pull, then the rounds engines for its fallbacks): exact
    monkeypatch.delenv("FSTAMD_LAZY_ONLY_FIRST", raising=False)
    monkeypatch.delenv("FSTAMD_LAZY_ENGINE", raising=False)
    rng = np.random.default_rng(8800 + seed)
    ns = int(rng.integers(2, 200))
    f = random_rhs(rng, ns, int(rng.integers(ns, 4 * ns)), 3, eps=False, wmax=2)
    blob = O.freeze(f)
    seqs = [[int(x) for x in rng.integers(1, 4, int(rng.integers(0, 24)))] for _ in range(96)]
    check(blob, *csr(seqs), LAZY)


def test_fromBytes_blob_out_of_olabel_order_skips_the_tier(monkeypatch):
    # arcs of one source into one target in descending olabel order (a blob written by
    # hand keeps file order): (id, ol) != (id, candidate), so the tier must not run; the
    # chain still answers exactly
    monkeypatch.setenv("FSTAMD_LAZY_ONLY_FIRST", "1")
    f = O.Fst()
    for i in range(6):
        f.add_state(0.0)
    f.start = 0
    for i in range(6):
        f.add_arc(i, 1, 9, 0.0, (i + 1) % 6)
        f.add_arc(i, 1, 3, 0.0, (i + 1) % 6)
    blob = bytearray(O.freeze(f))
    # swap the two arcs of every state in place (same ilabel: the blob stays valid)
    ns = 6
    base = 24 + 16 * ns
    for s in range(ns):
        a = base + 48 * s
        blob[a:a + 24], blob[a + 24:a + 48] = blob[a + 24:a + 48], blob[a:a + 24]
    blob = bytes(blob)
    labels, offsets = csr([[1] * 4, [1] * 7])
    got = F.compose_frozen_shortest_path_batch(load_blob(blob), labels, offsets, 1, LAZY)
    # the pull tier was skipped: the strings went to the rounds engine and are exact
    monkeypatch.delenv("FSTAMD_LAZY_ONLY_FIRST")
    check(blob, labels, offsets, LAZY)
    assert np.all(got.status == F.FST_PATH_OK)


def scaled_ambiguous(T, scale, stay=True):
    # the reference bench's ambiguous chain (bench/optimize-bench.zig:250-277) with its
    # weights b scaled: the pop-order keys d - dmin of a layer span ~3 k * scale
    f = O.Fst()
    for _ in range(T + 1):
        f.add_state(0.0)
    f.start = 0
    for i in range(T + 1):
        if stay:
            f.add_arc(i, 1, 1, 0.0, i)
        for b in range(4):
            f.add_arc(i, 1, (i + b) % 255 + 1, float(b * scale), min(i + b + 1, T))
    return f


@pytest.mark.parametrize("scale", [1, 7, 40, 1000])
def test_pop_order_sorts_counting_and_split(only_lp, scale):
    # layers of up to 257 tuples (5 chunks of 64 ids): scale 1 keeps every layer's keys
    # below 256 (the counting sort), 7 crosses 256 from layer ~13 on, 40 and 1000 use the
    # split sort almost everywhere; every string must match the oracle
    blob = O.freeze(scaled_ambiguous(300, scale))
    seqs = [[1] * L for L in (1, 2, 9, 17, 40, 64, 70)] + [[1] * 64] * 8
    got, took = run_lp(blob, seqs, expect_all=False)
    assert took.mean() > 0.5, took.mean()


@pytest.mark.parametrize("seed", range(4))
def test_random_wide_layers(only_lp, seed):
    # ~100-300 states, two labels: layers of well over 64 tuples with many equal integer
    # distances (chunks whose lanes share keys), some weights large enough to push the
    # key range past 256
    rng = np.random.default_rng(9900 + seed)
    ns = int(rng.integers(100, 300))
    f = O.Fst()
    for _ in range(ns):
        f.add_state(float(rng.integers(0, 3)) if rng.random() < 0.7 else math.inf)
    f.start = 0
    for s in range(ns):
        for _ in range(int(rng.integers(1, 5))):
            w = float(rng.integers(0, 3)) if rng.random() < 0.9 else float(rng.integers(50, 400))
            f.add_arc(s, int(rng.integers(1, 3)), int(rng.integers(1, 9)), w,
                      int(rng.integers(ns)))
    blob = O.freeze(f)
    seqs = [[int(x) for x in rng.integers(1, 3, int(rng.integers(0, 30)))] for _ in range(96)]
    run_lp(blob, seqs, expect_all=False)


@pytest.mark.parametrize("sem_case", ["ties", "counting", "wide"])
def test_many_strings_per_wave(only_lp, sem_case, monkeypatch):
    # FSTAMD_LP_GRID=3: three waves take every string, so each wave holds up to 14 pending
    # chase jobs (LazyPullLds::job, after the sort buffers) while it sorts later strings'
    # layers -- a sort that wrote past its buffers would corrupt them (round 4: the f32
    # cells' 128-bin counting sort wrote a 256-bin prefix)
    monkeypatch.setenv("FSTAMD_LP_GRID", "3")
    rng = np.random.default_rng(4242)
    if sem_case == "ties":
        f = random_rhs(rng, 40, 160, 3, eps=False, wmax=2)
        seqs = [[int(x) for x in rng.integers(1, 4, int(rng.integers(0, 16)))] for _ in range(400)]
    elif sem_case == "counting":
        f = scaled_ambiguous(300, 1)
        seqs = [[1] * int(L) for L in rng.integers(1, 70, 200)]
    else:
        f = scaled_ambiguous(300, 40)
        seqs = [[1] * int(L) for L in rng.integers(1, 70, 200)]
    got, took = run_lp(O.freeze(f), seqs, expect_all=False)
    assert took.mean() > 0.5, took.mean()
