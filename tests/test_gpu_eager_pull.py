"""GPU parity of the pull tier (kernels/eager_pull.hpp) on its own.

FSTAMD_EAGER_ONLY_FIRST=1 stops the eager chain after tier P, so a string P cannot hold
stays OVERFLOW instead of moving on to the push tiers: these tests check both that P
takes what it should (banded / small rhs: every string) and that whatever it returns as
OK is bit-exact against the oracle's compose + shortestPath (compose.zig:29-198,
shortest-path.zig:18-139).  The shapes target the reverse mirror's corners: groups of in-
arcs longer than one block (hub states), several in-labels per state (gtab search),
same-label runs of 8 (j = 7), labels that collide with the span markers, full 320-state
layers (ranks up to 319, all 40 bitmap words), +inf arc and final weights -- each in the
direct and the indirect record layout.
"""
import math

import numpy as np
import pytest

import libfst_amd as F
import oracle_ffi as O
from test_gpu_parity import bits, csr, expected_status, load_blob, random_rhs

pytestmark = pytest.mark.gpu

EAGER = F.FST_SEM_EAGER


@pytest.fixture(params=["direct", "indirect"])
def only_p(request, monkeypatch):
    # direct: block 0 of every state at a fixed record index (single-label rhs, the
    # default there); indirect: group lookup first (FSTAMD_PULL_INDIRECT forces it)
    monkeypatch.setenv("FSTAMD_EAGER_ONLY_FIRST", "1")
    monkeypatch.delenv("FSTAMD_EAGER_TIER1", raising=False)
    if request.param == "indirect":
        monkeypatch.setenv("FSTAMD_PULL_INDIRECT", "1")
    else:
        monkeypatch.delenv("FSTAMD_PULL_INDIRECT", raising=False)


def run_p(blob, seqs, expect_all=True):
    """Tier P alone; every string it reports OK (or EMPTY) must match the oracle."""
    labels, offsets = csr(seqs)
    rhs = load_blob(blob)
    got = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, EAGER)
    ref = O.batch_run(blob, labels, offsets, 1, 1)
    exp = expected_status(ref)
    took = (got.status == F.FST_PATH_OK) | (got.status == F.FST_PATH_EMPTY)
    if expect_all:
        assert took.all(), np.unique(got.status, return_counts=True)
    assert np.array_equal(got.status[took], exp[took])
    for i in np.nonzero(took & (exp == F.FST_PATH_OK))[0]:
        a0, a1 = int(got.offsets[i]), int(got.offsets[i + 1])
        b0, b1 = int(ref.offsets[i]), int(ref.offsets[i + 1])
        assert np.array_equal(got.ilabels[a0:a1], ref.ilabels[b0:b1]), i
        assert np.array_equal(got.olabels[a0:a1], ref.olabels[b0:b1]), i
        assert np.array_equal(bits(got.weights[a0:a1]), bits(ref.weights[b0:b1])), i
        assert bits(got.finals[i:i + 1])[0] == bits(ref.finals[i:i + 1])[0], i
    return got, took


def test_metric_shape_entirely_in_p(only_p):
    blob = O.freeze(O.gen("ambiguous", 4096, 12))
    seqs = [[1] * 64] * 40 + [[1] * L for L in (0, 1, 2, 63, 65, 79)]
    seqs += [[1] * 30 + [2] + [1] * 10]  # dies halfway
    got, _ = run_p(blob, seqs)
    assert list(got.olabels[:64]) == [1] * 64
    # layer k of 1^k spans states 0..4k: from L = 80 on the window outgrows 320 states
    got, took = run_p(blob, [[1] * L for L in (80, 100, 128)], expect_all=False)
    assert np.all(got.status == F.FST_PATH_OVERFLOW)


@pytest.mark.parametrize("seed", range(6))
def test_random_graphs_under_window(only_p, seed):
    # ns <= 300 < 320: every window fits, so P must take every string.  Random targets
    # give hub states (in-groups over one block), labels 1..4 give several in-labels per
    # state, fractional weights give few ties, integer ones many.
    rng = np.random.default_rng(4400 + seed)
    ns = int(rng.integers(2, 300))
    f = random_rhs(rng, ns, int(rng.integers(ns, 6 * ns)), 4, eps=False, frac=seed % 2 == 1)
    blob = O.freeze(f)
    seqs = [[int(x) for x in rng.integers(1, 5, int(rng.integers(0, 24)))] for _ in range(96)]
    run_p(blob, seqs)


def test_hub_state_many_blocks(only_p):
    # every state has an arc into state 0 (a hub with ~250 in-arcs of one label: ~50
    # blocks) and a chain arc; ties at the hub are broken by the smallest source rank
    f = O.Fst()
    ns = 250
    for i in range(ns):
        f.add_state(0.0 if i % 7 == 0 else math.inf)
    f.start = 0
    for i in range(ns):
        f.add_arc(i, 1, 3, 0.0, 0)
        f.add_arc(i, 1, 4, 0.0, (i + 1) % ns)
        f.add_arc(i, 1, 5, 1.0, (i + 2) % ns)
    blob = O.freeze(f)
    run_p(blob, [[1] * L for L in (0, 1, 3, 10, 40, 90)])


def test_same_label_runs_of_eight(only_p):
    # 8 arcs of one label per state (j = 0..7, the key's full 3 bits), zero-weight ties
    f = O.Fst()
    ns = 200
    for i in range(ns):
        f.add_state(float(i % 2))
    f.start = 0
    for i in range(ns):
        for b in range(8):
            f.add_arc(i, 1, 10 + b, float(b % 2), (i + b) % ns)
    blob = O.freeze(f)
    run_p(blob, [[1] * L for L in (1, 2, 7, 20, 33)])


def test_full_window_layers(only_p):
    # 320 states, each with arcs to 4 random states: layers fill the whole window (ranks
    # up to 319, first keys in all 40 bitmap words)
    rng = np.random.default_rng(99)
    f = O.Fst()
    ns = 320
    for i in range(ns):
        f.add_state(float(rng.integers(0, 4)))
    f.start = 0
    for i in range(ns):
        for b in range(4):
            f.add_arc(i, 1, int(rng.integers(1, 9)), float(rng.integers(0, 2)),
                      int(rng.integers(ns)))
    blob = O.freeze(f)
    got, _ = run_p(blob, [[1] * L for L in (5, 12, 30)])


def test_marker_labels_and_infinities(only_p):
    # ilabels 0xFFFFFFFE / 0xFFFFFFFF (the span markers' values) and +inf arc / final
    # weights: the marker labels go through the group table, +inf never wins a back-pointer
    big = [0xFFFFFFFE, 0xFFFFFFFF]
    f = O.Fst()
    ns = 60
    for i in range(ns):
        f.add_state(math.inf if i % 4 == 0 else float(i % 3))
    f.start = 0
    for i in range(ns):
        f.add_arc(i, 1, 1, 0.0, (i + 1) % ns)
        f.add_arc(i, big[i % 2], 2, 1.0, (i + 2) % ns)
        f.add_arc(i, big[(i + 1) % 2], 3, math.inf, (i + 3) % ns)
        f.add_arc(i, 1, 4, math.inf, (i + 5) % ns)
    blob = O.freeze(f)
    rng = np.random.default_rng(5)
    seqs = [[int(rng.choice([1] + big)) for _ in range(int(rng.integers(0, 15)))] for _ in range(64)]
    run_p(blob, seqs)


def test_wide_rhs_hands_strings_on(only_p):
    # 1000 states with random targets: windows exceed 320, P reports OVERFLOW for those
    # strings (the push tiers take them in the full chain) and is exact on the rest
    rng = np.random.default_rng(77)
    f = random_rhs(rng, 1000, 4000, 4, eps=False, frac=True)
    blob = O.freeze(f)
    seqs = [[int(x) for x in rng.integers(1, 5, int(rng.integers(0, 14)))] for _ in range(64)]
    got, took = run_p(blob, seqs, expect_all=False)
    assert np.all((got.status[~took] == F.FST_PATH_OVERFLOW))


@pytest.mark.parametrize("wmax", [3, 200])
def test_many_strings_per_wave(only_p, wmax, monkeypatch):
    # FSTAMD_P_GRID=3: three waves take every string (16 back slabs each, chased in
    # batches), 8-B records (wmax 3) and 16-B ones (200)
    monkeypatch.setenv("FSTAMD_P_GRID", "3")
    rng = np.random.default_rng(4500 + wmax)
    f = random_rhs(rng, 120, 500, 3, eps=False, wmax=wmax)
    seqs = [[int(x) for x in rng.integers(1, 4, int(rng.integers(0, 40)))] for _ in range(500)]
    got, took = run_p(O.freeze(f), seqs, expect_all=False)
    assert took.mean() > 0.5, took.mean()
