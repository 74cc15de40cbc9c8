"""GPU parity of every tier of the eager layered chain (device_engine.hip run_chain).

The chain is P (pull over the reverse mirror, eager_pull.hpp) -> A0 (direct-mapped
window, eager_window.hpp) -> A (hashed wave, eager_wave.hpp) -> B (256-thread LDS tables)
-> C (HBM tables) -> general BFS; each tier takes the strings the previous one reports as
OVERFLOW.  FSTAMD_EAGER_TIER1=window starts the chain at A0, =wave at A and =wg at B, so
each tier is checked on its own as well as behind the others, against the oracle's compose + shortestPath (compose.zig:29-198,
shortest-path.zig:18-139), bit-exact.
"""
import math

import numpy as np
import pytest

import libfst_amd as F
import oracle_ffi as O
from test_gpu_parity import check, csr, load_blob, random_rhs

pytestmark = pytest.mark.gpu

EAGER = F.FST_SEM_EAGER
STARTS = ["", "window", "wave", "wg"]


@pytest.fixture(params=STARTS, ids=["P", "A0", "A", "B"])
def tier(request, monkeypatch):
    if request.param:
        monkeypatch.setenv("FSTAMD_EAGER_TIER1", request.param)
    else:
        monkeypatch.delenv("FSTAMD_EAGER_TIER1", raising=False)
    return request.param


@pytest.fixture(scope="module")
def ambiguous():
    blob = O.freeze(O.gen("ambiguous", 4096, 12))
    return blob, load_blob(blob)


def test_metric_and_dead_strings(tier, ambiguous):
    blob, rhs = ambiguous
    rng = np.random.default_rng(5)
    seqs = [[1] * 64] * 8 + [[1] * L for L in (0, 1, 63, 65, 100, 128)]
    for _ in range(48):
        L = int(rng.integers(1, 80))
        s = [1] * L
        if rng.random() < 0.3:
            s[int(rng.integers(L))] = 2  # every rhs arc has ilabel 1: the lattice dies
        seqs.append(s)
    check(blob, *csr(seqs), EAGER, rhs=rhs)


def test_wide_window_random_graph(tier):
    # ~1000 states with random targets: every layer spans far more than A0's window of
    # 320 states, so A0 hands each string to A (and A to B once a layer exceeds 320).
    rng = np.random.default_rng(77)
    f = random_rhs(rng, 1000, 4000, 4, eps=False, frac=True)
    blob = O.freeze(f)
    seqs = [[int(x) for x in rng.integers(1, 5, int(rng.integers(0, 14)))] for _ in range(64)]
    check(blob, *csr(seqs), EAGER)


@pytest.mark.parametrize("seed", range(4))
def test_random_small_graphs(tier, seed):
    rng = np.random.default_rng(3000 + seed)
    f = random_rhs(rng, int(rng.integers(2, 300)), int(rng.integers(4, 900)), 4, eps=False,
                   frac=seed % 2 == 1)
    blob = O.freeze(f)
    seqs = [[int(x) for x in rng.integers(1, 5, int(rng.integers(0, 20)))] for _ in range(64)]
    check(blob, *csr(seqs), EAGER)


def test_long_spans_overflow_to_wide_tiers(tier):
    # 7 arcs per (state, label) > KMAX = 5 of the wave tiers: B takes every string
    f = O.Fst()
    ns = 40
    for _ in range(ns):
        f.add_state(0.0)
    f.start = 0
    for s in range(ns):
        for b in range(7):
            f.add_arc(s, 1, b + 1, float(b % 3), (s + b) % ns)
    blob = O.freeze(f)
    seqs = [[1] * L for L in (0, 1, 5, 12, 30)]
    check(blob, *csr(seqs), EAGER)


@pytest.mark.parametrize("jump", [3, 40, 200, 400])
def test_banded_and_long_jump_transducers(tier, jump):
    # Forward arcs i -> i+1..i+3 plus one long jump i -> i+jump and a backward arc: A0's
    # banded window (RhsView::jump_*) holds for small jumps, and falls back to the exact
    # per-candidate window (or hands the string on) when the band outgrows 320 states.
    f = O.Fst()
    ns = 700
    for i in range(ns):
        f.add_state(float(i % 3) if i % 5 else math.inf)
    f.start = 0
    rng = np.random.default_rng(jump)
    for i in range(ns):
        for b in range(1, 4):
            f.add_arc(i, 1 + (i + b) % 2, b, float(rng.integers(0, 3)), min(i + b, ns - 1))
        f.add_arc(i, 1, 7, 1.0, min(i + jump, ns - 1))
        f.add_arc(i, 2, 8, 0.5, max(i - 2, 0))
    blob = O.freeze(f)
    seqs = [[int(x) for x in rng.integers(1, 3, int(rng.integers(0, 40)))] for _ in range(48)]
    check(blob, *csr(seqs), EAGER)
