"""The parallel lazy-engine plan (tests/lazy_model.py) against the oracle's
sequential composeShortestPath replay (src/ops/compose-shortest-path.zig:26-401).

CPU only: the model is the specification the device engine is built to; it must give the
reference's exact result (ids, back-pointers, best, backtrace) on every input."""
import numpy as np
import pytest

import lazy_model as M
import oracle_ffi as O
from test_gpu_parity import random_rhs


def oracle_lazy(lhs, blob):
    rc, res = O.compose_shortest_path(lhs, blob, 1)
    if rc == O.OR_ERR_CYCLE:
        return "cycle"
    assert rc == O.OR_OK
    return O.chain(res)


def chain_of(labels):
    f = O.Fst()
    for _ in range(len(labels) + 1):
        f.add_state()
    f.start = 0
    f.finals[len(labels)] = 0.0
    for i, x in enumerate(labels):
        f.add_arc(i, x, x, 0.0, i + 1)
    return f


@pytest.mark.parametrize("block", range(4))
def test_model_random_with_epsilons(block):
    for seed in range(block * 100, block * 100 + 100):
        rng = np.random.default_rng(9000 + seed)
        lhs = random_rhs(rng, int(rng.integers(1, 8)), int(rng.integers(1, 25)), 3, eps=True,
                         wmax=2, frac=seed % 3 == 0)
        rhs = random_rhs(rng, int(rng.integers(1, 15)), int(rng.integers(1, 60)), 3, eps=True,
                         wmax=2, frac=seed % 3 == 0)
        blob = O.freeze(rhs)
        got, _ = M.lazy_via_rounds(lhs, blob)
        assert got == oracle_lazy(lhs, blob), seed


@pytest.mark.parametrize("name,T,L,max_rounds", [("ambiguous", 4096, 64, 257),
                                                 ("eps_dense", 64, 12, None)])
def test_model_bench_shapes(name, T, L, max_rounds):
    lhs = chain_of([1] * L)
    blob = O.freeze(O.gen(name, T, 12))
    got, rounds = M.lazy_via_rounds(lhs, blob)
    assert got == oracle_lazy(lhs, blob)
    if max_rounds is not None:
        # 4 pops' worth of depth per input symbol: the metric's 8385 pops in 257 rounds
        assert rounds <= max_rounds


@pytest.mark.parametrize("block", range(3))
def test_bucket_model_random(block):
    """The dense replay's model (kernels/lazy_dense.hpp: open-at-dcur bitmap + future list)
    gives the oracle's exact lazy result on chain inputs without label 0."""
    for seed in range(block * 200, block * 200 + 200):
        rng = np.random.default_rng(5000 + seed)
        rhs = random_rhs(rng, int(rng.integers(1, 15)), int(rng.integers(1, 60)), 3, eps=True,
                         wmax=2, frac=seed % 3 == 0)
        labels = [int(x) for x in rng.integers(1, 4, size=int(rng.integers(0, 9)))]
        blob = O.freeze(rhs)
        assert M.lazy_via_buckets(labels, rhs) == oracle_lazy(chain_of(labels), blob), seed


@pytest.mark.parametrize("name,T,L", [("eps_dense", 64, 12), ("eps_dense", 256, 24),
                                      ("ambiguous", 4096, 64)])
def test_bucket_model_bench_shapes(name, T, L):
    rhs = O.gen(name, T, 12)
    st = {"order": []}
    got = M.lazy_via_buckets([1] * L, rhs, st)
    assert got == oracle_lazy(chain_of([1] * L), O.freeze(rhs))
    # pops run in near-id order: the cached lowest leaf serves almost every pop
    o = st["order"]
    leaf_changes = sum(1 for a, b in zip(o, o[1:]) if a // 64 != b // 64)
    assert leaf_changes <= len(o) // 8


@pytest.mark.parametrize("block", range(3))
def test_early_exit_model_random(block):
    """The band replay's early exit on the bucket model: same answers as
    the oracle's whole replay on random tie-heavy epsilon rhs (finals >= 0; any arc
    direction: the argument does not need forward arcs), with fewer pops on most."""
    saved = 0
    for seed in range(block * 300, block * 300 + 300):
        rng = np.random.default_rng(7700 + seed)
        rhs = random_rhs(rng, int(rng.integers(1, 20)), int(rng.integers(1, 80)), 3, eps=True,
                         wmax=2, frac=seed % 3 == 0)
        labels = [int(x) for x in rng.integers(1, 4, size=int(rng.integers(0, 10)))]
        blob = O.freeze(rhs)
        full, early = {}, {}
        want = oracle_lazy(chain_of(labels), blob)
        assert M.lazy_via_buckets(labels, rhs, full) == want, seed
        assert M.lazy_via_buckets(labels, rhs, early, early=True) == want, seed
        assert early["pops"] <= full["pops"]
        saved += full["pops"] - early["pops"]
    assert saved > 0


def test_early_exit_model_negative_finals_not_taken():
    rng = np.random.default_rng(7799)
    rhs = random_rhs(rng, 12, 50, 3, eps=True, wmax=2)
    rhs.finals = [-1.0 if not np.isinf(x) else x for x in rhs.finals]
    st = {}
    labels = [1, 2, 3, 1]
    assert M.lazy_via_buckets(labels, rhs, st, early=True) == \
        oracle_lazy(chain_of(labels), O.freeze(rhs))
    assert not st["early_exit"]


@pytest.mark.parametrize("T,L", [(512, 24), (2048, 40)])
def test_early_exit_model_eps_dense(T, L):
    # config 3's shape: the exit comes after ~2 L^2 pops whatever T is
    rhs = O.gen("eps_dense", T, 12)
    st = {}
    got = M.lazy_via_buckets([1] * L, rhs, st, early=True)
    assert got == oracle_lazy(chain_of([1] * L), O.freeze(rhs))
    assert st["early_exit"] and st["pops"] < 3 * L * L
