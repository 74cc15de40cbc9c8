"""GPU parity of the lazy engines against the oracle's sequential composeShortestPath
(src/ops/compose-shortest-path.zig:26-401): the parallel rounds engines -- layered
(kernels/lazy_layered.hpp) and general (kernels/eager_bfs.hpp, bfs_lazy_path) -- and the
replay (kernels/lazy_wave.hpp) and the dense replay (kernels/lazy_dense.hpp).

FSTAMD_LAZY_ENGINE=replay | rounds | dense forces one engine (FSTAMD_LAZY_LAYERED=0 keeps the
rounds on the general engine); unset, the engine is chosen by the rhs and batch shape
(fst_last_launch_stats().engine: 1 replay, 3 general rounds, 4 layered + general,
5 dense replay + general rounds for its leftovers)."""
import math

import numpy as np
import pytest

import libfst_amd as F
import oracle_ffi as O
from test_gpu_parity import LAZY, check, csr, load_blob, random_rhs

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["rounds", "general", "replay", "replay_hbm", "dense", "lds", "lds_chain"])
def engine(request, monkeypatch):
    monkeypatch.delenv("FSTAMD_LAZY_ENGINE", raising=False)
    monkeypatch.delenv("FSTAMD_LAZY_LAYERED", raising=False)
    monkeypatch.delenv("FSTAMD_LAZY_TINY", raising=False)
    if request.param.startswith("lds"):  # the LDS replay (kernels/lazy_tiny.hpp) first
        monkeypatch.setenv("FSTAMD_LAZY_ENGINE", "lds")
        if request.param == "lds_chain":  # 128 tuples first, then 256, 512, 1024, HBM;
            # 4 waves: each takes many strings (tables reused across strings)
            monkeypatch.setenv("FSTAMD_LAZY_TINY_START", "1")
            monkeypatch.setenv("FSTAMD_TINY_WAVES", "4")
        return "dense"
    if request.param == "replay_hbm":  # the hashed replay without its LDS first launch
        monkeypatch.setenv("FSTAMD_LAZY_ENGINE", "replay")
        monkeypatch.setenv("FSTAMD_LAZY_TINY", "0")
        return "replay"
    if request.param in ("replay", "dense"):
        monkeypatch.setenv("FSTAMD_LAZY_ENGINE", request.param)
        return request.param
    monkeypatch.setenv("FSTAMD_LAZY_ENGINE", "rounds")
    if request.param == "general":  # general rounds engine only (no layered engine)
        monkeypatch.setenv("FSTAMD_LAZY_LAYERED", "0")
    return "rounds"


def expect_engine(engine):
    st = F.last_launch_stats()
    # 3 = general rounds engine, 4 = layered engine first (rhs without input epsilons)
    assert st.engine in {"rounds": (3, 4), "replay": (1,), "dense": (5,)}[engine]


@pytest.mark.parametrize("seed", range(16))
def test_random_tie_heavy(engine, seed):
    rng = np.random.default_rng(31000 + seed)
    f = random_rhs(rng, int(rng.integers(2, 30)), int(rng.integers(4, 120)), 3,
                   eps=seed % 4 != 3, wmax=2, frac=seed % 3 == 0)
    blob = O.freeze(f)
    seqs = [[int(x) for x in rng.integers(0, 4, int(rng.integers(0, 10)))] for _ in range(48)]
    check(blob, *csr(seqs), LAZY)
    expect_engine(engine)


def test_metric_shape(engine):
    blob = O.freeze(O.gen("ambiguous", 4096, 12))
    rhs = load_blob(blob)
    seqs = [[1] * 64] * 6 + [[1] * L for L in (0, 1, 2, 17, 63, 128)] + [[1, 2, 1]]
    check(blob, *csr(seqs), LAZY, rhs=rhs)
    expect_engine(engine)


@pytest.mark.parametrize("T,lens", [(64, (0, 1, 5, 12, 40)), (256, (11, 24, 40))])
def test_epsilon_dense(engine, T, lens):
    blob = O.freeze(O.gen("eps_dense", T, 12))
    check(blob, *csr([[1] * L for L in lens]), LAZY)
    expect_engine(engine)


def test_zero_weight_cycles_through_start(engine):
    # start carries 0-weight self loops and a 0-weight 2-cycle: the lazy backtrace stops
    # at the start id (compose-shortest-path.zig:372), so these are not CYCLE
    f = O.Fst()
    for _ in range(3):
        f.add_state(math.inf)
    f.start = 0
    f.finals[2] = 0.0
    f.add_arc(0, 0, 5, 0.0, 0)
    f.add_arc(0, 1, 6, 0.0, 1)
    f.add_arc(1, 0, 7, 0.0, 0)
    f.add_arc(1, 1, 8, 0.0, 2)
    f.add_arc(2, 0, 9, 0.0, 1)
    check(O.freeze(f), *csr([[1], [1, 1], [1, 1, 1], []]), LAZY)
    expect_engine(engine)


def test_infinite_arc_weights_use_the_replay(monkeypatch):
    monkeypatch.delenv("FSTAMD_LAZY_ENGINE", raising=False)
    f = O.Fst()
    for _ in range(3):
        f.add_state(math.inf)
    f.start = 0
    f.finals[2] = 0.0
    f.add_arc(0, 1, 1, math.inf, 1)
    f.add_arc(0, 1, 2, 1.0, 1)
    f.add_arc(1, 1, 3, 0.0, 2)
    check(O.freeze(f), *csr([[1, 1], [1], [1, 1, 1]]), LAZY)
    assert F.last_launch_stats().engine == 1


def test_engines_agree_on_a_large_varied_batch(monkeypatch):
    blob = O.freeze(O.gen("ambiguous", 4096, 12))
    rhs = load_blob(blob)
    rng = np.random.default_rng(77)
    seqs = [[int(x) for x in (rng.random(int(L)) < 0.02) + 1] for L in rng.integers(0, 65, 2048)]
    labels, offsets = csr(seqs)
    monkeypatch.setenv("FSTAMD_LAZY_ENGINE", "rounds")
    a = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, LAZY)
    monkeypatch.setenv("FSTAMD_LAZY_ENGINE", "replay")
    b = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, LAZY)
    assert np.array_equal(a.status, b.status)
    assert np.array_equal(a.offsets, b.offsets)
    assert np.array_equal(a.ilabels, b.ilabels) and np.array_equal(a.olabels, b.olabels)
    assert np.array_equal(a.weights.view(np.uint64), b.weights.view(np.uint64))
    assert np.array_equal(a.finals.view(np.uint64), b.finals.view(np.uint64))


def test_wide_states(engine):
    # states with more than 64 arcs: candidates are enumerated in chunks of 64 (dense
    # replay) and relaxations of one pop hit the same target across chunks
    rng = np.random.default_rng(4242)
    f = O.Fst()
    for _ in range(6):
        f.add_state(float(rng.integers(0, 3)))
    f.start = 0
    for s in range(6):
        for _ in range(int(rng.integers(60, 140))):
            f.add_arc(s, int(rng.integers(0, 3)), int(rng.integers(0, 4)),
                      float(rng.integers(0, 3)), int(rng.integers(0, 6)))
    blob = O.freeze(f)
    seqs = [[int(x) for x in rng.integers(1, 3, int(rng.integers(0, 6)))] for _ in range(24)]
    check(blob, *csr(seqs), LAZY)
    expect_engine(engine)


@pytest.mark.parametrize("buckets", [2, 3, 7])
def test_dense_length_buckets(monkeypatch, buckets):
    # Length buckets of the dense replay (device_engine.hip run_lazy_dense): the strings
    # are sorted by length and launched per bucket, each launch sizing the per-wave dense
    # state by its own longest string.  Forced here (on a large rhs they start by
    # themselves); the answers must not depend on the partition.  Mixed lengths, label-0
    # strings (passed on to the general rounds engine) and random tie-heavy rhs.
    monkeypatch.setenv("FSTAMD_LAZY_ENGINE", "dense")
    monkeypatch.setenv("FSTAMD_DENSE_BUCKETS", str(buckets))
    rng = np.random.default_rng(4100 + buckets)
    blob = O.freeze(O.gen("eps_dense", 128, 12))
    lens = [int(x) for x in rng.integers(0, 60, 40)]
    check(blob, *csr([[1] * L for L in lens]), LAZY)
    assert F.last_launch_stats().engine == 5
    f = random_rhs(rng, 24, 90, 3, eps=True, wmax=2, frac=True)
    blob = O.freeze(f)
    seqs = [[int(x) for x in rng.integers(0 if i % 9 == 0 else 1, 4, int(rng.integers(0, 14)))]
            for i in range(64)]
    check(blob, *csr(seqs), LAZY)


def test_dense_replay_beyond_64k_lds(monkeypatch):
    # config 3 at full size (T = 65,536, L up to 251) needs ~65 KB of dynamic LDS for the
    # dense replay's summary bitmap; such a launch goes past HIP's default 64 KB limit.
    # FSTAMD_DENSE_LDS_MIN inflates a small launch to 100 KB: the engine must still run
    # (engine 5, not the rounds fallback) and be exact
    monkeypatch.setenv("FSTAMD_LAZY_ENGINE", "dense")
    monkeypatch.setenv("FSTAMD_DENSE_LDS_MIN", "100000")
    blob = O.freeze(O.gen("eps_dense", 256, 12))
    check(blob, *csr([[1] * L for L in (0, 3, 11, 24, 40)]), LAZY)
    assert F.last_launch_stats().engine == 5
