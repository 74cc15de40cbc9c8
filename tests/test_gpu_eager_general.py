"""GPU parity of the general eager engine (kernels/eager_bfs.hpp) with the CPU oracle.

* fst_compose_frozen: the whole lattice (state numbering, arc order, labels, weight bits,
  finals) must equal src/ops/compose.zig's (oracle or_compose);
* fst_shortest_path: src/ops/shortest-path.zig (oracle or_shortest_path), non-negative
  weights; a back-pointer cycle (the reference would not terminate) -> invalid handle;
* batch eager semantics on lattices the layered kernels do not take (rhs epsilons,
  label-0 inputs), bit-exact against oracle compose + shortestPath.
"""
import math

import numpy as np
import pytest

import libfst_amd as F
import oracle_ffi as O
from test_gpu_parity import EAGER, LAZY, bits, check, csr, load_blob, random_rhs, to_product

pytestmark = pytest.mark.gpu


def lattice_lists(f):
    start, finals, arcs = f.to_lists()
    return (start, [int(bits([x])[0]) for x in finals],
            [[(a, b, int(bits([w])[0]), d) for (a, b, w, d) in al] for al in arcs])


def oracle_lists(f: O.Fst):
    return (f.start, [int(bits([x])[0]) for x in f.finals],
            [[(a, b, int(bits([w])[0]), d) for (a, b, w, d) in al] for al in f.arcs])


def compare_compose(lhs: O.Fst, blob: bytes):
    rc, ref = O.compose(lhs, blob)
    assert rc == O.OR_OK
    got = F.compose_frozen(to_product(lhs), load_blob(blob))
    assert got is not None
    g, r = lattice_lists(got), oracle_lists(ref)
    assert g[0] == r[0]
    assert len(g[1]) == len(r[1])
    assert g[1] == r[1]
    assert g[2] == r[2]


# ---------------------------------------------------------------------------------------
# fst_compose_frozen
# ---------------------------------------------------------------------------------------

def test_compose_known_answers():
    # compose.zig:223 (a -> b -> c), :282 (no final), :311 (frozen rhs)
    ab = O.compile_string_transducer(b"a", b"b")
    bc = O.freeze(O.compile_string_transducer(b"b", b"c"))
    compare_compose(ab, bc)
    nofinal = O.Fst()
    nofinal.add_state(float("inf"))
    nofinal.add_state(float("inf"))
    nofinal.start = 0
    nofinal.add_arc(0, 98, 98, 0.5, 1)
    compare_compose(O.compile_string(b"a"), O.freeze(nofinal))
    compare_compose(O.compile_string(b"123"), O.freeze(O.compile_string_transducer(b"123", b"abc")))


def test_compose_empty_sides():
    empty = O.Fst()
    compare_compose(O.compile_string(b"ab"), O.freeze(empty))
    got = F.compose_frozen(F.MutableFst(), load_blob(O.freeze(O.compile_string(b"ab"))))
    assert got is not None and got.num_states == 0


@pytest.mark.parametrize("L", [0, 1, 5, 17])
def test_compose_chain_vs_epsilon_dense(L):
    # config 1's shape (eager compose of a repeat string against eps-dense), small T
    compare_compose(chain_of([1] * L), O.freeze(O.gen("eps_dense", 48, 12)))


def chain_of(labels):
    f = O.Fst()
    for _ in range(len(labels) + 1):
        f.add_state(float("inf"))
    f.start = 0
    f.finals[len(labels)] = 0.0
    for i, x in enumerate(labels):
        f.add_arc(i, x, x, 0.0, i + 1)
    return f


@pytest.mark.parametrize("seed", range(12))
def test_compose_random_with_epsilons(seed):
    rng = np.random.default_rng(5000 + seed)
    lhs = random_rhs(rng, int(rng.integers(1, 12)), int(rng.integers(1, 40)), 3, eps=True)
    rhs = random_rhs(rng, int(rng.integers(1, 25)), int(rng.integers(1, 90)), 3, eps=True,
                     frac=seed % 2 == 1)
    compare_compose(lhs, O.freeze(rhs))


# ---------------------------------------------------------------------------------------
# fst_shortest_path on explicit FSTs
# ---------------------------------------------------------------------------------------

def compare_sp(f: O.Fst, n=1):
    rc, ref = O.shortest_path(f, n)
    got = F.shortest_path(to_product(f), n)
    if rc in (O.OR_ERR_UNSUPPORTED_N, O.OR_ERR_CYCLE):
        assert got is None
        return
    assert rc == O.OR_OK and got is not None
    assert lattice_lists(got) == oracle_lists(ref)


@pytest.fixture(params=["settle", "label-correcting", "sweeps"])
def sp_mode(request, monkeypatch):
    # the distances of fst_shortest_path: settled in distance order (default), label
    # correcting over a frontier (its fallback, forced by FSTAMD_SP_MAX_ADV=0 here), or
    # Gauss-Seidel sweeps over every arc (FSTAMD_SP_SWEEP)
    monkeypatch.delenv("FSTAMD_SP_SWEEP", raising=False)
    monkeypatch.delenv("FSTAMD_SP_MAX_ADV", raising=False)
    if request.param == "label-correcting":
        monkeypatch.setenv("FSTAMD_SP_MAX_ADV", "0")
    elif request.param == "sweeps":
        monkeypatch.setenv("FSTAMD_SP_SWEEP", "1")
    return request.param


@pytest.mark.parametrize("seed", range(12))
def test_shortest_path_random_graphs(seed, sp_mode):
    rng = np.random.default_rng(6000 + seed)
    f = random_rhs(rng, int(rng.integers(1, 30)), int(rng.integers(0, 120)), 4, eps=True,
                   frac=seed % 3 == 0)
    for n in (0, 1, 2):
        compare_sp(f, n)


@pytest.mark.parametrize("seed", range(4))
def test_shortest_path_large_tie_heavy_graphs(seed, sp_mode):
    # hundreds of nodes, 0-weight cycles and many equal distances: frontiers of several
    # chunks of 1024 nodes, nodes reached first at a larger distance and then lowered, and
    # (fractional weights) many distinct distances
    rng = np.random.default_rng(6100 + seed)
    ns = int(rng.integers(500, 3000))
    f = random_rhs(rng, ns, ns * int(rng.integers(2, 6)), 3, eps=True, wmax=2,
                   frac=seed % 2 == 1)
    compare_sp(f, 1)


def test_shortest_path_on_compose_result():
    # the eager pipeline through the two single-call entries
    lhs = O.compile_string(b"123")
    rhs = O.freeze(O.compile_string_transducer(b"123", b"abc"))
    lat = F.compose_frozen(to_product(lhs), load_blob(rhs))
    sp = F.shortest_path(lat, 1)
    assert sp.print_string(output_tape=True) == b"abc"


def test_shortest_path_negative_weight_chain():
    # a negative weight takes the exact heap replay (sp_replay_kernel)
    f = chain_of([1, 2])
    f.arcs[0][0] = (1, 1, -1.0, 1)
    compare_sp(f)
    assert F.last_launch_stats().engine == 6


def negative_graph(rng, ns, na, frac):
    # Forward arcs (s < next) carry weights in [-3, 3]; backward arcs and self-loops are
    # heavier than any negative forward path (no negative cycle), so back-pointer chains
    # end at the start.  A few -0.0 / -inf (a Zero) / -2.5 specials, negative finals.
    f = O.Fst()
    for _ in range(ns):
        fin = float(rng.integers(-2, 3)) if rng.random() < 0.5 else math.inf
        f.add_state(fin)
    f.start = 0
    specials = [-0.0, -math.inf, -2.5, 0.0]
    for _ in range(na):
        s, x = int(rng.integers(ns)), int(rng.integers(ns))
        w = float(rng.integers(-3, 4)) if s < x else float(rng.integers(250, 254))
        if frac:
            w += float(rng.random()) * (1 if w >= 0 else -1)
        if rng.random() < 0.06:
            w = specials[int(rng.integers(len(specials)))] if s < x else 250.0
        f.add_arc(s, int(rng.integers(0, 5)), int(rng.integers(0, 5)), w, x)
    return f


@pytest.mark.parametrize("seed", range(24))
def test_shortest_path_negative_weights(seed):
    # Dijkstra with negative arcs: settled states still move (shortest-path.zig:70-84) and
    # the answer depends on the (dist, id) pop order -- replayed exactly, checked against
    # the oracle's heap.  Back-pointer cycles (the reference would not terminate) are
    # reported as errors on both sides.
    rng = np.random.default_rng(6100 + seed)
    f = negative_graph(rng, int(rng.integers(2, 60)), int(rng.integers(1, 240)), seed % 2 == 1)
    compare_sp(f)


@pytest.mark.parametrize("seed", range(8))
def test_shortest_path_negative_cycles(seed):
    # unconstrained signs: mostly back-pointer cycles (zero-weight self-loops on the start,
    # negative cycles), which both sides report, plus the occasional path
    rng = np.random.default_rng(6200 + seed)
    f = random_rhs(rng, int(rng.integers(1, 40)), int(rng.integers(0, 160)), 4, eps=True,
                   frac=seed % 2 == 1)
    for s in range(len(f.arcs)):
        f.arcs[s] = [(il, ol, -w if rng.random() < 0.3 else w, nx) for il, ol, w, nx in f.arcs[s]]
    compare_sp(f)


# ---------------------------------------------------------------------------------------
# batch eager semantics beyond layered lattices
# ---------------------------------------------------------------------------------------

def test_batch_eager_epsilon_dense():
    blob = O.freeze(O.gen("eps_dense", 64, 12))
    seqs = [[1] * L for L in (0, 1, 3, 8, 17, 30)]
    check(blob, *csr(seqs), EAGER)


def test_batch_eager_label_zero_inputs():
    amb = O.freeze(O.gen("ambiguous", 256, 12))
    seqs = [[1, 0, 1], [0], [0, 0, 1, 1], [1, 1, 0], [1] * 9]  # layered tier takes the last
    check(amb, *csr(seqs), EAGER)
    eps = O.freeze(O.gen("eps_dense", 32, 6))
    check(eps, *csr(seqs), EAGER)


@pytest.mark.parametrize("seed", range(8))
def test_batch_eager_random_with_epsilons(seed):
    rng = np.random.default_rng(7000 + seed)
    f = random_rhs(rng, int(rng.integers(2, 40)), int(rng.integers(4, 160)), 4, eps=True,
                   frac=seed % 2 == 0)
    blob = O.freeze(f)
    seqs = [[int(x) for x in rng.integers(0, 5, int(rng.integers(0, 12)))] for _ in range(48)]
    check(blob, *csr(seqs), EAGER)


@pytest.mark.parametrize("seed", range(12))
def test_batch_eager_negative_weights(seed):
    # eager batch on an rhs with negative weights: the general engine builds each lattice
    # (compose.zig ids) and replays shortestPath's heap order on it (sp_replay), checked
    # bit-exact against the oracle's compose + heap Dijkstra, CYCLE statuses included
    rng = np.random.default_rng(6300 + seed)
    f = negative_graph(rng, int(rng.integers(2, 30)), int(rng.integers(4, 120)), seed % 2 == 1)
    blob = O.freeze(f)
    seqs = [[int(x) for x in rng.integers(0 if i % 7 == 0 else 1, 5, int(rng.integers(0, 10)))]
            for i in range(48)]
    check(blob, *csr(seqs), EAGER)
    assert F.last_launch_stats().engine == 6


@pytest.mark.parametrize("sem", ["eager", "eager_256", "eager_wide", "lazy_rounds"])
@pytest.mark.parametrize("seed", range(6))
def test_batch_tiny_tier_mixed_sizes(monkeypatch, sem, seed):
    # the general engine's tiny tiers (tables and labels in LDS) take the short strings;
    # strings past their label / node / arc / hash caps report OVERFLOW there and finish in
    # the HBM tiers.  Bit-exact against the oracle, for both semantics (lazy through the
    # general rounds engine).  Eager: the compact tables (eager_tiny.hpp) from 128 tuples,
    # from 256 (FSTAMD_BFS_TINY_START=2), and eager_bfs.hpp's kTiny tables
    # (FSTAMD_EAGER_CTINY=0)
    if sem == "lazy_rounds":
        monkeypatch.setenv("FSTAMD_LAZY_ENGINE", "rounds")
    if sem == "eager_256":
        monkeypatch.setenv("FSTAMD_BFS_TINY_START", "2")
    if sem == "eager_wide":
        monkeypatch.setenv("FSTAMD_EAGER_CTINY", "0")
    rng = np.random.default_rng(8100 + seed)
    f = random_rhs(rng, int(rng.integers(3, 24)), int(rng.integers(8, 80)), 4, eps=True,
                   frac=seed % 2 == 1)
    blob = O.freeze(f)
    lens = [int(x) for x in rng.integers(0, 24, 56)] + [100, 125, 126, 127, 140, 60, 90, 33]
    seqs = [[int(x) for x in rng.integers(1 if i % 5 else 0, 5, L)] for i, L in enumerate(lens)]
    check(blob, *csr(seqs), LAZY if sem == "lazy_rounds" else EAGER)


@pytest.mark.parametrize("env", ["FSTAMD_BFS_TINY", "FSTAMD_EAGER_CTINY"])
def test_batch_tiny_tier_off_matches(monkeypatch, env):
    # FSTAMD_BFS_TINY=0 (HBM tiers only) and FSTAMD_EAGER_CTINY=0 (eager_bfs.hpp's kTiny
    # tables instead of the compact ones) give the same bits as the default on config 4's
    # stand-ins
    import libfst_amd.synthetic as SY
    stages = [SY.to_mutable(SY.tagger()).freeze(), SY.to_mutable(SY.verbalizer()).freeze()]
    labels, offsets = SY.to_labels(SY.utterances(np.random.default_rng(9), 512))
    a = F.pipeline_batch(stages, labels, offsets, 1, EAGER)
    monkeypatch.setenv(env, "0")
    b = F.pipeline_batch(stages, labels, offsets, 1, EAGER)
    assert np.array_equal(a.status, b.status) and np.all(a.status == F.FST_PATH_OK)
    assert np.array_equal(a.offsets, b.offsets)
    assert np.array_equal(a.ilabels, b.ilabels) and np.array_equal(a.olabels, b.olabels)
    assert np.array_equal(a.weights.view(np.uint64), b.weights.view(np.uint64))
    assert np.array_equal(a.finals.view(np.uint64), b.finals.view(np.uint64))
