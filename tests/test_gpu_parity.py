"""GPU parity: the HIP engines vs the CPU oracle, through the C ABI, bit-exact.

Labels, state sequences and path structure must match exactly; f64 weights are
compared bit-for-bit (stricter than the 1e-9 the north star allows).  Oracle status
-> C ABI status: OK+empty -> FST_PATH_EMPTY, OK -> FST_PATH_OK, UnsupportedNShortest ->
FST_PATH_ERROR_N, back-pointer cycle (the reference would hang) -> FST_PATH_CYCLE.
"""
import math
import os
import tempfile

import numpy as np
import pytest

import libfst_amd as F
import oracle_ffi as O

pytestmark = pytest.mark.gpu

EAGER, LAZY = F.FST_SEM_EAGER, F.FST_SEM_LAZY


def load_blob(blob: bytes) -> F.Fst:
    with tempfile.NamedTemporaryFile(suffix=".fst", delete=False) as fh:
        fh.write(blob)
        p = fh.name
    try:
        return F.Fst.load(p)
    finally:
        os.unlink(p)


def expected_status(ref):
    st = np.full(len(ref.status), -1, np.int32)
    ok = ref.status == O.OR_OK
    st[ok & (ref.empty == 1)] = F.FST_PATH_EMPTY
    st[ok & (ref.empty == 0)] = F.FST_PATH_OK
    st[ref.status == O.OR_ERR_UNSUPPORTED_N] = F.FST_PATH_ERROR_N
    st[ref.status == O.OR_ERR_CYCLE] = F.FST_PATH_CYCLE
    return st


def bits(x):
    return np.ascontiguousarray(x, dtype=np.float64).view(np.uint64)


def check(blob, labels, offsets, sem, n=1, rhs=None, allow_unsupported=False):
    rhs = rhs or load_blob(blob)
    got = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, n, sem)
    ref = O.batch_run(blob, labels, offsets, 0 if sem == LAZY else 1, n)
    exp = expected_status(ref)
    if allow_unsupported and np.all(got.status == F.FST_PATH_UNSUPPORTED):
        return got, ref
    assert np.array_equal(got.status, exp), (np.nonzero(got.status != exp)[0][:10],
                                             got.status[got.status != exp][:10],
                                             exp[got.status != exp][:10])
    okm = exp == F.FST_PATH_OK
    # per-string path arrays
    assert np.array_equal(np.diff(got.offsets)[okm], np.diff(ref.offsets)[okm])
    for i in np.nonzero(okm)[0]:
        a0, a1 = int(got.offsets[i]), int(got.offsets[i + 1])
        b0, b1 = int(ref.offsets[i]), int(ref.offsets[i + 1])
        assert np.array_equal(got.ilabels[a0:a1], ref.ilabels[b0:b1]), i
        assert np.array_equal(got.olabels[a0:a1], ref.olabels[b0:b1]), i
        assert np.array_equal(bits(got.weights[a0:a1]), bits(ref.weights[b0:b1])), i
    assert np.array_equal(bits(got.finals[okm]), bits(ref.finals[okm]))
    return got, ref


def csr(seqs):
    lens = [len(s) for s in seqs]
    labels = np.concatenate([np.asarray(s, np.uint32) for s in seqs]) if seqs else np.zeros(0, np.uint32)
    offsets = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    return labels.astype(np.uint32), offsets


# ---------------------------------------------------------------------------------------
# metric workload (compose_frozen_shortest_path_ambiguous, T=4096, B=12)
# ---------------------------------------------------------------------------------------

@pytest.fixture(scope="module")
def ambiguous():
    blob = O.freeze(O.gen("ambiguous", 4096, 12))
    return blob, load_blob(blob)


@pytest.mark.parametrize("sem", [EAGER, LAZY])
def test_metric_strings(ambiguous, sem):
    blob, rhs = ambiguous
    labels, offsets = csr([[1] * 64] * 16)
    got, _ = check(blob, labels, offsets, sem, rhs=rhs)
    assert list(got.olabels[:64]) == [1] * 64


@pytest.mark.parametrize("sem", [EAGER, LAZY])
def test_metric_varied_batch(ambiguous, sem):
    blob, rhs = ambiguous
    rng = np.random.default_rng(11 + sem)
    seqs = []
    for _ in range(96):
        L = int(rng.integers(0, 65))
        s = [1] * L
        if L and rng.random() < 0.2:
            s[int(rng.integers(L))] = 2  # dies: every rhs arc has ilabel 1
        seqs.append(s)
    check(blob, *csr(seqs), sem, rhs=rhs)


def test_metric_full_length_range(ambiguous):
    blob, rhs = ambiguous
    seqs = [[1] * L for L in (0, 1, 2, 5, 11, 19, 33, 64, 96, 128)]
    check(blob, *csr(seqs), EAGER, rhs=rhs)
    check(blob, *csr(seqs[:8]), LAZY, rhs=rhs)


# ---------------------------------------------------------------------------------------
# other reference bench topologies
# ---------------------------------------------------------------------------------------

@pytest.mark.parametrize("sem", [EAGER, LAZY])
def test_branching_transducer(sem):
    blob = O.freeze(O.gen("branching_frozen_src", 512, 12))
    seqs = [[(i % 12) + 1 for i in range(L)] for L in (1, 7, 33, 64)]
    seqs += [[int(x) for x in np.random.default_rng(L).integers(1, 14, L)] for L in (5, 20, 40)]
    check(blob, *csr(seqs), sem)


def test_epsilon_dense_lazy_and_eager_route():
    blob = O.freeze(O.gen("eps_dense", 64, 12))
    seqs = [[1] * L for L in (0, 1, 3, 8, 17, 30)]
    check(blob, *csr(seqs), LAZY)
    check(blob, *csr(seqs), EAGER)  # general BFS engine (rhs epsilons)


# ---------------------------------------------------------------------------------------
# edge cases the reference defines
# ---------------------------------------------------------------------------------------

@pytest.mark.parametrize("sem", [EAGER, LAZY])
def test_n_and_empty_rules(ambiguous, sem):
    blob, rhs = ambiguous
    labels, offsets = csr([[1] * 3, [], [2]])
    for n in (0, 1, 2, 7):
        check(blob, labels, offsets, sem, n=n, rhs=rhs)
    empty = O.freeze(O.Fst())
    check(empty, labels, offsets, sem, n=1)
    check(empty, labels, offsets, sem, n=2)


def test_label_zero_inputs_lazy():
    # lhs epsilon outputs exercise phases 2 and 4 (compose-shortest-path.zig:227-365)
    blob = O.freeze(O.gen("eps_dense", 32, 6))
    seqs = [[1, 0, 1], [0], [0, 0, 1, 1], [1, 1, 0]]
    check(blob, *csr(seqs), LAZY)


# ---------------------------------------------------------------------------------------
# random transducers (tie-heavy small weights, epsilons, cycles)
# ---------------------------------------------------------------------------------------

def random_rhs(rng, ns, na, max_label, eps=True, wmax=3, frac=False):
    f = O.Fst()
    for _ in range(ns):
        f.add_state(float(rng.integers(0, 3)) if rng.random() < 0.5 else math.inf)
    f.start = 0
    lo = 0 if eps else 1
    for _ in range(na):
        w = float(rng.integers(0, wmax + 1))
        if frac:
            w += float(rng.random())
        f.add_arc(int(rng.integers(ns)), int(rng.integers(lo, max_label + 1)),
                  int(rng.integers(0, max_label + 1)), w, int(rng.integers(ns)))
    return f


@pytest.mark.parametrize("seed", range(8))
def test_random_lazy(seed):
    rng = np.random.default_rng(1000 + seed)
    f = random_rhs(rng, int(rng.integers(2, 40)), int(rng.integers(4, 160)), 4,
                   eps=seed % 2 == 0, frac=seed % 3 == 0)
    blob = O.freeze(f)
    seqs = [[int(x) for x in rng.integers(1, 5, int(rng.integers(0, 12)))] for _ in range(40)]
    check(blob, *csr(seqs), LAZY)


@pytest.mark.parametrize("seed", range(8))
def test_random_eager_layered(seed):
    rng = np.random.default_rng(2000 + seed)
    f = random_rhs(rng, int(rng.integers(2, 60)), int(rng.integers(4, 300)), 4, eps=False,
                   frac=seed % 2 == 1)
    blob = O.freeze(f)
    seqs = [[int(x) for x in rng.integers(1, 5, int(rng.integers(0, 16)))] for _ in range(64)]
    check(blob, *csr(seqs), EAGER)


# ---------------------------------------------------------------------------------------
# single-call C ABI: fst_compose_frozen_shortest_path with a general lhs MutableFst
# ---------------------------------------------------------------------------------------

def to_product(f: O.Fst) -> F.MutableFst:
    m = F.MutableFst()
    for _ in range(f.num_states):
        m.add_state()
    if f.start != O.NO_STATE:
        m.set_start(f.start)
    for s, fw in enumerate(f.finals):
        m.set_final(s, fw)
    for s, al in enumerate(f.arcs):
        for (il, ol, w, nx) in al:
            m.add_arc(s, il, ol, w, nx)
    return m


def compare_single(lhs: O.Fst, rhs_blob: bytes, n=1):
    rc, ref = O.compose_shortest_path(lhs, rhs_blob, n)
    got = F.compose_frozen_shortest_path(to_product(lhs), load_blob(rhs_blob), n)
    if rc == O.OR_ERR_UNSUPPORTED_N or rc == O.OR_ERR_CYCLE:
        assert got is None
        return
    assert rc == O.OR_OK and got is not None
    start, finals, arcs = got.to_lists()
    assert start == ref.start
    assert [bits([x]) for x in finals] == [bits([x]) for x in ref.finals]
    assert [[(a, b, bits([w])[0], d) for (a, b, w, d) in al] for al in arcs] == \
        [[(a, b, bits([w])[0], d) for (a, b, w, d) in al] for al in ref.arcs]


def test_single_call_known_answer():
    # compose-shortest-path.zig:447-471
    lhs = O.compile_string(b"123")
    rhs = O.freeze(O.compile_string_transducer(b"123", b"abc"))
    compare_single(lhs, rhs)
    got = F.compose_frozen_shortest_path(to_product(lhs), load_blob(rhs))
    assert got.print_string(output_tape=True) == b"abc"


def test_single_call_transducer_lhs_with_epsilons():
    lhs = O.compile_string_transducer(b"abcde", b"xy")      # epsilon outputs
    rhs = O.freeze(O.compile_string_transducer(b"xy", b"uvw"))  # epsilon inputs
    compare_single(lhs, rhs)


@pytest.mark.parametrize("seed", range(10))
def test_single_call_random_graphs(seed):
    rng = np.random.default_rng(3000 + seed)
    lhs = random_rhs(rng, int(rng.integers(1, 10)), int(rng.integers(1, 30)), 3, eps=True)
    rhs = random_rhs(rng, int(rng.integers(1, 20)), int(rng.integers(1, 80)), 3, eps=True)
    compare_single(lhs, O.freeze(rhs))


@pytest.mark.parametrize("rhs_kind", ["ambiguous", "eps_dense", "random_eps"])
def test_single_call_chain_route(rhs_kind):
    # a compileString lhs runs the batch engines on one string (c_api.cpp as_chain): the
    # layered pull tier on the metric rhs, the dense replay on an epsilon rhs; near-chains
    # (a weight, a second final, an output label that differs) keep the general-lhs path.
    # Both bit-exact against the oracle's composeShortestPath
    rng = np.random.default_rng(41)
    if rhs_kind == "ambiguous":
        blob = O.freeze(O.gen("ambiguous", 512, 12))
    elif rhs_kind == "eps_dense":
        blob = O.freeze(O.gen("eps_dense", 128, 6))
    else:
        blob = O.freeze(random_rhs(rng, 12, 60, 4, eps=True))
    # hand-built compileString-shaped chains with epsilon:epsilon (label 0) arcs: as_chain
    # takes them, the batch engines hand label-0 strings to the general engine
    for labels in ([0], [1, 0, 2], [0, 0, 1, 1, 0], [3, 0, 0, 0, 2, 1]):
        zero = O.Fst()
        for _ in range(len(labels) + 1):
            zero.add_state(math.inf)
        zero.start = 0
        zero.finals[len(labels)] = 0.0
        for i, x in enumerate(labels):
            zero.add_arc(i, x, x, 0.0, i + 1)
        compare_single(zero, blob)
    for text in (b"", b"\x00", b"\x00" * 37, bytes(rng.integers(0, 4, 19).tolist())):
        lhs = O.compile_string(text)
        compare_single(lhs, blob)
        if rhs_kind == "ambiguous" and text:
            assert F.last_launch_stats().engine == 7  # the lazy pull tier took it
        if len(text) > 2:
            near = O.compile_string(text)
            near.arcs[1] = [(near.arcs[1][0][0], near.arcs[1][0][1], 0.5, 2)]
            compare_single(near, blob)
            near = O.compile_string(text)
            near.finals[1] = 0.25
            compare_single(near, blob)
            near = O.compile_string(text)
            a = near.arcs[0][0]
            near.arcs[0] = [(a[0], a[1] + 1, a[2], a[3])]
            compare_single(near, blob)


# ---------------------------------------------------------------------------------------
# an rhs with scattered state ids (device renumbering, device_engine.hip bfs_renumbering)
# ---------------------------------------------------------------------------------------

def scattered(f: O.Fst, seed) -> O.Fst:
    perm = np.random.default_rng(seed).permutation(f.num_states)
    g = O.Fst(start=int(perm[f.start]), finals=[0.0] * f.num_states,
              arcs=[[] for _ in range(f.num_states)])
    for s, fw in enumerate(f.finals):
        g.finals[int(perm[s])] = fw
    for s, al in enumerate(f.arcs):
        g.arcs[int(perm[s])] = [(a, b, w, int(perm[d])) for (a, b, w, d) in al]
    return g


@pytest.mark.parametrize("sem", [EAGER, LAZY])
def test_scattered_state_ids_take_the_pull_tiers(sem):
    blob = O.freeze(scattered(O.gen("ambiguous", 2048, 12), 5))
    rhs = load_blob(blob)
    rng = np.random.default_rng(12)
    seqs = [[1] * int(L) for L in rng.integers(0, 97, 200)]
    check(blob, *csr(seqs), sem, rhs=rhs)
    # renumbered breadth-first on the device, the banded pull tiers take every string
    labels, offsets = csr([[1] * 64] * 64)
    F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem)
    st = F.last_launch_stats()
    assert st.engine == (7 if sem == LAZY else 0)
