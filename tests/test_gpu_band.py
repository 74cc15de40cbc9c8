"""The band replay (kernels/lazy_band.hpp): exact lazy composeShortestPath over a sliding
window of rhs states, for rhs whose arcs all go forward (RhsView::jump_back == 0) -- config
3's epsilon-dense transducer.  Every case is bit-compared with the oracle, and the route
log (FSTAMD_ROUTE_LOG, C-level stderr) shows which strings the band took:

* epsilon-dense lattices larger than the window (slides), lengths 0..251;
* random forward-only rhs with epsilon arcs, epsilon self-loops, tie-heavy weights and
  finals, with the 1-, 2- and 4-byte back-pointer encodings (arcs per state, jump sizes);
* a window forced too small (FSTAMD_BAND_WS): every string overflows to the dense replay,
  whose answers are the same;
* strings the band does not take (label 0: lhs epsilon phases) go on to the rounds engine.
"""
import math
import re

import numpy as np
import pytest

import libfst_amd as F
import oracle_ffi as O
from test_gpu_parity import LAZY, check, csr, load_blob

pytestmark = pytest.mark.gpu


def handed_on(err):
    """Strings each band launch handed on: the capped launch with the early exit, then
    (if any) the whole-rhs launch."""
    m = re.findall(r"band replay \([^)]*\) handed on (\d+)", err)
    return [int(x) for x in m]


@pytest.fixture(params=["early", "full"])
def early_mode(request, monkeypatch):
    """Both ways of running the band: with the exact early exit (the default) and the
    reference's whole-product replay (FSTAMD_NO_EARLY=1)."""
    if request.param == "full":
        monkeypatch.setenv("FSTAMD_NO_EARLY", "1")
    return request.param


@pytest.fixture
def route(monkeypatch):
    monkeypatch.setenv("FSTAMD_ROUTE_LOG", "1")
    monkeypatch.setenv("FSTAMD_LAZY_TINY", "0")  # straight to the band (no LDS replays)


def forward_rhs(rng, ns, deg, jump, labels=3, wmax=2, frac=False, eps_loops=True):
    """A rhs whose arcs go forward (t >= s): deg arcs per state, t - s <= jump."""
    f = O.Fst()
    for _ in range(ns):
        f.add_state(float(rng.integers(0, 3)) if rng.random() < 0.6 else math.inf)
    f.start = 0
    for s in range(ns):
        for _ in range(int(rng.integers(1, deg + 1))):
            il = int(rng.integers(0, labels + 1))
            t = min(ns - 1, s + int(rng.integers(0 if (il or eps_loops) else 1, jump + 1)))
            w = float(rng.integers(0, wmax + 1)) + (float(rng.random()) if frac else 0.0)
            f.add_arc(s, il, int(rng.integers(0, labels + 1)), w, t)
    return f


@pytest.mark.parametrize("T", [1024, 3000])
def test_eps_dense_slides(route, capfd, early_mode, T):
    blob = O.freeze(O.gen("eps_dense", T, 12))
    lens = [0, 1, 2, 11, 64, 130, 200, 251]
    check(blob, *csr([[1] * L for L in lens]), LAZY)
    assert handed_on(capfd.readouterr().err) == [0]


@pytest.mark.parametrize("seed", range(12))
def test_random_forward(route, capfd, early_mode, seed):
    rng = np.random.default_rng(7100 + seed)
    # deg / jump chosen so the back pointer takes 1 B (seeds 0-3), 2 B (4-7), 4 B (8-11)
    deg, jump = [(4, 3), (40, 5), (30, 5000)][seed // 4]
    ns = int(rng.integers(20, 400)) if seed < 8 else 6000
    f = forward_rhs(rng, ns, deg, jump, frac=seed % 3 == 0)
    blob = O.freeze(f)
    seqs = [[int(x) for x in rng.integers(1, 4, int(rng.integers(0, 40)))] for _ in range(24)]
    check(blob, *csr(seqs), LAZY)
    err = capfd.readouterr().err
    assert handed_on(err), err[-2000:]  # the band ran


def test_window_too_small_falls_back(route, capfd, monkeypatch):
    monkeypatch.setenv("FSTAMD_BAND_WS", "64")
    blob = O.freeze(O.gen("eps_dense", 512, 12))
    lens = [70, 90, 151]  # open states span L + 3 > 64
    check(blob, *csr([[1] * L for L in lens]), LAZY)
    # both band launches (capped, then the whole rhs) hand all three on
    assert handed_on(capfd.readouterr().err) == [3, 3]


def test_label0_strings_go_on(route, capfd):
    blob = O.freeze(O.gen("eps_dense", 256, 12))
    seqs = [[1] * 20, [1, 0, 1], [0], [1] * 33]
    got, _ = check(blob, *csr(seqs), LAZY)
    assert got.status[0] == F.FST_PATH_OK and got.status[3] == F.FST_PATH_OK


def test_early_exit_beyond_state_cap(route, capfd):
    # the capped launch keeps back pointers for 2 x window states past the start; strings
    # whose best final lies further (the epsilon-dense rhs with only its last state final)
    # overflow there and are answered by the whole-rhs launch (and again if the host entry
    # reruns the batch with a larger path arena: the paths carry ~T epsilon arcs)
    f = O.gen("eps_dense", 1000, 12)
    f.finals = [math.inf] * (f.num_states - 1) + [0.0]
    blob = O.freeze(f)
    check(blob, *csr([[1] * L for L in (1, 3, 8)]), LAZY)
    h = handed_on(capfd.readouterr().err)
    assert h and h[0::2] == [3] * len(h[0::2]) and h[1::2] == [0] * len(h[1::2]), h


@pytest.mark.parametrize("seed", range(4))
def test_negative_finals_no_early_exit(route, capfd, seed):
    # a negative final weight breaks the early exit's bound (total >= dist): such an rhs
    # goes to the hashed replay (weights not all >= +0), which takes no early exit, and the
    # answers stay the oracle's
    rng = np.random.default_rng(7300 + seed)
    f = forward_rhs(rng, int(rng.integers(20, 200)), 4, 3)
    for s in range(0, f.num_states, 3):
        f.finals[s] = -float(rng.integers(1, 4))
    blob = O.freeze(f)
    seqs = [[int(x) for x in rng.integers(1, 4, int(rng.integers(0, 30)))] for _ in range(24)]
    check(blob, *csr(seqs), LAZY)
    assert handed_on(capfd.readouterr().err) == []  # not the band


def test_without_arc_table(route, capfd, monkeypatch):
    # the strided per-state arc table (DeviceFst::band_il / band_rec) is the default; the
    # span-then-arcs reads without it must give the same answers
    monkeypatch.setenv("FSTAMD_NO_BAND_TABLE", "1")
    blob = O.freeze(O.gen("eps_dense", 1024, 12))
    check(blob, *csr([[1] * L for L in (0, 1, 11, 64, 200)]), LAZY)
    rng = np.random.default_rng(7400)
    f = forward_rhs(rng, 300, 40, 5)
    blob = O.freeze(f)
    seqs = [[int(x) for x in rng.integers(1, 4, int(rng.integers(0, 40)))] for _ in range(24)]
    check(blob, *csr(seqs), LAZY)
    assert handed_on(capfd.readouterr().err)


@pytest.mark.parametrize("seed", range(4))
def test_slot_fold_mixed_pops(route, capfd, early_mode, seed):
    # the slot fold takes a pop only when every candidate distance is a finite, >= +0 value
    # with 6 clear low mantissa bits; integer and dyadic weights with a few 0.1 ones make
    # pops of both kinds within one string, and states past 64 arcs (seeds 2, 3: no arc
    # table, the wave-wide span search) take the old fold throughout
    rng = np.random.default_rng(7500 + seed)
    deg = 8 if seed < 2 else 90
    f = forward_rhs(rng, int(rng.integers(40, 300)), deg, 6, labels=2)
    for st in range(len(f.arcs)):
        arcs = []
        for il, ol, w, t in f.arcs[st]:
            r = rng.random()
            arcs.append((il, ol, w + (0.1 if r < 0.1 else 0.5 if r < 0.3 else 0.0), t))
        f.arcs[st] = arcs
    blob = O.freeze(f)
    seqs = [[int(x) for x in rng.integers(1, 3, int(rng.integers(0, 40)))] for _ in range(32)]
    check(blob, *csr(seqs), LAZY)
    assert handed_on(capfd.readouterr().err)
