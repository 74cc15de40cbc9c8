"""GPU parity of the pull tiers' f32 cells (kernels/eager_pull.hpp, kernels/lazy_pull.hpp).

The pull tiers keep distances in f32 when every distance of the launch is an integer below
2^24 (integer arc weights in [0, 2^24) and max_len * max weight < 2^24: pull_f32 in
eager_pull.hip); every f32 sum, min and compare then equals the f64 one, so the answers
are the reference's f64 answers bit for bit (compose.zig:104, shortest-path.zig:72,
compose-shortest-path.zig:108).  These tests sit on the edges of that rule:
  * distances up to 2^24 - 1 (the largest exact f32 integers), f32 chosen;
  * the same rhs with one string longer, so the launch must take the f64 cells;
  * the f64 cells forced (FSTAMD_P_F64 / FSTAMD_LP_F64) on integer weights;
  * a device call whose max_len understates its strings: the f32 kernels must hand the
    longer strings on (their distances pass 2^24, where f32 would round).
"""
import ctypes as C

import numpy as np
import pytest
import torch

import libfst_amd as F
import libfst_amd.fst as FF
import oracle_ffi as O
from test_gpu_parity import bits, check, csr, expected_status, load_blob

pytestmark = pytest.mark.gpu

EAGER, LAZY = F.FST_SEM_EAGER, F.FST_SEM_LAZY


def banded_int_rhs(rng, ns, wmax, labels=3, fanout=3):
    """A banded rhs without input epsilon (tier P / LP window) and integer weights up to
    wmax, several in-arcs per state, ties on purpose (half the weights are wmax)."""
    f = O.Fst()
    for _ in range(ns):
        f.add_state(float(rng.integers(0, 5)) if rng.random() < 0.7 else float("inf"))
    f.start = 0
    for s in range(ns):
        for _ in range(fanout):
            t = min(ns - 1, s + int(rng.integers(0, 4)))
            w = float(wmax) if rng.random() < 0.5 else float(rng.integers(0, wmax + 1))
            f.add_arc(s, int(rng.integers(1, labels + 1)), int(rng.integers(1, 9)), w, t)
    return f


@pytest.mark.parametrize("sem", [EAGER, LAZY])
def test_distances_up_to_2p24(sem):
    rng = np.random.default_rng(77)
    max_len = 63
    wmax = (1 << 24) // max_len  # 63 * wmax = 2^24 - 1: the largest exact f32 integer
    assert max_len * wmax < 1 << 24 <= (max_len + 1) * wmax
    blob = O.freeze(banded_int_rhs(rng, 200, wmax))
    seqs = [[int(x) for x in rng.integers(1, 4, int(rng.integers(40, max_len + 1)))]
            for _ in range(300)]
    seqs.append([1] * max_len)
    check(blob, *csr(seqs), sem)
    # one string of 64 labels: the launch's max_len makes every distance bound 2^24 or
    # more, so the f64 cells run -- for every string of the batch
    check(blob, *csr(seqs + [[1] * (max_len + 1)]), sem)


@pytest.mark.parametrize("sem", [EAGER, LAZY])
def test_f64_cells_forced_on_integer_weights(sem, monkeypatch):
    monkeypatch.setenv("FSTAMD_P_F64", "1")
    monkeypatch.setenv("FSTAMD_LP_F64", "1")
    rng = np.random.default_rng(78)
    blob = O.freeze(banded_int_rhs(rng, 150, 7))
    seqs = [[int(x) for x in rng.integers(1, 4, int(rng.integers(0, 30)))] for _ in range(200)]
    check(blob, *csr(seqs), sem)


def device_call(rhs, seqs, max_len, sem):
    labels, offsets = csr(seqs)
    dev = torch.device("cuda", 0)
    lab = torch.as_tensor(labels.astype(np.int32), device=dev)
    off = torch.as_tensor(offsets.astype(np.int64), device=dev)
    n = len(seqs)
    cap = int(offsets[-1]) * 4 + 64
    status = torch.empty(n, dtype=torch.int32, device=dev)
    plen = torch.empty(n, dtype=torch.int32, device=dev)
    poff = torch.empty(n, dtype=torch.int64, device=dev)
    fin = torch.empty(n, dtype=torch.float64, device=dev)
    il = torch.empty(cap, dtype=torch.int32, device=dev)
    ol = torch.empty(cap, dtype=torch.int32, device=dev)
    w = torch.empty(cap, dtype=torch.float64, device=dev)
    cur = torch.zeros(1, dtype=torch.int64, device=dev)
    desc = FF.FstDeviceBatch(status.data_ptr(), plen.data_ptr(), poff.data_ptr(),
                             fin.data_ptr(), il.data_ptr(), ol.data_ptr(), w.data_ptr(), cap,
                             cur.data_ptr(), 0)
    opts = FF.FstBatchOptions(0, sem, 0)
    rc = F.lib().fst_device_compose_shortest_path(
        rhs.h, C.c_void_p(lab.data_ptr()), C.c_void_p(off.data_ptr()), n, max_len, 1,
        C.byref(opts), C.byref(desc), None)
    assert rc == FF.FST_OK
    torch.cuda.synchronize()
    return (status.cpu().numpy(), plen.cpu().numpy(), poff.cpu().numpy(), fin.cpu().numpy(),
            il.cpu().numpy().view(np.uint32), ol.cpu().numpy().view(np.uint32), w.cpu().numpy())


@pytest.mark.parametrize("sem", [EAGER, LAZY])
def test_understated_max_len_hands_longer_strings_on(sem):
    rng = np.random.default_rng(79)
    wmax = (1 << 24) // 32 + 1  # 32 labels reach 2^24 + 32: odd sums round in f32
    blob = O.freeze(banded_int_rhs(rng, 160, wmax))
    rhs = load_blob(blob)
    seqs = [[int(x) for x in rng.integers(1, 4, L)] for L in (8, 31, 40, 48, 60, 16, 55)]
    # the caller claims max_len 16: f32 by that bound, but 5 strings are longer
    status, plen, poff, fin, il, ol, w = device_call(rhs, seqs, 16, sem)
    labels, offsets = csr(seqs)
    ref = O.batch_run(blob, labels, offsets, 0 if sem == LAZY else 1, 1)
    exp = expected_status(ref)
    assert np.array_equal(status, exp)
    for i in np.nonzero(exp == F.FST_PATH_OK)[0]:
        a, b = int(ref.offsets[i]), int(ref.offsets[i + 1])
        assert plen[i] == b - a, i
        g = slice(int(poff[i]), int(poff[i]) + b - a)
        assert np.array_equal(il[g], ref.ilabels[a:b]), i
        assert np.array_equal(ol[g], ref.olabels[a:b]), i
        assert np.array_equal(bits(w[g]), bits(ref.weights[a:b])), i
        assert bits(fin[i:i + 1])[0] == bits(ref.finals[i:i + 1])[0], i


@pytest.mark.parametrize("sem", [EAGER, LAZY])
@pytest.mark.parametrize("wmax", [7, 8])
def test_record_widths_at_the_rec8_bound(sem, wmax, monkeypatch):
    # integer weights <= 7 take the 8-B records (RevView::rrec8: the weight in y's low 3
    # bits, riding in the candidate keys); 8 takes the 16-B rrec32.  Both, and the 16-B
    # records forced (FSTAMD_NO_REC8), give the oracle's bits -- ties on purpose (half the
    # weights are wmax, finals 0..4)
    rng = np.random.default_rng(80 + wmax)
    blob = O.freeze(banded_int_rhs(rng, 180, wmax))
    seqs = [[int(x) for x in rng.integers(1, 4, int(rng.integers(0, 50)))] for _ in range(300)]
    check(blob, *csr(seqs), sem)
    # tier P's 4-B records (RevView::rrec4: sources relative to targets; the random suites
    # cover backward arcs) off, then the 8-B ones too
    monkeypatch.setenv("FSTAMD_NO_REC4", "1")
    check(blob, *csr(seqs), sem)
    monkeypatch.setenv("FSTAMD_NO_REC8", "1")
    check(blob, *csr(seqs), sem)


@pytest.mark.parametrize("sem", [EAGER, LAZY])
@pytest.mark.parametrize("back", [7_800, 8_100])
def test_long_backward_arc_and_the_rec4_bias(sem, back, monkeypatch):
    # tier P's 4-B records hold 8 * (target - source) + bias; a padding record is 0xFFFF.
    # One backward arc of `back` states makes the bias ~8 * back, so rows of windows near
    # state 0 (t >= (0xFFFF - bias) / 8) would read padding as an in-window cell if the
    # records were built: the bound must refuse them (both sizes straddle the old,
    # bias-only bound) and the answers stay the oracle's, with and without FSTAMD_NO_REC4
    ns = back + 200
    f = O.Fst()
    for i in range(ns):
        f.add_state(float(i % 3))
    f.start = 0
    for s in range(ns - 1):
        f.add_arc(s, 1, 1 + s % 5, float(s % 2), s + 1)
        f.add_arc(s, 1, 7, 3.0, min(ns - 1, s + 2))
        f.add_arc(s, 3, 9, 1.0, s)
    f.add_arc(back, 2, 11, 0.0, 0)  # the only backward arc
    blob = O.freeze(f)
    rng = np.random.default_rng(back)
    seqs = [[1] * L for L in (60, 100, 150, 200, 250)]
    seqs += [[int(x) for x in rng.choice([1, 1, 1, 3], int(rng.integers(80, 250)))]
             for _ in range(60)]
    check(blob, *csr(seqs), sem)
    monkeypatch.setenv("FSTAMD_NO_REC4", "1")
    check(blob, *csr(seqs), sem)


def dyadic_rhs(rng, ns, den, nmax, final=None):
    """banded_int_rhs with every arc weight n / den, n in [0, nmax] (one arc 1 / den, so
    den is the smallest scale that makes them integers); finals as given, or k / 4."""
    f = O.Fst()
    for _ in range(ns):
        fw = final if final is not None else float(rng.integers(0, 9)) / 4
        f.add_state(fw if rng.random() < 0.7 else float("inf"))
    f.start = 0
    for s in range(ns):
        for _ in range(3):
            t = min(ns - 1, s + int(rng.integers(0, 4)))
            n = nmax if rng.random() < 0.5 else int(rng.integers(0, nmax + 1))
            f.add_arc(s, int(rng.integers(1, 4)), int(rng.integers(1, 9)), n / den, t)
    f.add_arc(0, 1, 1, 1.0 / den, 0)
    return f


def routed_records(err, sem):
    tag = "[libfst_amd route] %s pull: records " % ("eager" if sem == EAGER else "lazy")
    got = [ln[len(tag):].split(", weight scale ") for ln in err.splitlines() if ln.startswith(tag)]
    assert got, err
    return {(int(r), float(s)) for r, s in got}


@pytest.mark.parametrize("sem", [EAGER, LAZY])
@pytest.mark.parametrize("den,nmax", [(2, 7), (4, 31), (256, 255), (256, 9000)])
def test_dyadic_weights_take_the_integer_records(sem, den, nmax, monkeypatch, capfd):
    # weights n / 2^k (grammar costs like 0.5, 1.25): the mirror scales them by 2^k into the
    # integer records; every f64 sum of them is exact, so integer sums order and tie as the
    # reference's f64 ones, and the kernels unscale (exactly) only what they output
    monkeypatch.setenv("FSTAMD_ROUTE_LOG", "1")
    rng = np.random.default_rng(90 + den + nmax)
    blob = O.freeze(dyadic_rhs(rng, 180, den, nmax))
    seqs = [[int(x) for x in rng.integers(1, 4, int(rng.integers(0, 50)))] for _ in range(300)]
    capfd.readouterr()
    check(blob, *csr(seqs), sem)
    # the compact records (tier P's 4-B / the 8-B ones) up to 7, the 16-B ones above; the
    # lazy f32 cells only up to 255 (kLpF32WMax), f64 cells (scale 1) past it
    # (tier P's 4-B records need the direct layout as well: 3 or 2 for eager)
    if nmax <= 7:
        want = {(3, den), (2, den)} if sem == EAGER else {(2, den)}
    else:
        want = {(1, den)} if sem == EAGER or nmax <= 255 else {(0, 1.0)}
    got = routed_records(capfd.readouterr().err, sem)
    assert len(got) == 1 and got <= want, got


@pytest.mark.parametrize("sem", [EAGER, LAZY])
@pytest.mark.parametrize("den", [3, 10, 512])
def test_non_dyadic_weights_take_the_f64_cells(sem, den, monkeypatch, capfd):
    # 1/3, 0.1 and 2^-9 (past the largest scale, 2^8): no integer records, f64 cells
    monkeypatch.setenv("FSTAMD_ROUTE_LOG", "1")
    rng = np.random.default_rng(95 + den)
    blob = O.freeze(dyadic_rhs(rng, 150, den, 7))
    seqs = [[int(x) for x in rng.integers(1, 4, int(rng.integers(0, 40)))] for _ in range(200)]
    capfd.readouterr()
    check(blob, *csr(seqs), sem)
    # eager: tier P's 4-B records with indices into the table of distinct weights (RK 4,
    # f64 cells) when the rhs has the direct layout, else the f64 records (the lazy pull:
    # the f64 records -- its own table-index records measured slower)
    got = routed_records(capfd.readouterr().err, sem)
    assert got <= ({(4, 1.0), (0, 1.0)} if sem == EAGER else {(0, 1.0)}) and len(got) == 1, got


def metric_like_rhs(T, B, delta):
    """bench.fractional_ambiguous at a small T: the metric's chain, every weight + delta"""
    f = O.Fst()
    for _ in range(T + 1):
        f.add_state(0.0)
    f.start = 0
    for i in range(T + 1):
        f.add_arc(i, 1, 1, 0.0 + delta, i)
        for b in range(max(1, min(B, 4))):
            f.add_arc(i, 1, ((i + b) % 255) + 1, float(b) + delta, min(i + b + 1, T))
    return f


@pytest.mark.parametrize("sem", [EAGER, LAZY])
@pytest.mark.parametrize("delta", [0.1, 1.0 / 3.0])
def test_weight_table_records_on_the_metric_shape(sem, delta, monkeypatch, capfd):
    # non-dyadic weights on the metric's chain: tier P reads 4-B records whose low byte
    # indexes the weight table (RK 4), with f64 cells; the lazy pull its f64 records.
    # Bit-exact with the oracle, and with the f64 records (FSTAMD_NO_REC4) -- ties on
    # purpose (every string is 1^L)
    monkeypatch.setenv("FSTAMD_ROUTE_LOG", "1")
    blob = O.freeze(metric_like_rhs(512, 12, delta))
    rng = np.random.default_rng(99)
    seqs = [[1] * int(L) for L in rng.integers(0, 65, 400)] + [[1] * 64] * 8
    capfd.readouterr()
    check(blob, *csr(seqs), sem)
    assert routed_records(capfd.readouterr().err, sem) == {(4 if sem == EAGER else 0, 1.0)}
    monkeypatch.setenv("FSTAMD_NO_REC4", "1")
    check(blob, *csr(seqs), sem)
    assert routed_records(capfd.readouterr().err, sem) == {(0, 1.0)}


@pytest.mark.parametrize("sem", [EAGER, LAZY])
def test_more_distinct_weights_than_the_table_holds(sem, monkeypatch, capfd):
    # 65 distinct non-dyadic weights: one more than the table holds, so the f64 records
    monkeypatch.setenv("FSTAMD_ROUTE_LOG", "1")
    f = metric_like_rhs(512, 12, 0.1)
    for i in range(65):
        f.add_arc(i, 2, 1, 0.1 + i / 7.0, i + 1)
    blob = O.freeze(f)
    rng = np.random.default_rng(100)
    seqs = [[int(x) for x in rng.choice([1, 1, 1, 2], int(L))] for L in rng.integers(0, 65, 300)]
    capfd.readouterr()
    check(blob, *csr(seqs), sem)
    assert routed_records(capfd.readouterr().err, sem) == {(0, 1.0)}


@pytest.mark.parametrize("sem", [EAGER, LAZY])
@pytest.mark.parametrize("nw", [64, 65, 200, 256, 257])
def test_wide_weight_tables(sem, nw, monkeypatch, capfd):
    # nw distinct non-dyadic weights on the metric's chain (the direct layout): up to 64
    # tier P's 4-B records index the 64-entry table (RK 4), up to 256 the 256-entry one
    # (RK 5, round 6), beyond that the f64 records; the lazy pull reads its f64 records.
    # Bit-exact with the oracle and with the f64 records (FSTAMD_NO_REC4)
    monkeypatch.setenv("FSTAMD_ROUTE_LOG", "1")
    vals = [0.1 + k / 7.0 for k in range(nw)]
    T = 600
    f = O.Fst()
    for _ in range(T + 1):
        f.add_state(0.0)
    f.start = 0
    for i in range(T + 1):
        f.add_arc(i, 1, 1, vals[(5 * i) % nw], i)
        for b in range(4):
            f.add_arc(i, 1, ((i + b) % 255) + 1, vals[(5 * i + b + 1) % nw], min(i + b + 1, T))
    blob = O.freeze(f)
    assert len({w for al in f.arcs for (_, _, w, _) in al}) == nw
    rng = np.random.default_rng(101 + nw)
    seqs = [[1] * int(L) for L in rng.integers(0, 65, 300)] + [[1] * 64] * 8
    capfd.readouterr()
    check(blob, *csr(seqs), sem)
    want = (4 if nw <= 64 else 5 if nw <= 256 else 0) if sem == EAGER else 0
    assert routed_records(capfd.readouterr().err, sem) == {(want, 1.0)}
    monkeypatch.setenv("FSTAMD_NO_REC4", "1")
    check(blob, *csr(seqs), sem)
    assert routed_records(capfd.readouterr().err, sem) == {(0, 1.0)}


@pytest.mark.parametrize("sem", [EAGER, LAZY])
def test_dyadic_weights_with_non_dyadic_finals(sem, monkeypatch, capfd):
    # the best final adds a final weight of 0.1 to the unscaled distance in f64, as the
    # reference does; ties between finals broken by id
    monkeypatch.setenv("FSTAMD_ROUTE_LOG", "1")
    rng = np.random.default_rng(97)
    blob = O.freeze(dyadic_rhs(rng, 160, 8, 7, final=0.1))
    seqs = [[int(x) for x in rng.integers(1, 4, int(rng.integers(0, 45)))] for _ in range(300)]
    capfd.readouterr()
    check(blob, *csr(seqs), sem)
    got = routed_records(capfd.readouterr().err, sem)
    assert len(got) == 1 and got <= ({(3, 8.0), (2, 8.0)} if sem == EAGER else {(2, 8.0)}), got


@pytest.mark.parametrize("sem", [EAGER, LAZY])
def test_dyadic_distances_up_to_2p24(sem, monkeypatch, capfd):
    # scaled distances up to 2^24 - 1 keep the f32 cells; one string more takes f64 cells
    monkeypatch.setenv("FSTAMD_ROUTE_LOG", "1")
    rng = np.random.default_rng(98)
    max_len = 63
    nmax = (1 << 24) // max_len
    blob = O.freeze(dyadic_rhs(rng, 200, 64, nmax))
    seqs = [[int(x) for x in rng.integers(1, 4, int(rng.integers(40, max_len + 1)))]
            for _ in range(300)]
    seqs.append([1] * max_len)
    capfd.readouterr()
    check(blob, *csr(seqs), sem)
    rk = {r for r, _ in routed_records(capfd.readouterr().err, sem)}
    assert rk == ({1} if sem == EAGER else {0})  # lazy f32 cells need weights <= 255
    check(blob, *csr(seqs + [[1] * (max_len + 1)]), sem)
    assert routed_records(capfd.readouterr().err, sem) == {(0, 1.0)}
