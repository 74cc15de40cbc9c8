"""CPU tests of the C ABI library: it loads, exports every symbol include/*.h declares,
and its host-side logic (handles, MutableFst, freeze / fromBytes / load / save, strings)
matches the reference semantics -- cross-checked against the oracle.  No compute call
is made here (those need a GPU and live in test_gpu_parity.py)."""
import ctypes as C
import math
import os
import re
import struct

import numpy as np
import pytest

import libfst_amd as F
from libfst_amd import fst as FF
import oracle_ffi as O

INCLUDE = os.path.join(os.path.dirname(os.path.dirname(__file__)), "include")


def declared_symbols():
    names = set()
    for h in ("fst.h", "fst_batch.h"):
        text = open(os.path.join(INCLUDE, h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"\b(fst_[a-z0-9_]+)\s*\(", text):
            names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol():
    L = F.lib()
    names = declared_symbols()
    assert len(names) >= 30
    for n in names:
        assert hasattr(L, n), n
        assert n in FF.SIGNATURES, f"{n} missing from the Python mirror"


def build_pair(f: O.Fst):
    m = F.MutableFst()
    for _ in range(f.num_states):
        m.add_state()
    if f.start != O.NO_STATE:
        assert m.set_start(f.start) == 0
    for s, fw in enumerate(f.finals):
        assert m.set_final(s, fw) == 0
    for s, al in enumerate(f.arcs):
        for (il, ol, w, nx) in al:
            assert m.add_arc(s, il, ol, w, nx) == 0
    return m


def test_mutable_errors_and_queries():
    m = F.MutableFst()
    assert m.set_start(0) == FF.FST_INVALID_STATE
    s0 = m.add_state()
    s1 = m.add_state()
    assert (s0, s1) == (0, 1)
    assert m.add_arc(0, 1, 2, 0.5, 5) == FF.FST_INVALID_STATE
    assert m.add_arc(3, 1, 2, 0.5, 1) == FF.FST_INVALID_STATE
    assert m.add_arc(0, 1, 2, 0.5, 1) == 0
    assert m.set_final(1, 1.5) == 0
    assert m.set_start(0) == 0
    assert m.start == 0 and m.num_states == 2
    assert m.arcs(0) == [(1, 2, 0.5, 1)]
    assert m.final_weight(0) == math.inf and m.final_weight(1) == 1.5
    L = F.lib()
    assert L.fst_mutable_add_state(F.FST_INVALID_HANDLE) == F.FST_NO_STATE
    assert L.fst_mutable_set_start(F.FST_INVALID_HANDLE, 0) == FF.FST_INVALID_ARG
    assert L.fst_mutable_final_weight(m.h, 99) == math.inf


def test_stale_handle_cannot_reach_reused_slot():
    # src/c-api.zig:1426-1437
    L = F.lib()
    first = L.fst_mutable_new()
    L.fst_mutable_free(first)
    second = L.fst_mutable_new()
    assert first != second
    assert L.fst_mutable_add_state(first) == F.FST_NO_STATE
    assert L.fst_mutable_add_state(second) == 0
    L.fst_mutable_free(second)


@pytest.mark.parametrize("seed", range(6))
def test_freeze_matches_oracle_blob(seed, tmp_path):
    rng = np.random.default_rng(seed)
    f = O.Fst()
    ns = int(rng.integers(1, 12))
    for _ in range(ns):
        f.add_state(float(rng.integers(0, 3)) if rng.random() < 0.5 else math.inf)
    f.start = 0
    for _ in range(int(rng.integers(0, 40))):
        f.add_arc(int(rng.integers(ns)), int(rng.integers(0, 4)), int(rng.integers(0, 4)),
                  float(rng.integers(0, 3)), int(rng.integers(ns)))
    blob = O.freeze(f)
    m = build_pair(f)
    fz = m.freeze()
    path = str(tmp_path / "x.fst")
    assert fz.save(path) == 0
    assert open(path, "rb").read() == blob           # byte-identical frozen layout
    g = F.Fst.load(path)
    assert g.num_states == ns and g.start == 0
    for s in range(ns):
        assert g.arcs(s) == fz.arcs(s)
        assert g.final_weight(s) == f.finals[s]


def test_load_rejects_invalid_blobs(tmp_path):
    f = O.Fst(); f.add_state(); f.add_state(0.0); f.start = 0
    f.add_arc(0, 1, 1, 0.0, 1); f.add_arc(0, 2, 2, 0.0, 1)
    blob = bytearray(O.freeze(f))
    L = F.lib()
    cases = {}
    b = bytearray(blob); struct.pack_into("<I", b, 0, 0x12345678); cases["magic"] = b
    b = bytearray(blob); struct.pack_into("<H", b, 4, 2); cases["version"] = b
    b = bytearray(blob); b[6] = 1; cases["weight_type"] = b            # C ABI is tropical-only
    b = bytearray(blob); struct.pack_into("<II", b, 24, 1, 2); cases["arc_range"] = b
    b = bytearray(blob); struct.pack_into("<I", b, 24 + 32 + 16, 9); cases["nextstate"] = b
    b = bytearray(blob); struct.pack_into("<I", b, 24 + 32, 3); cases["unsorted"] = b
    cases["truncated"] = blob[:-1]
    for name, bad in cases.items():
        p = str(tmp_path / f"{name}.fst")
        open(p, "wb").write(bytes(bad))
        assert L.fst_load(p.encode()) == F.FST_INVALID_HANDLE, name
    p = str(tmp_path / "ok.fst")
    open(p, "wb").write(bytes(blob))
    h = L.fst_load(p.encode())
    assert h != F.FST_INVALID_HANDLE
    L.fst_free(h)


@pytest.mark.parametrize("s", [b"hello", b"", "中文".encode(), bytes(range(1, 255))])
def test_compile_and_print_strings(s):
    m = F.MutableFst.compile_string(s)
    o = O.compile_string(s)
    assert m.to_lists() == (o.start, o.finals, o.arcs)
    assert m.print_string() == s == O.print_string(o)
    assert m.print_string(output_tape=True) == s


def test_print_string_not_a_chain():
    m = F.MutableFst()
    for _ in range(3):
        m.add_state()
    m.set_start(0)
    m.set_final(2, 0.0)
    m.add_arc(0, 2, 2, 0.0, 1)
    m.add_arc(0, 3, 3, 0.0, 2)
    assert m.print_string() is None


def test_bench_transducers_match_oracle_generators():
    for kind, name, T, B in [(F.BENCH_AMBIGUOUS, "ambiguous", 64, 12),
                             (F.BENCH_EPS_DENSE, "eps_dense", 64, 12),
                             (F.BENCH_BRANCHING, "branching_frozen_src", 64, 5)]:
        fz = F.Fst.bench_transducer(kind, T, B)
        ref = O.gen(name, T, B)
        blob = O.freeze(ref)
        ns = struct.unpack_from("<I", blob, 8)[0]
        assert fz.num_states == ns
        for s in range(ns):
            exp = [(a[0], a[1], a[2], a[3]) for a in sorted(ref.arcs[s], key=lambda a: a)]
            assert fz.arcs(s) == exp
            assert fz.final_weight(s) == ref.finals[s]


def test_compose_entries_validate_handles_without_gpu_work():
    L = F.lib()
    m = F.MutableFst.compile_string(b"ab")
    # invalid handles fail before any device work
    assert L.fst_compose_frozen_shortest_path(m.h, F.FST_INVALID_HANDLE, 1) == F.FST_INVALID_HANDLE
    assert L.fst_compose_frozen_shortest_path(F.FST_INVALID_HANDLE, 123, 1) == F.FST_INVALID_HANDLE
    fz = F.Fst.bench_transducer(F.BENCH_AMBIGUOUS, 8, 4)
    # n == 0 -> empty FST, n not in {0,1} -> invalid (compose-shortest-path.zig:30-33)
    r = F.compose_frozen_shortest_path(m, fz, 0)
    assert r is not None and r.num_states == 0 and r.start == F.FST_NO_STATE
    assert F.compose_frozen_shortest_path(m, fz, 2) is None


def test_log_weight_blobs_load_through_batch_loaders(tmp_path):
    """fst_load stays tropical-only (src/c-api.zig:601); fst_batch_load* take the header's
    weight type (0 or 1) with the same fromBytes validation otherwise."""
    f = O.gen("ambiguous", 16, 12)
    blob_log = O.freeze(f, 1)
    p = str(tmp_path / "log.fst")
    open(p, "wb").write(blob_log)
    L = F.lib()
    assert L.fst_load(p.encode()) == F.FST_INVALID_HANDLE
    g = F.Fst.load_any(p)
    assert g.h != F.FST_INVALID_HANDLE and g.weight_type == 1
    g2 = F.Fst.from_bytes(blob_log)
    assert g2.weight_type == 1 and g2.num_states == g.num_states
    assert F.Fst.from_bytes(O.freeze(f, 0)).weight_type == 0
    bad = bytearray(blob_log)
    bad[6] = 2
    assert L.fst_batch_load_bytes(bytes(bad), len(bad)) == F.FST_INVALID_HANDLE
    # the bench generator frozen as Log: same arcs, header weight type 1
    fz = F.Fst.bench_transducer(F.BENCH_AMBIGUOUS, 16, 12, weight_type=1)
    assert fz.weight_type == 1
    for s in range(fz.num_states):
        assert fz.arcs(s) == g.arcs(s)


def test_batch_result_views_free_once(monkeypatch):
    # the Python mirror's BatchResult arrays view the library's result buffers without a
    # copy, and fst_batch_result_free runs exactly once, after the last view is gone
    import ctypes as C
    import gc
    import libfst_amd.fst as FF

    freed = []

    class FakeLib:
        def fst_batch_result_free(self, ref):
            freed.append(1)

    monkeypatch.setattr(FF, "lib", lambda: FakeLib())
    status = np.array([0, 1, 0], np.int32)
    offs = np.array([0, 2, 2, 3], np.uint64)
    il = np.array([5, 6, 7], np.uint32)
    ol = np.array([8, 9, 10], np.uint32)
    w = np.array([0.5, 1.0, 2.0])
    fin = np.array([0.0, np.inf, 1.5])
    res = FF.FstBatchResult()
    res.num_strings = 3
    res.total_arcs = 3
    res.status = status.ctypes.data_as(C.POINTER(C.c_int32))
    res.path_offsets = offs.ctypes.data_as(C.POINTER(C.c_uint64))
    res.ilabels = il.ctypes.data_as(C.POINTER(C.c_uint32))
    res.olabels = ol.ctypes.data_as(C.POINTER(C.c_uint32))
    res.weights = w.ctypes.data_as(C.POINTER(C.c_double))
    res.final_weights = fin.ctypes.data_as(C.POINTER(C.c_double))
    out = FF._take_result(res, 3)
    assert np.array_equal(out.status, status) and np.array_equal(out.offsets, offs)
    assert np.array_equal(out.ilabels, il) and np.array_equal(out.olabels, ol)
    assert np.array_equal(out.weights, w) and np.array_equal(out.finals, fin)
    il[0] = 42  # a view, not a copy
    assert out.ilabels[0] == 42
    keep = out.weights
    del out
    gc.collect()
    assert freed == []  # one view still lives
    del keep
    gc.collect()
    assert freed == [1]
