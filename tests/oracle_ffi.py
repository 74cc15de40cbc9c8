"""ctypes binding to the CPU oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker / CPU baseline.  The product
package libfst_amd never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "build", "liboracle.so")

NO_STATE = 0xFFFFFFFF
EPS = 0

OR_OK = 0
OR_ERR_UNSUPPORTED_N = 1
OR_ERR_CYCLE = 2
OR_ERR_NAN = 3


class OrArc(C.Structure):
    _fields_ = [("ilabel", C.c_uint32), ("olabel", C.c_uint32), ("weight", C.c_double),
                ("nextstate", C.c_uint32)]


class OrBatchResult(C.Structure):
    _fields_ = [
        ("num_strings", C.c_uint32),
        ("status", C.POINTER(C.c_int32)),
        ("empty", C.POINTER(C.c_uint8)),
        ("offsets", C.POINTER(C.c_uint64)),
        ("ilabels", C.POINTER(C.c_uint32)),
        ("olabels", C.POINTER(C.c_uint32)),
        ("weights", C.POINTER(C.c_double)),
        ("finals", C.POINTER(C.c_double)),
        ("tuples", C.POINTER(C.c_uint64)),
        ("relaxations", C.POINTER(C.c_uint64)),
        ("total_arcs", C.c_uint64),
    ]


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    src = os.path.join(ORACLE_DIR, "fst_oracle.c")
    if not os.path.exists(ORACLE_SO) or (
        os.path.exists(src) and os.path.getmtime(src) > os.path.getmtime(ORACLE_SO)
    ):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    L = C.CDLL(ORACLE_SO)
    P = C.c_void_p
    u32, u64, f64 = C.c_uint32, C.c_uint64, C.c_double
    sig = {
        "or_mfst_new": (P, []),
        "or_mfst_free": (None, [P]),
        "or_mfst_add_state": (u32, [P]),
        "or_mfst_set_start": (None, [P, u32]),
        "or_mfst_set_final": (None, [P, u32, f64]),
        "or_mfst_add_arc": (C.c_int, [P, u32, u32, u32, f64, u32]),
        "or_mfst_start": (u32, [P]),
        "or_mfst_num_states": (u32, [P]),
        "or_mfst_num_arcs": (u32, [P, u32]),
        "or_mfst_total_arcs": (u64, [P]),
        "or_mfst_final": (f64, [P, u32]),
        "or_mfst_get_arc": (C.c_int, [P, u32, u32, C.POINTER(OrArc)]),
        "or_mfst_export": (None, [P, P, P, P]),
        "or_compile_string": (P, [C.c_char_p, u32]),
        "or_compile_string_transducer": (P, [C.c_char_p, u32, C.c_char_p, u32]),
        "or_print_string": (C.c_int32, [P, C.c_int, C.c_char_p, u32]),
        "or_freeze": (P, [P, C.c_uint8, C.POINTER(C.c_size_t)]),
        "or_blob_free": (None, [P]),
        "or_validate": (C.c_int, [C.c_char_p, C.c_size_t, C.c_uint8]),
        "or_arcs_by_ilabel": (None, [C.c_char_p, u32, u32, C.POINTER(u32), C.POINTER(u32)]),
        "or_find_arc": (C.c_int, [C.c_char_p, u32, u32, C.POINTER(OrArc)]),
        "or_compose": (C.c_int, [P, P, C.c_char_p, C.POINTER(P), C.POINTER(u64)]),
        "or_shortest_path": (C.c_int, [P, u32, C.POINTER(P), C.POINTER(u64)]),
        "or_compose_shortest_path": (C.c_int, [P, P, C.c_char_p, u32, C.POINTER(P), C.POINTER(u64)]),
        "or_gen_linear_acceptor": (P, [u32, u32]),
        "or_gen_repeat_acceptor": (P, [u32, u32]),
        "or_gen_branching_frozen_src": (P, [u32, u32]),
        "or_gen_eps_dense": (P, [u32, u32]),
        "or_gen_ambiguous": (P, [u32, u32]),
        "or_batch_run": (C.POINTER(OrBatchResult), [C.c_char_p, P, P, u32, C.c_int, u32, C.c_int]),
        "or_batch_result_free": (None, [C.POINTER(OrBatchResult)]),
        "or_batch_time": (f64, [C.c_char_p, P, P, u32, C.c_int, C.c_int, C.POINTER(u64)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


@dataclass
class Fst:
    """Plain-Python FST used to build oracle inputs and compare results."""

    start: int = NO_STATE
    finals: list = field(default_factory=list)          # per state, inf = non-final
    arcs: list = field(default_factory=list)            # per state: list of (il, ol, w, next)

    def add_state(self, final=float("inf")):
        self.finals.append(final)
        self.arcs.append([])
        return len(self.finals) - 1

    def add_arc(self, s, il, ol, w, nxt):
        self.arcs[s].append((il, ol, float(w), nxt))

    @property
    def num_states(self):
        return len(self.finals)

    def to_oracle(self):
        L = lib()
        m = L.or_mfst_new()
        for f in self.finals:
            s = L.or_mfst_add_state(m)
            L.or_mfst_set_final(m, s, f)
        if self.start != NO_STATE:
            L.or_mfst_set_start(m, self.start)
        for s, al in enumerate(self.arcs):
            for (il, ol, w, nx) in al:
                L.or_mfst_add_arc(m, s, il, ol, w, nx)
        return m

    @staticmethod
    def from_oracle(m, free=True):
        L = lib()
        f = Fst()
        n = L.or_mfst_num_states(m)
        for s in range(n):
            f.add_state(L.or_mfst_final(m, s))
            a = OrArc()
            for i in range(L.or_mfst_num_arcs(m, s)):
                L.or_mfst_get_arc(m, s, i, C.byref(a))
                f.add_arc(s, a.ilabel, a.olabel, a.weight, a.nextstate)
        f.start = L.or_mfst_start(m)
        if free:
            L.or_mfst_free(m)
        return f


def freeze(fst: Fst, weight_type: int = 0) -> bytes:
    """Fst.fromMutable (src/fst.zig:160-224) -> blob bytes."""
    L = lib()
    m = fst.to_oracle()
    n = C.c_size_t()
    p = L.or_freeze(m, weight_type, C.byref(n))
    blob = C.string_at(p, n.value)
    L.or_blob_free(p)
    L.or_mfst_free(m)
    return blob


def gen(name: str, *args) -> Fst:
    L = lib()
    return Fst.from_oracle(getattr(L, "or_gen_" + name)(*args))


def compose(a: Fst, b, stats=False):
    """compose(a, b); b is an Fst (mutable rhs, scan path) or bytes (frozen)."""
    L = lib()
    ma = a.to_oracle()
    mb = b.to_oracle() if isinstance(b, Fst) else None
    out = C.c_void_p()
    st = (C.c_uint64 * 2)()
    rc = L.or_compose(ma, mb, b if isinstance(b, bytes) else None, C.byref(out), st)
    L.or_mfst_free(ma)
    if mb:
        L.or_mfst_free(mb)
    res = Fst.from_oracle(out.value) if rc == OR_OK else None
    return (rc, res, (st[0], st[1])) if stats else (rc, res)


# or_arc / FstArc as a numpy record (24 B: il u32, ol u32, w f64, next u32, pad)
ARC_DTYPE = np.dtype([("il", "<u4"), ("ol", "<u4"), ("w", "<f8"), ("next", "<u4"),
                      ("pad", "<u4")])


@dataclass
class Csr:
    """A whole FST as arrays (large lattices: config 1 has 10 M arcs)."""
    start: int
    off: np.ndarray      # u64 [ns + 1]
    arcs: np.ndarray     # ARC_DTYPE [total]
    finals: np.ndarray   # f64 [ns]


def export_csr(m, free=True) -> Csr:
    L = lib()
    ns = L.or_mfst_num_states(m)
    tot = L.or_mfst_total_arcs(m)
    off = np.zeros(ns + 1, np.uint64)
    arcs = np.zeros(max(tot, 1), ARC_DTYPE)
    fin = np.zeros(max(ns, 1), np.float64)
    L.or_mfst_export(m, off.ctypes.data, arcs.ctypes.data, fin.ctypes.data)
    c = Csr(L.or_mfst_start(m), off, arcs[:tot], fin[:ns])
    if free:
        L.or_mfst_free(m)
    return c


def compose_csr(a: Fst, blob: bytes):
    """compose(a, frozen blob) with the result as arrays: (rc, Csr or None)."""
    L = lib()
    ma = a.to_oracle()
    out = C.c_void_p()
    st = (C.c_uint64 * 2)()
    rc = L.or_compose(ma, None, blob, C.byref(out), st)
    L.or_mfst_free(ma)
    return rc, (export_csr(out.value) if rc == OR_OK else None)


def shortest_path(a: Fst, n: int = 1, stats=False):
    L = lib()
    ma = a.to_oracle()
    out = C.c_void_p()
    st = (C.c_uint64 * 2)()
    rc = L.or_shortest_path(ma, n, C.byref(out), st)
    L.or_mfst_free(ma)
    res = Fst.from_oracle(out.value) if rc == OR_OK else None
    return (rc, res, (st[0], st[1])) if stats else (rc, res)


def compose_shortest_path(a: Fst, b, n: int = 1, stats=False):
    L = lib()
    ma = a.to_oracle()
    mb = b.to_oracle() if isinstance(b, Fst) else None
    out = C.c_void_p()
    st = (C.c_uint64 * 2)()
    rc = L.or_compose_shortest_path(ma, mb, b if isinstance(b, bytes) else None, n, C.byref(out), st)
    L.or_mfst_free(ma)
    if mb:
        L.or_mfst_free(mb)
    res = Fst.from_oracle(out.value) if rc == OR_OK else None
    return (rc, res, (st[0], st[1])) if stats else (rc, res)


def compile_string(s: bytes) -> Fst:
    L = lib()
    return Fst.from_oracle(L.or_compile_string(s, len(s)))


def compile_string_transducer(i: bytes, o: bytes) -> Fst:
    L = lib()
    return Fst.from_oracle(L.or_compile_string_transducer(i, len(i), o, len(o)))


def print_string(f: Fst, tape: int = 0):
    L = lib()
    m = f.to_oracle()
    buf = C.create_string_buffer(1 << 16)
    n = L.or_print_string(m, tape, buf, len(buf))
    L.or_mfst_free(m)
    return None if n < 0 else buf.raw[:n]


@dataclass
class BatchResult:
    status: np.ndarray
    empty: np.ndarray
    offsets: np.ndarray
    ilabels: np.ndarray
    olabels: np.ndarray
    weights: np.ndarray
    finals: np.ndarray
    tuples: np.ndarray
    relaxations: np.ndarray


def batch_run(blob: bytes, labels: np.ndarray, offsets: np.ndarray, semantics: int, n: int = 1,
              threads: int = 1) -> BatchResult:
    """semantics 0 = lazy composeShortestPath, 1 = eager shortestPath(compose())."""
    L = lib()
    labels = np.ascontiguousarray(labels, dtype=np.uint32)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    ns = len(offsets) - 1
    r = L.or_batch_run(blob, labels.ctypes.data, offsets.ctypes.data, ns, semantics, n, threads)
    R = r.contents
    tot = int(R.total_arcs)

    def arr(p, cnt, dt):
        return np.ctypeslib.as_array(p, shape=(max(cnt, 1),))[:cnt].astype(dt, copy=True)

    out = BatchResult(
        status=arr(R.status, ns, np.int32), empty=arr(R.empty, ns, np.uint8),
        offsets=arr(R.offsets, ns + 1, np.uint64), ilabels=arr(R.ilabels, tot, np.uint32),
        olabels=arr(R.olabels, tot, np.uint32), weights=arr(R.weights, tot, np.float64),
        finals=arr(R.finals, ns, np.float64), tuples=arr(R.tuples, ns, np.uint64),
        relaxations=arr(R.relaxations, ns, np.uint64))
    L.or_batch_result_free(r)
    return out


def batch_time(blob: bytes, labels, offsets, semantics: int, threads: int):
    L = lib()
    labels = np.ascontiguousarray(labels, dtype=np.uint32)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    ck = C.c_uint64()
    secs = L.or_batch_time(blob, labels.ctypes.data, offsets.ctypes.data, len(offsets) - 1,
                           semantics, threads, C.byref(ck))
    return secs, ck.value


def read_att(text: str) -> Fst:
    """AT&T text reader, restating src/io/text.zig:20-110 (first src = start)."""
    f = Fst()
    start_set = False

    def ensure(s):
        while f.num_states <= s:
            f.add_state()

    def parse_w(s):
        if s in ("inf", "Infinity"):
            return float("inf")
        return float(s)

    def parse_u32(s):
        if not s.isdigit():
            raise ValueError(s)
        v = int(s)
        if v > 0xFFFFFFFF:
            raise ValueError(s)
        return v

    for raw in text.split("\n"):
        line = raw.strip("\r \t")
        if not line:
            continue
        fields = line.split()
        src = parse_u32(fields[0])
        ensure(src)
        if not start_set:
            f.start = src
            start_set = True
        if len(fields) == 1:
            f.finals[src] = 0.0
            continue
        try:
            dest = parse_u32(fields[1])
        except ValueError:
            f.finals[src] = parse_w(fields[1])
            continue
        if len(fields) == 2:
            try:
                f.finals[src] = parse_w(fields[1])
            except ValueError:
                ensure(dest)
                f.add_arc(src, 0, 0, 0.0, dest)
            continue
        ensure(dest)
        il = parse_u32(fields[2])
        ol, w = il, 0.0
        if len(fields) >= 4:
            try:
                ol = parse_u32(fields[3])
            except ValueError:
                w = parse_w(fields[3])
                f.add_arc(src, il, il, w, dest)
                continue
            if len(fields) >= 5:
                w = parse_w(fields[4])
        f.add_arc(src, il, ol, w, dest)
    return f


def chain(f: Fst):
    """A result chain -> (ilabels, olabels, weights, final) or None for empty."""
    if f.start == NO_STATE:
        return None
    il, ol, w = [], [], []
    s = f.start
    for _ in range(f.num_states):
        if not f.arcs[s]:
            break
        a = f.arcs[s][0]
        il.append(a[0]); ol.append(a[1]); w.append(a[2])
        s = a[3]
    return il, ol, w, f.finals[s]
