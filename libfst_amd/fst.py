"""Python host mirror of libfst's C ABI for the frozen-compose hot path.

Thin ctypes binding of libfst_amd.so (include/fst.h + include/fst_batch.h).  Names,
argument meaning and error behaviour follow the reference C API
(ontypehq/libfst src/c-api.zig): handles are u64, FST_INVALID_HANDLE signals
failure, n-shortest accepts only n in {0, 1}.  All compose / shortest-path work runs
in the HIP kernels of libfst_amd.so; if the library or a GPU is missing these calls
raise instead of computing anything on the CPU.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# LIBFST_AMD_LIB: an alternate build of the same library (A/B runs of kernel variants).
LIB_PATH = os.environ.get("LIBFST_AMD_LIB") or os.path.join(PKG_DIR, "libfst_amd.so")

FST_NO_STATE = 0xFFFFFFFF
FST_EPSILON = 0
FST_INVALID_HANDLE = 0xFFFFFFFFFFFFFFFF

FST_OK, FST_OOM, FST_INVALID_ARG, FST_INVALID_STATE, FST_IO_ERROR = range(5)
FST_SEM_LAZY, FST_SEM_EAGER = 0, 1
(FST_PATH_OK, FST_PATH_EMPTY, FST_PATH_ERROR_N, FST_PATH_CYCLE, FST_PATH_OVERFLOW,
 FST_PATH_UNSUPPORTED, FST_PATH_OUTPUT_FULL, FST_PATH_INTERNAL) = range(8)

BENCH_AMBIGUOUS, BENCH_EPS_DENSE, BENCH_BRANCHING = 0, 1, 2


class FstArc(C.Structure):
    _fields_ = [("ilabel", C.c_uint32), ("olabel", C.c_uint32), ("weight", C.c_double),
                ("nextstate", C.c_uint32)]


class FstBatchResult(C.Structure):
    _fields_ = [("num_strings", C.c_uint32), ("status", C.POINTER(C.c_int32)),
                ("path_offsets", C.POINTER(C.c_uint64)), ("ilabels", C.POINTER(C.c_uint32)),
                ("olabels", C.POINTER(C.c_uint32)), ("weights", C.POINTER(C.c_double)),
                ("final_weights", C.POINTER(C.c_double)), ("total_arcs", C.c_uint64)]


FST_BATCH_DEVICES = 1


class FstBatchOptions(C.Structure):
    _fields_ = [("device", C.c_int32), ("semantics", C.c_uint32), ("flags", C.c_uint32),
                ("num_shards", C.c_uint32), ("device_mask", C.c_uint64)]


def batch_options(device=-1, semantics=FST_SEM_LAZY, devices=None, shards=0) -> FstBatchOptions:
    """FstBatchOptions; `devices` (a list of HIP ordinals) shards the batch over them
    (FST_BATCH_DEVICES), `shards` > len(devices) runs several shards per device."""
    if devices is None and not shards:
        return FstBatchOptions(device, semantics, 0, 0, 0)
    devs = list(devices) if devices is not None else [max(device, 0)]
    mask = 0
    for d in devs:
        mask |= 1 << int(d)
    return FstBatchOptions(device, semantics, FST_BATCH_DEVICES, int(shards), mask)


class FstDeviceBatch(C.Structure):
    _fields_ = [("status", C.c_void_p), ("path_len", C.c_void_p), ("path_offset", C.c_void_p),
                ("final_weight", C.c_void_p), ("ilabels", C.c_void_p), ("olabels", C.c_void_p),
                ("weights", C.c_void_p), ("arc_capacity", C.c_uint64), ("arc_cursor", C.c_void_p),
                ("work", C.c_void_p)]


class FstLaunchStats(C.Structure):
    _fields_ = [("kernel_ms", C.c_double), ("launches", C.c_uint32), ("engine", C.c_uint32),
                ("grid", C.c_uint32)]


# Every symbol include/fst.h and include/fst_batch.h declare, with its ctypes signature.
_u32, _u64, _f64, _i32, _P = C.c_uint32, C.c_uint64, C.c_double, C.c_int32, C.c_void_p
SIGNATURES = {
    "fst_mutable_new": (_u64, []),
    "fst_mutable_clone": (_u64, [_u64]),
    "fst_mutable_free": (None, [_u64]),
    "fst_mutable_add_state": (_u32, [_u64]),
    "fst_mutable_set_start": (C.c_int, [_u64, _u32]),
    "fst_mutable_set_final": (C.c_int, [_u64, _u32, _f64]),
    "fst_mutable_add_arc": (C.c_int, [_u64, _u32, _u32, _u32, _f64, _u32]),
    "fst_mutable_start": (_u32, [_u64]),
    "fst_mutable_num_states": (_u32, [_u64]),
    "fst_mutable_num_arcs": (_u32, [_u64, _u32]),
    "fst_mutable_final_weight": (_f64, [_u64, _u32]),
    "fst_mutable_get_arcs": (_u32, [_u64, _u32, C.POINTER(FstArc), _u32]),
    "fst_freeze": (_u64, [_u64]),
    "fst_free": (None, [_u64]),
    "fst_start": (_u32, [_u64]),
    "fst_num_states": (_u32, [_u64]),
    "fst_num_arcs": (_u32, [_u64, _u32]),
    "fst_final_weight": (_f64, [_u64, _u32]),
    "fst_get_arcs": (_u32, [_u64, _u32, C.POINTER(FstArc), _u32]),
    "fst_load": (_u64, [C.c_char_p]),
    "fst_save": (C.c_int, [_u64, C.c_char_p]),
    "fst_compose_frozen": (_u64, [_u64, _u64]),
    "fst_compose_frozen_shortest_path": (_u64, [_u64, _u64, _u32]),
    "fst_shortest_path": (_u64, [_u64, _u32]),
    "fst_compile_string": (_u64, [C.c_char_p, _u32]),
    "fst_print_string": (_i32, [_u64, C.c_char_p, _u32]),
    "fst_print_output_string": (_i32, [_u64, C.c_char_p, _u32]),
    "fst_teardown": (None, []),
    "fst_compose_frozen_shortest_path_batch": (
        C.c_int, [_u64, _P, _P, _u32, _u32, C.POINTER(FstBatchOptions), C.POINTER(FstBatchResult)]),
    "fst_batch_result_free": (None, [C.POINTER(FstBatchResult)]),
    "fst_device_compose_shortest_path": (
        C.c_int, [_u64, _P, _P, _u32, _u32, _u32, C.POINTER(FstBatchOptions),
                  C.POINTER(FstDeviceBatch), _P]),
    "fst_device_prepare": (C.c_int, [_u64, _i32]),
    "fst_device_adopt_blob": (_u64, [_P, _u64, _i32, _P]),
    "fst_last_launch_stats": (C.c_int, [C.POINTER(FstLaunchStats)]),
    "fst_bench_transducer": (_u64, [_u32, _u32, _u32]),
    "fst_bench_transducer_wt": (_u64, [_u32, _u32, _u32, _u32]),
    "fst_batch_load": (_u64, [C.c_char_p]),
    "fst_batch_load_bytes": (_u64, [C.c_void_p, C.c_uint64]),
    "fst_weight_type": (C.c_int32, [_u64]),
    "fst_read_text": (_u64, [C.c_char_p]),
    "fst_chain_cost": (_f64, [_u64, _u64]),
    "fst_debug_coalescer_state": (C.c_int32, [C.c_int32, C.POINTER(_u32)]),
    "fst_load_att": (_u64, [C.c_char_p, _u32]),
    "fst_device_project_output": (C.c_int, [C.c_void_p, _u32, C.c_void_p, C.c_void_p, C.c_void_p,
                                            C.POINTER(_u32), C.c_void_p]),
    "fst_pipeline_batch": (C.c_int, [C.c_void_p, _u32, C.c_void_p, C.c_void_p, _u32, _u32,
                                     C.c_void_p, C.c_void_p]),
}

_lib = None


def lib():
    """Load libfst_amd.so (built by __graft_entry__.build()); raise if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it first (python -c 'import __graft_entry__ as g; "
                "g.build()'); libfst_amd has no CPU fallback")
        # One HIP runtime per process: torch ships its own libamdhip64 (same soname
        # libamdhip64.so.7, but torch links it by the bare name), so if this library
        # loaded /opt/rocm's copy first, a later `import torch` would bring a second
        # runtime and one of the two would see no device.  Loading torch first makes
        # our DT_NEEDED resolve to the copy torch already holds.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


class MutableFst:
    """Owning wrapper of an FstMutableHandle (src/c-api.zig:437-503)."""

    def __init__(self, handle=None):
        self.h = lib().fst_mutable_new() if handle is None else handle
        if self.h == FST_INVALID_HANDLE:
            raise RuntimeError("invalid mutable handle")

    def __del__(self):
        if getattr(self, "h", FST_INVALID_HANDLE) != FST_INVALID_HANDLE and _lib is not None:
            _lib.fst_mutable_free(self.h)
            self.h = FST_INVALID_HANDLE

    def add_state(self):
        return lib().fst_mutable_add_state(self.h)

    def set_start(self, s):
        return lib().fst_mutable_set_start(self.h, s)

    def set_final(self, s, w):
        return lib().fst_mutable_set_final(self.h, s, w)

    def add_arc(self, src, il, ol, w, nxt):
        return lib().fst_mutable_add_arc(self.h, src, il, ol, w, nxt)

    @property
    def start(self):
        return lib().fst_mutable_start(self.h)

    @property
    def num_states(self):
        return lib().fst_mutable_num_states(self.h)

    def final_weight(self, s):
        return lib().fst_mutable_final_weight(self.h, s)

    def arcs(self, s):
        n = lib().fst_mutable_num_arcs(self.h, s)
        buf = (FstArc * max(n, 1))()
        m = lib().fst_mutable_get_arcs(self.h, s, buf, n)
        return [(buf[i].ilabel, buf[i].olabel, buf[i].weight, buf[i].nextstate) for i in range(m)]

    def freeze(self) -> "Fst":
        return Fst(lib().fst_freeze(self.h))

    def print_string(self, output_tape=False):
        buf = C.create_string_buffer(1 << 16)
        fn = lib().fst_print_output_string if output_tape else lib().fst_print_string
        n = fn(self.h, buf, len(buf))
        return None if n < 0 else buf.raw[:n]

    def to_lists(self):
        """(start, finals, arcs-per-state) for comparisons in tests."""
        ns = self.num_states
        return (self.start, [self.final_weight(s) for s in range(ns)],
                [self.arcs(s) for s in range(ns)])

    def to_arrays(self):
        """(start, offsets u64[ns + 1], arcs, finals f64[ns]) with `arcs` a numpy record
        array of FstArc {ilabel, olabel, weight, nextstate}: large results (config 1's
        lattice has 10 M arcs) without Python tuples."""
        L, ns = lib(), self.num_states
        cnt = np.fromiter((L.fst_mutable_num_arcs(self.h, s) for s in range(ns)), np.uint64, ns)
        off = np.zeros(ns + 1, np.uint64)
        np.cumsum(cnt, out=off[1:])
        tot = int(off[-1])
        buf = (FstArc * max(tot, 1))()
        base, sz, ptr = C.addressof(buf), C.sizeof(FstArc), C.POINTER(FstArc)
        for s in np.nonzero(cnt)[0]:
            L.fst_mutable_get_arcs(self.h, int(s), C.cast(base + int(off[s]) * sz, ptr), int(cnt[s]))
        dt = np.dtype([("il", "<u4"), ("ol", "<u4"), ("w", "<f8"), ("next", "<u4"), ("pad", "<u4")])
        arcs = np.frombuffer(buf, dtype=dt, count=tot).copy()
        fin = np.fromiter((L.fst_mutable_final_weight(self.h, s) for s in range(ns)), np.float64, ns)
        return self.start, off, arcs, fin

    @staticmethod
    def read_text(path) -> "MutableFst":
        """fst_read_text: OpenFst AT&T text (src/io/text.zig), labels as written."""
        h = lib().fst_read_text(os.fsencode(path))
        if h == FST_INVALID_HANDLE:
            raise ValueError(f"fst_read_text failed: {path}")
        return MutableFst(h)

    @staticmethod
    def compile_string(data: bytes) -> "MutableFst":
        return MutableFst(lib().fst_compile_string(data, len(data)))


class Fst:
    """Owning wrapper of an FstHandle (frozen FST)."""

    def __init__(self, handle):
        if handle == FST_INVALID_HANDLE:
            raise RuntimeError("invalid frozen handle")
        self.h = handle

    def __del__(self):
        if getattr(self, "h", FST_INVALID_HANDLE) != FST_INVALID_HANDLE and _lib is not None:
            _lib.fst_free(self.h)
            self.h = FST_INVALID_HANDLE

    @property
    def start(self):
        return lib().fst_start(self.h)

    @property
    def num_states(self):
        return lib().fst_num_states(self.h)

    def final_weight(self, s):
        return lib().fst_final_weight(self.h, s)

    def arcs(self, s):
        n = lib().fst_num_arcs(self.h, s)
        buf = (FstArc * max(n, 1))()
        m = lib().fst_get_arcs(self.h, s, buf, n)
        return [(buf[i].ilabel, buf[i].olabel, buf[i].weight, buf[i].nextstate) for i in range(m)]

    def save(self, path):
        return lib().fst_save(self.h, path.encode())

    @staticmethod
    def load(path) -> "Fst":
        return Fst(lib().fst_load(path.encode()))

    @staticmethod
    def load_any(path) -> "Fst":
        """Tropical or Log blob (fst_batch_load: weight type from the header)."""
        return Fst(lib().fst_batch_load(path.encode()))

    @staticmethod
    def load_att(path, shift_byte_labels=True) -> "Fst":
        """fst_load_att: AT&T text -> frozen, with att2lfst's +1 byte-label shift."""
        h = lib().fst_load_att(os.fsencode(path), 1 if shift_byte_labels else 0)
        if h == FST_INVALID_HANDLE:
            raise ValueError(f"fst_load_att failed: {path}")
        return Fst(h)

    @staticmethod
    def from_bytes(blob: bytes) -> "Fst":
        """Tropical or Log blob from memory (fst_batch_load_bytes)."""
        buf = C.create_string_buffer(blob, len(blob))
        return Fst(lib().fst_batch_load_bytes(C.cast(buf, C.c_void_p), len(blob)))

    @property
    def weight_type(self):
        return lib().fst_weight_type(self.h)

    @staticmethod
    def bench_transducer(kind, transducer_len, branches, weight_type=0) -> "Fst":
        return Fst(lib().fst_bench_transducer_wt(kind, transducer_len, branches, weight_type))

    def prepare(self, device=-1):
        rc = lib().fst_device_prepare(self.h, device)
        if rc != FST_OK:
            raise RuntimeError(f"fst_device_prepare failed: {rc}")


def compose_frozen_shortest_path(a: MutableFst, b: Fst, n: int = 1):
    """fst_compose_frozen_shortest_path (src/c-api.zig:744-811); None on FST_INVALID_HANDLE."""
    h = lib().fst_compose_frozen_shortest_path(a.h, b.h, n)
    return None if h == FST_INVALID_HANDLE else MutableFst(h)


def compose_frozen(a: MutableFst, b: Fst):
    h = lib().fst_compose_frozen(a.h, b.h)
    return None if h == FST_INVALID_HANDLE else MutableFst(h)


def shortest_path(a: MutableFst, n: int = 1):
    h = lib().fst_shortest_path(a.h, n)
    return None if h == FST_INVALID_HANDLE else MutableFst(h)


@dataclass
class BatchResult:
    status: np.ndarray
    offsets: np.ndarray
    ilabels: np.ndarray
    olabels: np.ndarray
    weights: np.ndarray
    finals: np.ndarray


def compose_frozen_shortest_path_batch(b: Fst, labels, offsets, n: int = 1,
                                       semantics: int = FST_SEM_LAZY, device: int = -1,
                                       devices=None, shards: int = 0) -> BatchResult:
    """Batched 1-best of many chain acceptors against one frozen rhs (fst_batch.h);
    `devices` / `shards`: cost-balanced shards over several GPUs (FST_BATCH_DEVICES)."""
    L = lib()
    labels = np.ascontiguousarray(labels, dtype=np.uint32)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    num = len(offsets) - 1
    opts = batch_options(device, semantics, devices, shards)
    res = FstBatchResult()
    rc = L.fst_compose_frozen_shortest_path_batch(b.h, labels.ctypes.data, offsets.ctypes.data,
                                                  num, n, C.byref(opts), C.byref(res))
    if rc != FST_OK:
        raise RuntimeError(f"fst_compose_frozen_shortest_path_batch failed: {rc}")
    return _take_result(res, num)


def pipeline_batch(stages, labels, offsets, n: int = 1, semantics: int = FST_SEM_LAZY,
                   device: int = -1, devices=None, shards: int = 0) -> BatchResult:
    """Multi-stage batch (tagger -> verbalizer ...): each stage's 1-best output tape is the
    next stage's input, projected on the device (fst_pipeline_batch)."""
    L = lib()
    labels = np.ascontiguousarray(labels, dtype=np.uint32)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    num = len(offsets) - 1
    hs = (C.c_uint64 * len(stages))(*[s.h for s in stages])
    opts = batch_options(device, semantics, devices, shards)
    res = FstBatchResult()
    rc = L.fst_pipeline_batch(hs, len(stages), labels.ctypes.data, offsets.ctypes.data, num, n,
                              C.byref(opts), C.byref(res))
    if rc != FST_OK:
        raise RuntimeError(f"fst_pipeline_batch failed: {rc}")
    return _take_result(res, num)


class _ResultOwner:
    """Owns one FstBatchResult; fst_batch_result_free runs once no array views it."""

    def __init__(self, res):
        self.res = res

    def __del__(self):
        try:
            lib().fst_batch_result_free(C.byref(self.res))
        except Exception:  # interpreter shutdown
            pass


def _take_result(res, num) -> BatchResult:
    """Numpy views of the library's (pinned) result arrays, no copy: they stay valid while
    any of the arrays lives, then go back to the library's pool."""
    tot = int(res.total_arcs)
    owner = _ResultOwner(res)

    def arr(p, cnt, dt, ct):
        if cnt == 0:
            return np.zeros(0, dt)
        buf = (ct * cnt).from_address(C.cast(p, C.c_void_p).value)
        buf._owner = owner  # the view keeps the result alive
        return np.frombuffer(buf, dtype=dt)

    return BatchResult(status=arr(res.status, num, np.int32, C.c_int32),
                       offsets=arr(res.path_offsets, num + 1, np.uint64, C.c_uint64),
                       ilabels=arr(res.ilabels, tot, np.uint32, C.c_uint32),
                       olabels=arr(res.olabels, tot, np.uint32, C.c_uint32),
                       weights=arr(res.weights, tot, np.float64, C.c_double),
                       finals=arr(res.final_weights, num, np.float64, C.c_double))


def coalescer_state(device: int = 0):
    """(leader slots in use, queued calls) of the single-call coalescer on `device`."""
    q = _u32(0)
    return int(lib().fst_debug_coalescer_state(device, C.byref(q))), int(q.value)


def last_launch_stats() -> FstLaunchStats:
    st = FstLaunchStats()
    lib().fst_last_launch_stats(C.byref(st))
    return st
