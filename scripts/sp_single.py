"""fst_compose_frozen + fst_shortest_path on config 1's lattice (one 1^96 string vs the
eps-dense T=4096 rhs: 781,313 states, 10.06 M arcs), GPU vs the CPU port (one thread).

usage: python scripts/sp_single.py
"""
import ctypes as C
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import libfst_amd as F  # noqa: E402
import oracle_ffi as O  # noqa: E402  (CPU baseline only)


def main():
    T, B, L = 4096, 12, 96
    fz = F.Fst.bench_transducer(F.BENCH_EPS_DENSE, T, B)
    lhs = F.MutableFst.compile_string(b"\x00" * L)
    lat = F.compose_frozen(lhs, fz)
    F.shortest_path(lat, 1)  # warm
    t0 = time.perf_counter()
    sp = F.shortest_path(lat, 1)
    wall = time.perf_counter() - t0
    st = F.last_launch_stats()
    # CPU: the port's compose then shortestPath, timed on the shortestPath only
    blob = O.freeze(O.gen("eps_dense", T, B))
    chain = O.Fst()
    for _ in range(L + 1):
        chain.add_state()
    chain.start = 0
    chain.finals[L] = 0.0
    for i in range(L):
        chain.add_arc(i, 1, 1, 0.0, i + 1)
    Lb = O.lib()
    ma = chain.to_oracle()
    res = C.c_void_p()
    st2 = (C.c_uint64 * 2)()
    assert Lb.or_compose(ma, None, blob, C.byref(res), st2) == O.OR_OK
    out = C.c_void_p()
    st3 = (C.c_uint64 * 2)()
    t0 = time.perf_counter()
    rc = Lb.or_shortest_path(res, 1, C.byref(out), st3)
    cpu = time.perf_counter() - t0
    assert rc == O.OR_OK
    print(json.dumps({"workload": "fst_shortest_path on config 1's lattice", "states": lat.num_states,
                      "gpu_call_ms": wall * 1e3, "gpu_kernel_ms": st.kernel_ms,
                      "path_states": sp.num_states, "cpu_ms": cpu * 1e3,
                      "cpu_path_states": int(st3[0]), "cpu_kind": "port, 1 thread"}))
    Lb.or_mfst_free(ma)
    Lb.or_mfst_free(res)
    Lb.or_mfst_free(out)


if __name__ == "__main__":
    main()
