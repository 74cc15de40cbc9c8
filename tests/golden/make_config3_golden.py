"""Generates tests/golden/config3_T65536.npz: config 3's full-size rhs (epsilon dense,
T=65,536, B=12; bench/optimize-bench.zig:219-248) against chain strings of the config's
length distribution (uniform in [11, 251], seed 0x5EED, :398-401) plus both ends of the
range near the top, with the oracle's lazy 1-best (its full composeShortestPath replay,
src/ops/compose-shortest-path.zig:26-401: 33 M tuples at L=251) and its work counts.

The rhs is not stored (O.gen / fst_bench_transducer rebuild it bit-identically); the
fixture holds the lengths and the expected outputs.  ~1 minute on 8 host threads:

    python tests/golden/make_config3_golden.py
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_ffi as O  # noqa: E402

T, B = 65536, 12


def lengths():
    rng = np.random.default_rng(0x5EED)
    return [151, 251] + [int(x) for x in rng.integers(11, 252, 6)]


def main():
    blob = O.freeze(O.gen("eps_dense", T, B))
    lens = lengths()
    labels = np.ones(sum(lens), np.uint32)
    offsets = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    t = time.time()
    r = O.batch_run(blob, labels, offsets, 0, 1, len(lens))
    print(f"oracle: {len(lens)} strings in {time.time() - t:.1f} s", flush=True)
    arrays = {"lengths": np.asarray(lens, np.uint32), "T": np.uint32(T), "B": np.uint32(B)}
    for fld in ("status", "empty", "offsets", "ilabels", "olabels", "weights", "finals",
                "tuples", "relaxations"):
        arrays[fld] = getattr(r, fld)
    np.savez_compressed(os.path.join(HERE, "config3_T65536.npz"), **arrays)
    print("lengths", lens, "tuples", r.tuples.tolist())


if __name__ == "__main__":
    main()
