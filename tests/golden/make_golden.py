"""Generates tests/golden/paths_v1.npz: seeded inputs and the oracle's 1-best results.

The fixtures freeze the oracle's answers (which are pinned to the reference's
known-answer tests, see tests/test_oracle_known_answers.py) so that a later change to
either the oracle or the HIP path shows up as a fixture diff.  Re-run only on purpose:

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_ffi as O  # noqa: E402


def random_rhs(rng, ns, na, max_label, eps, wmax=3, frac=False):
    f = O.Fst()
    for _ in range(ns):
        f.add_state(float(rng.integers(0, 3)) if rng.random() < 0.5 else float("inf"))
    f.start = 0
    lo = 0 if eps else 1
    for _ in range(na):
        w = float(rng.integers(0, wmax + 1)) + (float(rng.random()) if frac else 0.0)
        f.add_arc(int(rng.integers(ns)), int(rng.integers(lo, max_label + 1)),
                  int(rng.integers(0, max_label + 1)), w, int(rng.integers(ns)))
    return f


def cases():
    rng = np.random.default_rng(20261015)
    out = []
    amb = O.freeze(O.gen("ambiguous", 512, 12))
    lens = [0, 1, 2, 7, 31, 64, 100]
    seqs = [[1] * L for L in lens] + [[1, 1, 2, 1], [2]]
    out.append(("ambiguous_T512", amb, seqs, (0, 1)))
    br = O.freeze(O.gen("branching_frozen_src", 256, 12))
    seqs = [[(i % 12) + 1 for i in range(L)] for L in (1, 5, 40)]
    seqs += [[int(x) for x in rng.integers(1, 14, 25)] for _ in range(6)]
    out.append(("branching_T256", br, seqs, (0, 1)))
    eps = O.freeze(O.gen("eps_dense", 48, 12))
    seqs = [[1] * L for L in (0, 1, 4, 12, 20)] + [[1, 0, 1], [0, 0]]
    out.append(("eps_dense_T48", eps, seqs, (0,)))
    for k in range(6):
        f = random_rhs(rng, int(rng.integers(2, 30)), int(rng.integers(4, 120)), 4,
                       eps=(k % 2 == 0), frac=(k % 3 == 0))
        seqs = [[int(x) for x in rng.integers(1, 5, int(rng.integers(0, 10)))] for _ in range(24)]
        out.append((f"random_{k}", O.freeze(f), seqs, (0,) if k % 2 == 0 else (0, 1)))
    return out


def main():
    arrays = {}
    names = []
    for name, blob, seqs, sems in cases():
        lens = [len(s) for s in seqs]
        labels = np.concatenate([np.asarray(s, np.uint32) for s in seqs]).astype(np.uint32) \
            if sum(lens) else np.zeros(0, np.uint32)
        offsets = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        arrays[f"{name}/blob"] = np.frombuffer(blob, np.uint8)
        arrays[f"{name}/labels"] = labels
        arrays[f"{name}/offsets"] = offsets
        for sem in sems:
            r = O.batch_run(blob, labels, offsets, sem)
            p = f"{name}/sem{sem}/"
            for fld in ("status", "empty", "offsets", "ilabels", "olabels", "weights", "finals"):
                arrays[p + fld] = getattr(r, fld)
        names.append(f"{name}:{','.join(map(str, sems))}")
    arrays["cases"] = np.array(names)
    np.savez_compressed(os.path.join(HERE, "paths_v1.npz"), **arrays)
    print("wrote", len(names), "cases")


if __name__ == "__main__":
    main()
