"""States with many arcs under the wave-per-string replays (LDS, hashed, dense, band): the
label's arc run is counted by the whole wave (kernels/device_common.hpp
wave_span_by_ilabel) -- one round of 8 chunks up to 512 arcs, a 64-sample narrowing round
first beyond.  Hubs of 65..4000 arcs with duplicate-label runs, epsilon runs and labels
missing from the hub, bit-exact against the oracle for both semantics."""
import math

import numpy as np
import pytest

import oracle_ffi as O
from test_gpu_parity import EAGER, LAZY, check

pytestmark = pytest.mark.gpu


def hub_rhs(rng, hub_arcs, n_labels, leaves=40, eps=7):
    """State 0 is a hub: hub_arcs arcs over n_labels labels (runs of equal labels; some
    labels absent), `eps` epsilon arcs; leaves return to the hub and are final."""
    f = O.Fst()
    f.add_state(0.5)
    for i in range(leaves):
        f.add_state(float(rng.integers(0, 3)) if i % 3 else math.inf)
    f.start = 0
    labels = np.sort(rng.integers(1, n_labels + 1, hub_arcs - eps))
    for il in labels:
        f.add_arc(0, int(il), int(rng.integers(0, 5)), float(rng.integers(0, 4)),
                  int(rng.integers(1, leaves + 1)))
    for _ in range(eps):
        f.add_arc(0, 0, int(rng.integers(0, 5)), float(rng.integers(1, 4)),
                  int(rng.integers(1, leaves + 1)))
    for s in range(1, leaves + 1):
        f.add_arc(s, 0, 0, float(rng.integers(0, 2)), 0)
        for _ in range(int(rng.integers(0, 3))):
            f.add_arc(s, int(rng.integers(1, n_labels + 1)), int(rng.integers(0, 5)),
                      float(rng.integers(0, 3)), int(rng.integers(1, leaves + 1)))
    return f


@pytest.mark.parametrize("sem,route", [(LAZY, "lds"), (LAZY, "dense"), (EAGER, "")])
@pytest.mark.parametrize("hub_arcs,n_labels", [(65, 20), (300, 120), (511, 700), (513, 90),
                                               (1500, 400), (4000, 2500)])
def test_hub_state(sem, route, hub_arcs, n_labels, monkeypatch):
    if route == "dense":  # no LDS replay: the dense replay (HBM index) takes every string
        monkeypatch.setenv("FSTAMD_LAZY_TINY", "0")
    rng = np.random.default_rng(hub_arcs * 7 + n_labels)
    blob = O.freeze(hub_rhs(rng, hub_arcs, n_labels))
    seqs = [[int(x) for x in rng.integers(1, n_labels + 3, int(rng.integers(0, 12)))]
            for _ in range(96)]
    seqs += [[1], [n_labels], [n_labels + 1], []]  # first, last and an absent label
    lens = [len(q) for q in seqs]
    offsets = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    labels = np.concatenate([np.asarray(q, np.uint32) for q in seqs]).astype(np.uint32)
    check(blob, labels, offsets, sem)
