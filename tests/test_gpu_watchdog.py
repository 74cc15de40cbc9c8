"""GPU: the per-string watchdog and the arena-exhaustion path.

* The wall-clock watchdog (FSTAMD_WATCHDOG_MS) bounds each STRING, not the launch: a
  batch whose kernel runs several times longer than the limit must still finish every
  string, bit-exact against the oracle, as long as each string alone is well inside it.
* A string whose path outgrows every arena growth step reports FST_PATH_OUTPUT_FULL
  (batch and pipeline entries), never a crash (FSTAMD_ARENA_ARCS shrinks the first arena
  so a 2,000-arc path exhausts the six growth attempts: 1, 4, ..., 1,024 arcs).
"""
import numpy as np
import pytest

import libfst_amd as F
import oracle_ffi as O
from test_gpu_parity import bits, csr, expected_status

pytestmark = pytest.mark.gpu

EAGER, LAZY = F.FST_SEM_EAGER, F.FST_SEM_LAZY


def _distinct_strings():
    return [[1] * 64, [1] * 33, [1] * 64, [1] * 10 + [2] + [1] * 5, [1] * 57, [], [1]]


def _check_cycled(rhs_blob, uniq, reps, got, sem):
    """got = batch over `uniq` cycled `reps` times; compare every string with the oracle."""
    labels, offsets = csr(uniq)
    ref = O.batch_run(rhs_blob, labels, offsets, 0 if sem == LAZY else 1, 1)
    exp = expected_status(ref)
    u = len(uniq)
    n = u * reps
    assert len(got.status) == n
    st = got.status.reshape(reps, u)
    assert np.array_equal(st, np.broadcast_to(exp, (reps, u))), np.unique(got.status,
                                                                        return_counts=True)
    lens = np.diff(got.offsets.astype(np.int64)).reshape(reps, u)
    for j in range(u):
        if exp[j] != F.FST_PATH_OK:
            continue
        b0, b1 = int(ref.offsets[j]), int(ref.offsets[j + 1])
        P = b1 - b0
        assert np.all(lens[:, j] == P)
        idx = (np.arange(reps) * u + j)
        starts = got.offsets[idx].astype(np.int64)
        take = (starts[:, None] + np.arange(P)[None, :]).ravel()
        assert np.array_equal(got.ilabels[take].reshape(reps, P),
                              np.broadcast_to(ref.ilabels[b0:b1], (reps, P)))
        assert np.array_equal(got.olabels[take].reshape(reps, P),
                              np.broadcast_to(ref.olabels[b0:b1], (reps, P)))
        assert np.array_equal(bits(got.weights[take]).reshape(reps, P),
                              np.broadcast_to(bits(ref.weights[b0:b1]), (reps, P)))
        assert np.all(bits(got.finals[idx]) == bits(ref.finals[j:j + 1])[0])


@pytest.mark.parametrize("sem,reps", [(EAGER, 150000), (LAZY, 60000)])
def test_watchdog_is_per_string(sem, reps, monkeypatch):
    blob = O.freeze(O.gen("ambiguous", 4096, 12))
    rhs = F.Fst.from_bytes(blob)
    uniq = _distinct_strings()
    labels, offsets = csr(uniq * reps)
    # calibrate: the whole launch without an override (the first call also initialises
    # the engine's workspaces, so time the second)
    for _ in range(2):
        F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem)
    full_ms = F.last_launch_stats().kernel_ms
    wd_ms = int(full_ms / 3)
    # each string must be far inside the limit (~0.3 ms per string in either pull tier);
    # otherwise this box is too fast for the batch and the test proves nothing
    floor = 3
    assert wd_ms >= floor, f"launch {full_ms:.1f} ms too short to exercise the watchdog"
    monkeypatch.setenv("FSTAMD_WATCHDOG_MS", str(wd_ms))
    got = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem)
    ms = F.last_launch_stats().kernel_ms
    assert ms > wd_ms, (ms, wd_ms)  # the launch outlived the limit...
    _check_cycled(blob, uniq, reps, got, sem)  # ...and still finished every string


def _long_eps_rhs(n_eps):
    """0 -1:1-> 1 -ε:5-> 2 -ε:5-> ... -> n_eps+1 (final); 0 -2:2-> final sink."""
    f = O.Fst()
    for s in range(n_eps + 3):
        f.add_state(0.0 if s in (n_eps + 1, n_eps + 2) else float("inf"))
    f.start = 0
    f.add_arc(0, 1, 1, 0.0, 1)
    f.add_arc(0, 2, 2, 0.5, n_eps + 2)
    for s in range(1, n_eps + 1):
        f.add_arc(s, 0, 5, 0.25, s + 1)
    f.add_arc(n_eps + 2, 2, 2, 0.0, n_eps + 2)
    return f


@pytest.mark.parametrize("sem", [LAZY, EAGER])
def test_output_full_after_arena_growth(sem, monkeypatch):
    blob = O.freeze(_long_eps_rhs(2000))
    rhs = F.Fst.from_bytes(blob)
    seqs = [[1], [2], [2, 2, 2]]
    labels, offsets = csr(seqs)
    ref = O.batch_run(blob, labels, offsets, 0 if sem == LAZY else 1, 1)
    exp = expected_status(ref)
    assert exp[0] == F.FST_PATH_OK and int(ref.offsets[1] - ref.offsets[0]) == 2001
    # without the override the arena grows to fit
    got = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem)
    assert np.array_equal(got.status, exp)
    monkeypatch.setenv("FSTAMD_ARENA_ARCS", "1")  # 1, 4, ..., 1,024 arcs: 2,001 never fit
    got = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem)
    assert got.status[0] == F.FST_PATH_OUTPUT_FULL
    for i in range(1, len(seqs)):  # short paths: OK and exact, or crowded out of the arena
        assert got.status[i] in (exp[i], F.FST_PATH_OUTPUT_FULL)
        if got.status[i] == F.FST_PATH_OK:
            a0, a1 = int(got.offsets[i]), int(got.offsets[i + 1])
            b0, b1 = int(ref.offsets[i]), int(ref.offsets[i + 1])
            assert np.array_equal(got.olabels[a0:a1], ref.olabels[b0:b1])
            assert np.array_equal(bits(got.weights[a0:a1]), bits(ref.weights[b0:b1]))
    # the pipeline keeps the device outputs of an exhausted stage: statuses, no crash
    got = F.pipeline_batch([rhs, rhs], labels, offsets, 1, sem)
    assert got.status[0] == F.FST_PATH_OUTPUT_FULL
