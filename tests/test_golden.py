"""Golden fixtures (tests/golden/paths_v1.npz, made by tests/golden/make_golden.py):
the oracle must reproduce them on CPU, and the HIP path must match them bit-exactly."""
import os

import numpy as np
import pytest

import oracle_ffi as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "paths_v1.npz")


def load_cases():
    z = np.load(GOLDEN, allow_pickle=False)
    out = []
    for entry in z["cases"]:
        name, sems = str(entry).split(":")
        for sem in sems.split(","):
            out.append((name, int(sem)))
    return z, out


Z, CASES = load_cases()


def expected(name, sem):
    p = f"{name}/sem{sem}/"
    return {k: Z[p + k] for k in ("status", "empty", "offsets", "ilabels", "olabels", "weights",
                                  "finals")}


@pytest.mark.parametrize("name,sem", CASES)
def test_oracle_reproduces_golden(name, sem):
    blob = Z[f"{name}/blob"].tobytes()
    r = O.batch_run(blob, Z[f"{name}/labels"], Z[f"{name}/offsets"], sem)
    e = expected(name, sem)
    for k in e:
        got = getattr(r, k)
        if got.dtype == np.float64:
            assert np.array_equal(got.view(np.uint64), e[k].view(np.uint64)), k
        else:
            assert np.array_equal(got, e[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("name,sem", CASES)
def test_gpu_matches_golden(name, sem):
    import libfst_amd as F
    from test_gpu_parity import load_blob
    blob = Z[f"{name}/blob"].tobytes()
    e = expected(name, sem)
    got = F.compose_frozen_shortest_path_batch(load_blob(blob), Z[f"{name}/labels"],
                                               Z[f"{name}/offsets"], 1, sem)
    st = np.where(e["status"] == O.OR_ERR_CYCLE, F.FST_PATH_CYCLE,
                  np.where(e["empty"] == 1, F.FST_PATH_EMPTY, F.FST_PATH_OK))
    # every engine answers every golden case: no status may be UNSUPPORTED or skipped
    assert np.array_equal(got.status, st)
    ok = st == F.FST_PATH_OK
    assert np.array_equal(np.diff(got.offsets)[ok], np.diff(e["offsets"])[ok])
    for i in np.nonzero(ok)[0]:
        a, b = int(got.offsets[i]), int(got.offsets[i + 1])
        c, d = int(e["offsets"][i]), int(e["offsets"][i + 1])
        assert np.array_equal(got.ilabels[a:b], e["ilabels"][c:d])
        assert np.array_equal(got.olabels[a:b], e["olabels"][c:d])
        assert np.array_equal(got.weights[a:b].view(np.uint64), e["weights"][c:d].view(np.uint64))
    assert np.array_equal(got.finals[ok].view(np.uint64), e["finals"][ok].view(np.uint64))


def test_oracle_reproduces_config3_fixture_short():
    # tests/golden/config3_T65536.npz (config 3's full-size rhs, made by
    # make_config3_golden.py): the oracle re-derives its shortest string here (L=44,
    # 5.8 M tuples, ~10 s); the GPU suite checks all 8 (tests/test_gpu_fullsize.py)
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "config3_T65536.npz"),
                allow_pickle=False)
    lens = [int(x) for x in z["lengths"]]
    i = int(np.argmin(lens))
    blob = O.freeze(O.gen("eps_dense", int(z["T"]), int(z["B"])))
    L = lens[i]
    r = O.batch_run(blob, np.ones(L, np.uint32), np.array([0, L], np.uint64), 0)
    a, b = int(z["offsets"][i]), int(z["offsets"][i + 1])
    assert int(r.status[0]) == int(z["status"][i]) == 0
    assert np.array_equal(r.ilabels, z["ilabels"][a:b])
    assert np.array_equal(r.olabels, z["olabels"][a:b])
    assert np.array_equal(r.weights.view(np.uint64), z["weights"][a:b].view(np.uint64))
    assert r.finals.view(np.uint64)[0] == z["finals"].view(np.uint64)[i]
    assert int(r.tuples[0]) == int(z["tuples"][i])
