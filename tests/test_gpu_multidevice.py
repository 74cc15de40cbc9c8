"""Multi-GPU inside the library (FST_BATCH_DEVICES) and across processes, on a
one-GPU box: N logical shards on one device, gathered, must equal the one-shard run and
the oracle bit for bit.

* fst_compose_frozen_shortest_path_batch / fst_pipeline_batch with num_shards 2..7 on
  device 0 (each shard its own host thread, engine and stream);
* the shard plan is balanced by cost, not count (FSTAMD_SHARD_LOG);
* a device mask naming a device the process cannot see is an FST_INVALID_ARG;
* under HIP_VISIBLE_DEVICES=0 the mask {0} runs;
* two processes (gloo for the control plane) share cuda:0, each composes its
  cost-balanced shard (libfst_amd.dist.cost_shard_range) and rank 0 gathers.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import libfst_amd as F
import oracle_ffi as O
from test_gpu_configs import oracle_fst, oracle_pipeline
from test_gpu_parity import EAGER, LAZY, bits, csr, expected_status, load_blob

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def same_result(a, b):
    assert np.array_equal(a.status, b.status)
    assert np.array_equal(a.offsets, b.offsets)
    assert np.array_equal(a.ilabels, b.ilabels)
    assert np.array_equal(a.olabels, b.olabels)
    assert np.array_equal(bits(a.weights), bits(b.weights))
    ok = a.status == F.FST_PATH_OK
    assert np.array_equal(bits(a.finals[ok]), bits(b.finals[ok]))


def check_vs_oracle(got, ref):
    exp = expected_status(ref)
    assert np.array_equal(got.status, exp)
    ok = exp == F.FST_PATH_OK
    assert np.array_equal(np.diff(got.offsets)[ok], np.diff(ref.offsets)[ok])
    for i in np.nonzero(ok)[0]:
        a0, a1 = int(got.offsets[i]), int(got.offsets[i + 1])
        b0, b1 = int(ref.offsets[i]), int(ref.offsets[i + 1])
        assert np.array_equal(got.olabels[a0:a1], ref.olabels[b0:b1]), i
        assert np.array_equal(bits(got.weights[a0:a1]), bits(ref.weights[b0:b1])), i


@pytest.mark.parametrize("sem", [EAGER, LAZY])
@pytest.mark.parametrize("shards", [2, 3, 7])
def test_fake_multi_gpu_batch(sem, shards):
    blob = O.freeze(O.gen("ambiguous", 1024, 12))
    rhs = load_blob(blob)
    rng = np.random.default_rng(90 + shards)
    seqs = []
    for _ in range(700):
        L = int(rng.integers(0, 97))
        s = [1] * L
        if L and rng.random() < 0.1:
            s[int(rng.integers(L))] = 2
        seqs.append(s)
    labels, offsets = csr(seqs)
    one = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem)
    many = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem, devices=[0],
                                                shards=shards)
    same_result(many, one)
    check_vs_oracle(many, O.batch_run(blob, labels, offsets, 0 if sem == LAZY else 1, 1, 8))


def test_fake_multi_gpu_eps_dense_mixed_lengths():
    blob = O.freeze(O.gen("eps_dense", 256, 12))
    rhs = load_blob(blob)
    rng = np.random.default_rng(0x5EED)
    seqs = [[1] * int(L) for L in rng.integers(11, 252, 24)]
    labels, offsets = csr(seqs)
    got = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, LAZY, devices=[0],
                                               shards=4)
    check_vs_oracle(got, O.batch_run(blob, labels, offsets, 0, 1, 8))


@pytest.mark.parametrize("sem", [LAZY, EAGER])
def test_fake_multi_gpu_pipeline(sem):
    from libfst_amd import synthetic as SY
    tag, verb = SY.tagger(), SY.verbalizer()
    blobs = [O.freeze(oracle_fst(tag)), O.freeze(oracle_fst(verb))]
    stages = [F.Fst.from_bytes(b) for b in blobs]
    texts = SY.utterances(np.random.default_rng(5), 400) + ["", "7", "call 911"]
    labels, offsets = SY.to_labels(texts)
    one = F.pipeline_batch(stages, labels, offsets, 1, sem)
    many = F.pipeline_batch(stages, labels, offsets, 1, sem, devices=[0], shards=3)
    same_result(many, one)
    ref, exp = oracle_pipeline(blobs, labels, offsets, sem)
    assert np.array_equal(many.status, exp)


def run_py(code, env=None):
    e = dict(os.environ)
    e.update(env or {})
    e["PYTHONPATH"] = os.pathsep.join([os.path.dirname(HERE), HERE, e.get("PYTHONPATH", "")])
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                          timeout=180, env=e)


def test_shard_plan_balanced_by_cost():
    # lengths 11..251 against an epsilon rhs: cost ~ L, so the long strings' shard holds
    # fewer strings (T = 256 >= 251: every string has a path)
    code = r"""
import numpy as np, libfst_amd as F
rhs = F.Fst.bench_transducer(F.BENCH_EPS_DENSE, 256, 12)
lens = [11] * 60 + [251] * 6
lab = np.ones(sum(lens), np.uint32); off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
r = F.compose_frozen_shortest_path_batch(rhs, lab, off, 1, F.FST_SEM_LAZY, devices=[0], shards=2)
assert (r.status == F.FST_PATH_OK).all()
"""
    r = run_py(code, {"FSTAMD_SHARD_LOG": "1"})
    assert r.returncode == 0, r.stderr[-2000:]
    plan = [ln.split() for ln in r.stderr.splitlines() if "[libfst_amd shard]" in ln]
    assert len(plan) == 2
    spans = [tuple(int(x) for x in p[6].split("..")) for p in plan]
    costs = [float(p[8]) for p in plan]
    assert spans[0][0] == 0 and spans[0][1] == spans[1][0] and spans[1][1] == 66
    assert spans[0][1] - spans[0][0] > 2 * (spans[1][1] - spans[1][0])  # by cost, not count
    assert max(costs) / min(costs) < 1.5


def test_device_mask_validation():
    rhs = F.Fst.bench_transducer(F.BENCH_AMBIGUOUS, 64, 12)
    labels, offsets = csr([[1] * 5])
    with pytest.raises(RuntimeError):
        F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, LAZY, devices=[63])
    code = r"""
import numpy as np, libfst_amd as F
rhs = F.Fst.bench_transducer(F.BENCH_AMBIGUOUS, 64, 12)
lab = np.ones(10, np.uint32); off = np.array([0, 5, 10], np.uint64)
r = F.compose_frozen_shortest_path_batch(rhs, lab, off, 1, F.FST_SEM_EAGER, devices=[0], shards=2)
assert (r.status == F.FST_PATH_OK).all() and int(r.offsets[-1]) == 10
try:
    F.compose_frozen_shortest_path_batch(rhs, lab, off, 1, F.FST_SEM_EAGER, devices=[1])
    raise SystemExit("device 1 should be invisible")
except RuntimeError:
    pass
print("ok")
"""
    r = run_py(code, {"HIP_VISIBLE_DEVICES": "0"})
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_processes_one_gpu_shard_and_gather(tmp_path):
    # the multi-process path of bench.py / SURVEY 8(e) with a real compose per rank: each
    # rank takes its cost-balanced shard on cuda:0, rank 0 gathers (gloo) and saves
    world, port = 2, _free_port()
    out = str(tmp_path / "gathered.npz")
    worker = r"""
import os, sys, numpy as np, torch, torch.distributed as dist
import libfst_amd as F
from libfst_amd import dist as D
rank, world = int(sys.argv[1]), int(sys.argv[2])
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:" + sys.argv[3], rank=rank,
                        world_size=world)
torch.cuda.set_device(0)
rhs = F.Fst.bench_transducer(F.BENCH_EPS_DENSE, 128, 12)
rng = np.random.default_rng(0x5EED)
lens = rng.integers(11, 252, 40)
b, e = D.cost_shard_range(lens, rhs, rank, world)
mine = lens[b:e]
lab = np.ones(int(mine.sum()), np.uint32)
off = np.concatenate([[0], np.cumsum(mine)]).astype(np.uint64)
r = F.compose_frozen_shortest_path_batch(rhs, lab, off, 1, F.FST_SEM_LAZY)
part = (b, e, r.status.copy(), np.diff(r.offsets).copy(), r.ilabels.copy(), r.olabels.copy(),
        r.weights.copy(), r.finals.copy())
parts = [None] * world
dist.all_gather_object(parts, part)
if rank == 0:
    parts.sort(key=lambda p: p[0])
    assert parts[0][0] == 0 and parts[-1][1] == len(lens)
    assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
    np.savez(sys.argv[4], lens=lens, status=np.concatenate([p[2] for p in parts]),
             plen=np.concatenate([p[3] for p in parts]),
             il=np.concatenate([p[4] for p in parts]), ol=np.concatenate([p[5] for p in parts]),
             w=np.concatenate([p[6] for p in parts]), fin=np.concatenate([p[7] for p in parts]))
dist.barrier()
dist.destroy_process_group()
"""
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([os.path.dirname(HERE), env.get("PYTHONPATH", "")])
    procs = [subprocess.Popen([sys.executable, "-c", worker, str(r), str(world), str(port), out],
                              env=env, stderr=subprocess.PIPE, text=True) for r in range(world)]
    for p in procs:
        _, err = p.communicate(timeout=240)
        assert p.returncode == 0, err[-2000:]
    g = np.load(out)
    lens = g["lens"]
    blob = O.freeze(O.gen("eps_dense", 128, 12))
    labels = np.ones(int(lens.sum()), np.uint32)
    offsets = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    ref = O.batch_run(blob, labels, offsets, 0, 1, 8)
    assert np.array_equal(g["status"], expected_status(ref))
    assert np.array_equal(g["plen"], np.diff(ref.offsets))
    assert np.array_equal(g["il"], ref.ilabels) and np.array_equal(g["ol"], ref.olabels)
    assert np.array_equal(bits(g["w"]), bits(ref.weights))
    ok = g["status"] == F.FST_PATH_OK   # (strings longer than T have no path: EMPTY)
    assert ok.sum() > 0 and (~ok).sum() > 0
    assert np.array_equal(bits(g["fin"][ok]), bits(ref.finals[ok]))


@pytest.mark.parametrize("mode", ["strong", "weak"])
def test_bench_two_ranks_one_gpu(mode):
    # bench.py's multi-process path in both scaling modes (the driver's 1/2/4/8-GPU runs
    # use RCCL, one GPU per rank): two ranks share cuda:0 over gloo here, each times its
    # shard and checks a sample against the oracle; rank 0 prints the one JSON line
    # strong: under an explicit torchrun (the driver's form); weak: `bench.py --gpus 2`
    # alone, which starts its two ranks itself (a child torchrun)
    repo = os.path.dirname(HERE)
    port = _free_port()
    launcher = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                "--nproc-per-node=2", "--master-addr", "127.0.0.1", "--master-port", str(port)]
    cmd = (launcher if mode == "strong" else [sys.executable]) + [
           os.path.join(repo, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--backend", "gloo", "--scaling", mode, "--global-batch", "8192", "--batch", "4096",
           "--no-cpu", "--no-varied", "--lazy-batch", "0", "--no-f64"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["scaling"] == mode
    assert line["config"]["global_batch"] == 8192
    assert line["config"]["strings_per_gpu"] == 4096
    assert line["checked_vs_oracle"] == 256 and line["value"] > 0


@pytest.mark.parametrize("sem", [EAGER, LAZY])
def test_pipelined_host_batch(monkeypatch, sem):
    # the one-device pipelined host batch (sub-shards, each download overlapping the next
    # compute): the same result as the one-shard path and the oracle, with dead strings,
    # empty strings and label-0 strings in the mix
    rng = np.random.default_rng(4242)
    blob = O.freeze(O.gen("ambiguous", 300, 12))
    rhs = load_blob(blob)
    seqs = []
    for i in range(2000):
        L = int(rng.integers(0, 40))
        s = [1] * L
        if L and i % 7 == 0:
            s[int(rng.integers(0, L))] = 2     # dies
        if L and i % 13 == 0:
            s[int(rng.integers(0, L))] = 0     # lhs epsilon
        seqs.append(s)
    labels, offsets = csr(seqs)
    monkeypatch.setenv("FSTAMD_PIPELINE", "0")
    one = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem)
    for parts in ("3", "7"):
        monkeypatch.setenv("FSTAMD_PIPELINE", parts)
        got = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem)
        for k in ("status", "offsets", "ilabels", "olabels"):
            assert np.array_equal(getattr(got, k), getattr(one, k)), (parts, k)
        assert np.array_equal(bits(got.weights), bits(one.weights))
        assert np.array_equal(bits(got.finals), bits(one.finals))
    ref = O.batch_run(blob, labels, offsets, 0 if sem == LAZY else 1, 1, 8)
    assert np.array_equal(one.status, expected_status(ref))
    assert np.array_equal(one.olabels, ref.olabels)
    assert np.array_equal(bits(one.weights), bits(ref.weights))
