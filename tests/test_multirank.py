"""N>1 path on CPU: world_size-2 gloo run of the sharding + one-time rhs broadcast that
bench.py uses over RCCL on GPUs.  Each rank must end with a byte-identical blob and the
shards must tile the batch exactly."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    import torch
    import torch.distributed as dist
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(here))
    import libfst_amd as F
    from libfst_amd import dist as D

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        blob = None
        if rank == 0:
            blob = D.blob_bytes(F.Fst.bench_transducer(F.BENCH_AMBIGUOUS, 256, 12))
        buf = D.broadcast_blob(blob, rank, torch.device("cpu"))
        data = bytes(buf.numpy().tobytes())
        rhs = D.load_host_blob(data)
        ref = F.Fst.bench_transducer(F.BENCH_AMBIGUOUS, 256, 12)
        same = rhs.num_states == ref.num_states and all(
            rhs.arcs(s) == ref.arcs(s) for s in range(0, ref.num_states, 17))
        import zlib
        digest = torch.tensor([zlib.crc32(data)], dtype=torch.int64)
        gathered = [torch.zeros_like(digest) for _ in range(world)]
        dist.all_gather(gathered, digest)
        b, e = D.shard_range(1_000_003, rank, world)
        q.put((rank, same, len(set(int(g) for g in gathered)) == 1, b, e))
    finally:
        dist.destroy_process_group()


def test_two_rank_blob_broadcast_and_shards():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    assert all(r[1] for r in res), "rank saw a different rhs"
    assert all(r[2] for r in res), "blob bytes differ across ranks"
    spans = [(r[3], r[4]) for r in res]
    assert spans[0][0] == 0 and spans[-1][1] == 1_000_003
    assert all(spans[i][1] == spans[i + 1][0] for i in range(len(spans) - 1))


@pytest.mark.parametrize("num,world", [(0, 4), (7, 8), (1_000_000, 8), (13, 3)])
def test_shard_range_tiles(num, world):
    from libfst_amd.dist import shard_range
    parts = [shard_range(num, r, world) for r in range(world)]
    assert parts[0][0] == 0 and parts[-1][1] == num
    assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
    sizes = [e - b for b, e in parts]
    assert max(sizes) - min(sizes) <= 1


def _shard_worker(rank, world, port, q):
    """Each rank takes its cost-balanced shard (libfst_amd.dist.cost_shard_range, the
    library's own work estimate), composes it (on a CPU rank: the oracle, the checker;
    tests/test_gpu_multidevice.py runs the same with the GPU engines) and all ranks
    gather the per-string results in input order."""
    import sys
    import torch.distributed as dist
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(here))
    sys.path.insert(0, here)
    import libfst_amd as F
    from libfst_amd import dist as D
    import oracle_ffi as O

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rhs = F.Fst.bench_transducer(F.BENCH_EPS_DENSE, 32, 12)
        blob = D.blob_bytes(rhs)
        lens = np.random.default_rng(0x5EED).integers(11, 252, 30)
        b, e = D.cost_shard_range(lens, rhs, rank, world)
        mine = lens[b:e]
        offs = np.concatenate([[0], np.cumsum(mine)]).astype(np.uint64)
        r = O.batch_run(blob, np.ones(int(mine.sum()), np.uint32), offs, 0, 1)
        part = (b, e, [(int(r.status[i]), r.olabels[int(r.offsets[i]):int(r.offsets[i + 1])].tolist(),
                        float(r.finals[i])) for i in range(e - b)])
        parts = [None] * world
        dist.all_gather_object(parts, part)
        if rank == 0:
            parts.sort(key=lambda p: p[0])
            got = [x for p in parts for x in p[2]]
            offs_all = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
            ra = O.batch_run(blob, np.ones(int(lens.sum()), np.uint32), offs_all, 0, 1)
            exp = [(int(ra.status[i]), ra.olabels[int(ra.offsets[i]):int(ra.offsets[i + 1])].tolist(),
                    float(ra.finals[i])) for i in range(len(lens))]
            costs = [sum(F.lib().fst_chain_cost(rhs.h, int(L)) for L in lens[p[0]:p[1]]) for p in parts]
            q.put((got == exp, [(p[0], p[1]) for p in parts], max(costs) / max(min(costs), 1)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_ranks_compose_cost_shards_and_gather(world):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    same, spans, imbalance = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert same, "gathered shards differ from the whole-batch answer"
    assert spans[0][0] == 0 and spans[-1][1] == 30
    assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
    assert imbalance < 1.6
