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
