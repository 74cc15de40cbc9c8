"""Multi-GPU plumbing for the batch engine: string sharding and a one-time rhs broadcast.

The path shards trivially by string (no per-step collective).  The frozen rhs blob is
built or loaded on rank 0 and broadcast once with torch.distributed (RCCL over xGMI on
GPUs, gloo in CPU tests); every rank then adopts it (fst_device_adopt_blob on a GPU, or
fst_load of the bytes on a host).
"""
from __future__ import annotations

import os
import tempfile

import torch
import torch.distributed as dist

from . import fst as F


def shard_range(num: int, rank: int, world: int):
    """Contiguous, balanced [begin, end) of `num` strings for `rank` of `world`."""
    base, rem = divmod(num, world)
    begin = rank * base + min(rank, rem)
    return begin, begin + base + (1 if rank < rem else 0)


def cost_shard_range(lengths, rhs: "F.Fst", rank: int, world: int):
    """Contiguous [begin, end) of the strings for `rank`, balanced by the library's work
    estimate (fst_chain_cost: product tuples per string) instead of by count -- config 3's
    lengths 11..251 differ 20x in cost.  Shards tile the batch; every shard is non-empty
    when there are at least `world` strings."""
    import numpy as np
    lengths = np.asarray(lengths, dtype=np.int64)
    num = len(lengths)
    if num == 0:
        return 0, 0
    L = F.lib()
    # one call per distinct length
    uniq, inv = np.unique(lengths, return_inverse=True)
    cost = np.array([L.fst_chain_cost(rhs.h, int(u)) for u in uniq])[inv]
    cum = np.concatenate([[0.0], np.cumsum(cost)])

    def cut(j):  # first string of shard j
        if j <= 0:
            return 0
        if j >= world:
            return num
        i = int(np.searchsorted(cum, cum[-1] * j / world, side="left"))
        return min(max(i, j if num >= world else 0), num - (world - j) if num >= world else num)
    return cut(rank), cut(rank + 1)


def blob_bytes(fst: "F.Fst") -> bytes:
    """The frozen blob of an Fst handle (fst_save, src/io/binary.zig:9-13)."""
    fd, path = tempfile.mkstemp(suffix=".fst")
    os.close(fd)
    try:
        if fst.save(path) != F.FST_OK:
            raise RuntimeError("fst_save failed")
        with open(path, "rb") as fh:
            return fh.read()
    finally:
        os.unlink(path)


def broadcast_blob(blob: bytes | None, rank: int, device: torch.device) -> torch.Tensor:
    """Broadcast rank 0's blob bytes to every rank; returns a uint8 tensor on `device`."""
    n = torch.tensor([len(blob) if rank == 0 else 0], dtype=torch.int64, device=device)
    dist.broadcast(n, src=0)
    buf = torch.empty(int(n.item()), dtype=torch.uint8, device=device)
    if rank == 0:
        buf.copy_(torch.frombuffer(bytearray(blob), dtype=torch.uint8))
    dist.broadcast(buf, src=0)
    return buf


def adopt_on_device(buf: torch.Tensor, device_index: int) -> "F.Fst":
    """Adopt a device-resident blob (after broadcast_blob on a GPU)."""
    torch.cuda.synchronize(device_index)
    h = F.lib().fst_device_adopt_blob(buf.data_ptr(), buf.numel(), device_index, None)
    return F.Fst(h)


def load_host_blob(data: bytes) -> "F.Fst":
    """Adopt a blob on the host (fst_load of the bytes; validates like fromBytes)."""
    fd, path = tempfile.mkstemp(suffix=".fst")
    os.close(fd)
    try:
        with open(path, "wb") as fh:
            fh.write(data)
        return F.Fst.load(path)
    finally:
        os.unlink(path)
