"""bench.py -- strings/s on compose_frozen_shortest_path_ambiguous (BASELINE.json metric).

Workload (BASELINE.json configs[1] / metric; reference bench/optimize-bench.zig:250-277,
:182-196, :374-380): each string is the `repeat` acceptor 1^64, composed against the
frozen ambiguous-chain transducer (T=4096, B=12) and reduced to its 1-best path with the
scenario's semantics: eager fst_compose_frozen + fst_shortest_path.  A "step" is one
pass of the engine over a device-resident batch of --batch strings per GPU (default 1M).

N GPUs: one process per GPU (torchrun); the frozen rhs blob is built on rank 0 and
broadcast once over xGMI with RCCL (torch.distributed "nccl"), then adopted by every
rank (fst_device_adopt_blob).  No per-step collectives: each rank runs its own shard
(weak scaling); timing is barrier + synchronize on both sides, max over ranks.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import libfst_amd as F  # noqa: E402
from libfst_amd import dist as D  # noqa: E402
from libfst_amd import fst as FF  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# Measured HBM traffic of the metric kernel: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes
# over this same command (scripts/profile_bench.sh), reduced by scripts/pmc_summary.py.
TRAFFIC_FILE = os.path.join(REPO, "profiles", "pmc_traffic.json")
# SQ instruction mix of the metric kernel (scripts/sq_counters.sh + sq_summary.py --json):
# the kernel's real bound is VALU issue, not bytes
ISSUE_FILE = os.path.join(REPO, "profiles", "sq_issue.json")
L2_PEAK_GBS = 34500.0  # MI355X aggregate L2 (MI355X_MICROARCH.md "L2 (per XCD)")


EAGER_KERNEL = "eager_pull_kernel"     # tier P, takes every metric string
LAZY_KERNEL = "lazy_pull_kernel"


def measured_traffic(args, sem):
    """Per-launch HBM bytes from the committed PMC summary (metric config only), else None.
    The summary must name the kernel this run times (a stale file gives None)."""
    if sem != F.FST_SEM_EAGER or (args.len, args.transducer_len, args.branches) != (64, 4096, 12):
        return None, None
    try:
        t = json.load(open(TRAFFIC_FILE))
    except (OSError, ValueError):
        return None, None
    if t.get("kernel") != EAGER_KERNEL:
        return None, None
    return t["traffic_per_string"] * args.batch, t.get("source", TRAFFIC_FILE)


def issue_profile(sem):
    """VALU issue figures of the eager metric kernel from the committed SQ summary."""
    if sem != F.FST_SEM_EAGER:
        return None
    try:
        t = json.load(open(ISSUE_FILE))
    except (OSError, ValueError):
        return None
    if t.get("kernel") != EAGER_KERNEL:
        return None
    ps, wc = t["per_string"], t["of_wave_cycles"]
    return {"bound": "valu-issue",
            "valu_insts_per_string": ps.get("SQ_INSTS_VALU"),
            "salu_insts_per_string": ps.get("SQ_INSTS_SALU"),
            "lds_insts_per_string": ps.get("SQ_INSTS_LDS"),
            "valu_active_per_wave": wc.get("SQ_ACTIVE_INST_VALU"),
            "source": t.get("source", ISSUE_FILE)}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--batch", type=int, default=1 << 20, help="strings per GPU per step")
    p.add_argument("--len", type=int, default=64)
    p.add_argument("--transducer-len", type=int, default=4096)
    p.add_argument("--branches", type=int, default=12)
    p.add_argument("--semantics", choices=["eager", "lazy"], default="eager")
    p.add_argument("--varied", action="store_true",
                   help="also time a varied batch (lengths 1..len, 10%% dead strings)")
    p.add_argument("--lazy-batch", type=int, default=-1,
                   help="also time the lazy engine on this many metric strings "
                        "(-1 = the eager batch size, 0 = off)")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget")
    p.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, cpu_count)")
    p.add_argument("--no-cpu", action="store_true")
    return p.parse_args()


def dev_ptr(t):
    return C.c_void_p(t.data_ptr())


class DeviceBatch:
    """Device-resident inputs + outputs of one batch (torch tensors as plumbing)."""

    def __init__(self, lengths, label_fn, dev, arc_factor=1):
        B = len(lengths)
        lens = torch.as_tensor(lengths, dtype=torch.int64)
        self.offsets = torch.zeros(B + 1, dtype=torch.int64)
        self.offsets[1:] = torch.cumsum(lens, 0)
        total = int(self.offsets[-1])
        self.labels = label_fn(total).to(dev)
        self.offsets = self.offsets.to(dev)
        self.num = B
        self.max_len = int(lens.max()) if B else 0
        # path arena: L arcs per string on the metric; epsilon lattices (arc_factor > 1)
        # can produce longer paths
        self.cap = max(arc_factor * total + 64, 1024)
        self.status = torch.empty(B, dtype=torch.int32, device=dev)
        self.plen = torch.empty(B, dtype=torch.int32, device=dev)
        self.poff = torch.empty(B, dtype=torch.int64, device=dev)
        self.fin = torch.empty(B, dtype=torch.float64, device=dev)
        self.il = torch.empty(self.cap, dtype=torch.int32, device=dev)
        self.ol = torch.empty(self.cap, dtype=torch.int32, device=dev)
        self.w = torch.empty(self.cap, dtype=torch.float64, device=dev)
        self.cursor = torch.zeros(1, dtype=torch.int64, device=dev)
        self.work = torch.empty(2 * B, dtype=torch.int32, device=dev)
        # timed steps produce the results only; the per-string work counters (tuples,
        # relaxations: instrumentation for the roofline's B_alg) come from one extra run
        self.desc = FF.FstDeviceBatch(
            self.status.data_ptr(), self.plen.data_ptr(), self.poff.data_ptr(),
            self.fin.data_ptr(), self.il.data_ptr(), self.ol.data_ptr(), self.w.data_ptr(),
            self.cap, self.cursor.data_ptr(), 0)
        self.desc_work = FF.FstDeviceBatch(
            self.status.data_ptr(), self.plen.data_ptr(), self.poff.data_ptr(),
            self.fin.data_ptr(), self.il.data_ptr(), self.ol.data_ptr(), self.w.data_ptr(),
            self.cap, self.cursor.data_ptr(), self.work.data_ptr())

    def run(self, rhs, sem, dev_index, stream, work=False):
        opts = FF.FstBatchOptions(dev_index, sem, 0)
        rc = F.lib().fst_device_compose_shortest_path(
            rhs.h, dev_ptr(self.labels), dev_ptr(self.offsets), self.num, self.max_len, 1,
            C.byref(opts), C.byref(self.desc_work if work else self.desc), C.c_void_p(stream))
        if rc != FF.FST_OK:
            raise RuntimeError(f"fst_device_compose_shortest_path failed: {rc}")
        return F.last_launch_stats()


def check_sample(batch, blob_bytes, sem, n=256):
    """Bit-compares the first n strings of the last run with the oracle (compose.zig +
    shortest-path.zig, or compose-shortest-path.zig): status, path labels, arc weights and
    final weight, f64 bit patterns.  The oracle is the checker here, never the thing timed."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ffi as O  # checker / CPU baseline only

    n = min(n, batch.num)
    offs = batch.offsets[: n + 1].cpu().numpy().astype(np.uint64)
    labels = batch.labels[: int(offs[-1])].cpu().numpy().astype(np.uint32)
    ref = O.batch_run(blob_bytes, labels, offs, 1 if sem == F.FST_SEM_EAGER else 0, 1)
    status = batch.status[:n].cpu().numpy()
    exp = np.where(ref.empty == 1, F.FST_PATH_EMPTY, F.FST_PATH_OK)
    assert np.all(ref.status == O.OR_OK) and np.array_equal(status, exp), "status mismatch"
    plen = batch.plen[:n].cpu().numpy().astype(np.int64)
    poff = batch.poff[:n].cpu().numpy().astype(np.int64)
    fin = batch.fin[:n].cpu().numpy()
    il, ol, w = batch.il.cpu().numpy(), batch.ol.cpu().numpy(), batch.w.cpu().numpy()
    for i in np.nonzero(exp == F.FST_PATH_OK)[0]:
        a, b = int(ref.offsets[i]), int(ref.offsets[i + 1])
        assert plen[i] == b - a, ("path length", i)
        g = slice(int(poff[i]), int(poff[i]) + b - a)
        assert np.array_equal(il[g].astype(np.uint32), ref.ilabels[a:b]), ("ilabels", i)
        assert np.array_equal(ol[g].astype(np.uint32), ref.olabels[a:b]), ("olabels", i)
        assert np.array_equal(w[g].view(np.uint64), ref.weights[a:b].view(np.uint64)), ("w", i)
        assert fin[i:i + 1].view(np.uint64)[0] == ref.finals[i:i + 1].view(np.uint64)[0], i
    return int(n)


def b_alg_bytes(work, lengths, plen):
    """B_alg = 24 R + 16 X + 4 L + 16 P per string (exact, from counters)."""
    X = work[0::2].astype(np.int64)
    R = work[1::2].astype(np.int64)
    return int((24 * R + 16 * X + 4 * np.asarray(lengths, np.int64) + 16 * plen).sum())


def timed(batch, rhs, sem, dev_index, steps, warmup, world):
    stream = torch.cuda.current_stream().cuda_stream
    for _ in range(warmup):
        batch.run(rhs, sem, dev_index, stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    kms = []
    t0 = time.perf_counter()
    for _ in range(steps):
        st = batch.run(rhs, sem, dev_index, stream)
        kms.append(st.kernel_ms)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=f"cuda:{dev_index}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el, kms, st


def cpu_baseline(args, blob_bytes, sem, seconds=None):
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ffi as O  # checker / CPU baseline only

    threads = args.cpu_threads or min(16, os.cpu_count() or 1)
    L = args.len

    def run(n, th):
        labels = np.ones(n * L, np.uint32)
        offs = (np.arange(n + 1, dtype=np.uint64) * L)
        secs, _ = O.batch_time(blob_bytes, labels, offs, sem, th)
        return secs

    probe = 64
    s = run(probe, 1)
    single = probe / s
    budget = args.cpu_seconds if seconds is None else seconds
    n = int(max(threads * 8, min(2_000_000, single * threads * budget * 0.8)))
    s = run(n, threads)
    return {"value": n / s, "unit": "strings/s", "cores": threads, "kind": "port",
            "single_thread_value": single,
            "sample": f"{n} strings (1^{L} vs ambiguous T={args.transducer_len} B={args.branches}, "
                      f"{'eager compose+shortestPath' if sem else 'lazy composeShortestPath'}) "
                      f"on {threads} host threads, oracle/fst_oracle.c -O3"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    sem = F.FST_SEM_EAGER if args.semantics == "eager" else F.FST_SEM_LAZY

    # ---- rhs: built on rank 0, broadcast once over xGMI (RCCL), adopted on every rank ----
    blob_host = None
    if rank == 0:
        blob_host = D.blob_bytes(
            F.Fst.bench_transducer(F.BENCH_AMBIGUOUS, args.transducer_len, args.branches))
    if world > 1:
        buf = D.broadcast_blob(blob_host, rank, dev)
    else:
        buf = torch.frombuffer(bytearray(blob_host), dtype=torch.uint8).to(dev)
    rhs = D.adopt_on_device(buf, local)
    del buf

    L = args.len
    lengths = np.full(args.batch, L, np.int64)
    batch = DeviceBatch(lengths, lambda t: torch.ones(t, dtype=torch.int32), dev)
    el, kms, st = timed(batch, rhs, sem, local, args.steps, args.warmup, world)

    # correctness of the last timed step: every metric string has one answer, and a fixed
    # sample is bit-compared with the oracle
    status = batch.status.cpu().numpy()
    plen = batch.plen.cpu().numpy().astype(np.int64)
    assert np.all(status == F.FST_PATH_OK), np.unique(status, return_counts=True)
    assert np.all(plen == L)
    blob_check = blob_host if blob_host is not None else D.blob_bytes(
        F.Fst.bench_transducer(F.BENCH_AMBIGUOUS, args.transducer_len, args.branches))
    checked = check_sample(batch, blob_check, sem)
    # one untimed run with the per-string work counters (B_alg of the roofline)
    batch.run(rhs, sem, local, torch.cuda.current_stream().cuda_stream, work=True)
    torch.cuda.synchronize()
    work = batch.work.cpu().numpy().astype(np.int64)

    total_strings = args.batch * args.steps * world
    value = total_strings / el
    avg_k = float(np.mean(kms))
    balg = b_alg_bytes(work, lengths, plen)   # bytes per launch on this rank
    achieved = balg / (avg_k * 1e-3) / 1e9
    # relaxations per second and the compulsory HBM bytes (labels in,
    # path + status/offset/final out) beside the logical bytes
    relax_per_s = float(work[1::2].astype(np.int64).sum()) / (avg_k * 1e-3)
    compulsory = int((4 * lengths + 16 * plen + 24).sum())

    extra = {}
    if args.varied:
        rng = np.random.default_rng(1234 + rank)
        vl = rng.integers(1, L + 1, size=args.batch)

        def vlabels(t):
            x = torch.ones(t, dtype=torch.int32)
            kill = torch.from_numpy((rng.random(t) < (0.1 / L)).astype(np.int32))
            return x + kill
        vb = DeviceBatch(vl, vlabels, dev)
        vel, vk, _ = timed(vb, rhs, sem, local, args.steps, args.warmup, world)
        extra["varied"] = {"value": args.batch * args.steps * world / vel,
                           "kernel_ms": float(np.mean(vk)),
                           "lengths": "uniform 1..%d, ~10%% strings with a dead label" % L,
                           "checked_vs_oracle": check_sample(vb, blob_check, sem)}
        del vb
    if args.lazy_batch < 0:
        args.lazy_batch = args.batch
    if args.lazy_batch and sem == F.FST_SEM_EAGER:
        lb = DeviceBatch(np.full(args.lazy_batch, L, np.int64),
                         lambda t: torch.ones(t, dtype=torch.int32), dev)
        lel, lk, lst = timed(lb, rhs, F.FST_SEM_LAZY, local, 3, 1, world)
        ls = lb.status.cpu().numpy()
        assert np.all(ls == F.FST_PATH_OK)
        extra["lazy"] = {"value": args.lazy_batch * 3 * world / lel, "kernel_ms": float(np.mean(lk)),
                         "batch": args.lazy_batch,
                         "checked_vs_oracle": check_sample(lb, blob_check, F.FST_SEM_LAZY),
                         "note": "fst_compose_frozen_shortest_path semantics (lazy_pull_kernel, exact vs the oracle)"}
        if rank == 0 and not args.no_cpu and world == 1:  # the CPU port beside it (~3 s)
            extra["lazy"]["cpu_baseline"] = cpu_baseline(args, blob_check, 0, seconds=3.0)

    if rank == 0:
        traffic, traffic_src = measured_traffic(args, sem)
        cpu = None
        if not args.no_cpu and world == 1:  # the CPU baseline is an N=1 figure
            cpu = cpu_baseline(args, blob_host, 1 if sem == F.FST_SEM_EAGER else 0)
        line = {
            "metric": "strings/sec, compose_frozen_shortest_path_ambiguous len=64 batch=1M",
            "value": value,
            "unit": "strings/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": el / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (reference bench generators: 1^64 repeat acceptors, "
                    "ambiguous-chain rhs)",
            "config": {"workload": "compose_frozen_shortest_path_ambiguous",
                       "semantics": args.semantics, "len": L,
                       "transducer_len": args.transducer_len, "branches": args.branches,
                       "strings_per_gpu": args.batch,
                       "global_batch": args.batch * world,
                       "parallelism": f"dp{world} (string shards, rhs replicated via RCCL broadcast)"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel_ms": avg_k, "b_alg_per_string": balg / args.batch,
                         "relaxations_per_s": relax_per_s,
                         "compulsory_bytes_per_string": compulsory / args.batch,
                         "kernel": EAGER_KERNEL if sem else LAZY_KERNEL,
                         # measured DRAM bytes / kernel time: what really crosses HBM
                         "hbm_traffic_gbs": (traffic / (avg_k * 1e-3) / 1e9) if traffic else None,
                         "hbm_traffic_frac": (traffic / (avg_k * 1e-3) / 1e9 / HBM_PEAK_GBS)
                         if traffic else None,
                         "l2_peak": L2_PEAK_GBS,
                         "l2_frac": achieved / L2_PEAK_GBS,
                         "issue": issue_profile(sem),
                         "note": "achieved = SURVEY 8(d) logical bytes (24 B per arc relaxed, 16 B "
                                 "per tuple expanded, labels, path) / kernel time. Those reads hit "
                                 "the 0.6 MB L2-resident rhs mirror (and LDS), never HBM, so frac "
                                 "(vs the 8 TB/s HBM peak) exceeds 1; l2_frac prices them against "
                                 "the 34.5 TB/s L2. hbm_traffic_* is the PMC-measured DRAM traffic "
                                 "(back records, labels, paths). The kernel is bound by VALU issue "
                                 "(issue: SQ counters)"},
            "cpu_baseline": cpu,
            "checked_vs_oracle": checked,
        }
        line.update(extra)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
