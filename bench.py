"""bench.py -- strings/s on compose_frozen_shortest_path_ambiguous (BASELINE.json metric).

Workload (BASELINE.json configs[1] / metric; reference bench/optimize-bench.zig:250-277,
:182-196, :374-380): each string is the `repeat` acceptor 1^64, composed against the
frozen ambiguous-chain transducer (T=4096, B=12) and reduced to its 1-best path with the
scenario's semantics: eager fst_compose_frozen + fst_shortest_path.  A "step" is one
pass of the engine over a device-resident batch of --batch strings per GPU (default 1M).

N GPUs: one process per GPU (torchrun); the frozen rhs blob is built on rank 0 and
broadcast once over xGMI with RCCL (torch.distributed "nccl"), then adopted by every
rank (fst_device_adopt_blob).  No per-step collectives: each rank runs its own shard;
timing is barrier + synchronize on both sides, max over ranks.  The metric's form is
"batch=1M, 1/2/4/8 GPU".  By default (--scaling weak) every rank gets --batch strings
(1M) per step, so an N-GPU step processes N x 1M strings and `value` is their sum over the
max-over-ranks time; --scaling strong splits --global-batch strings (1M) of a step over
the ranks instead.
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
# VALU issue peak: 256 CUs x 4 SIMDs, each SIMD busy with VALU at most every cycle of the
# 2.4 GHz max clock (MI355X_MICROARCH.md: 4 SIMDs per CU, max clock 2400 MHz)
SIMDS = 256 * 4
CLOCK_GHZ = 2.4
VALU_PEAK_GCYC = SIMDS * CLOCK_GHZ   # G SIMD-cycles/s
# Measured HBM traffic of the metric kernel: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes
# over this same command (scripts/profile_bench.sh), reduced by scripts/pmc_summary.py.
TRAFFIC_FILES = {1: os.path.join(REPO, "profiles", "pmc_traffic.json"),
                 0: os.path.join(REPO, "profiles", "pmc_traffic_lazy.json")}
# SQ instruction mix of the metric kernel (scripts/sq_counters.sh + sq_summary.py --json):
# the kernel's real bound is VALU issue, not bytes
ISSUE_FILES = {1: os.path.join(REPO, "profiles", "sq_issue.json"),
               0: os.path.join(REPO, "profiles", "sq_issue_lazy.json")}
L2_PEAK_GBS = 34500.0  # MI355X aggregate L2 (MI355X_MICROARCH.md "L2 (per XCD)")


EAGER_KERNEL = "eager_pull_kernel"     # tier P, takes every metric string
LAZY_KERNEL = "lazy_pull_kernel"
KERNELS = {1: EAGER_KERNEL, 0: LAZY_KERNEL}


def measured_traffic(args, sem):
    """Per-launch HBM bytes from the committed PMC summary (metric config only), else None.
    The summary must name the kernel this run times (a stale file gives None)."""
    if (args.len, args.transducer_len, args.branches) != (64, 4096, 12):
        return None, None
    try:
        t = json.load(open(TRAFFIC_FILES[sem]))
    except (OSError, ValueError):
        return None, None
    if t.get("kernel") != KERNELS[sem]:
        return None, None
    return t["traffic_per_string"] * args.batch, t.get("source", TRAFFIC_FILES[sem])


def issue_profile(args, sem):
    """SQ instruction mix of the eager metric kernel (committed summary of rocprofv3 --pmc
    SQ_* passes over this command at 65,536 strings), or None for another workload."""
    if (args.len, args.transducer_len, args.branches) != (64, 4096, 12):
        return None
    try:
        t = json.load(open(ISSUE_FILES[sem]))
    except (OSError, ValueError):
        return None
    if t.get("kernel") != KERNELS[sem]:
        return None
    return t


def roofline_block(args, sem, avg_k_ms, balg, work, lengths, plen, traffic, traffic_src):
    """The roofline of the dominant kernel against the resource that binds it.

    The metric kernel is bound by VALU issue (SQ counters: VALU busy ~2/3 of SIMD cycles,
    HBM ~1/5 of peak), so `achieved` = VALU-busy SIMD cycles per second: the committed SQ
    profile's SQ_ACTIVE_INST_VALU per string (quad-cycles, x4) x the strings of this launch
    / the kernel time measured live (HIP events on the launch stream); `peak` = 1024 SIMDs x
    2.4 GHz.  HBM (PMC-measured bytes / kernel time) and the SURVEY 8(d) logical bytes
    (B_alg: L2/LDS-served, so above the HBM peak) are reported beside it, each with its own
    fraction."""
    ks = avg_k_ms * 1e-3
    n = args.batch
    hbm = None
    if traffic:
        gbs = traffic / ks / 1e9
        hbm = {"achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
               "bytes_per_string": traffic / n, "source": traffic_src}
    logical = balg / ks / 1e9
    b_alg = {"achieved": logical, "unit": "GB/s", "bytes_per_string": balg / n,
             "frac_vs_hbm_peak": logical / HBM_PEAK_GBS, "frac_vs_l2_peak": logical / L2_PEAK_GBS,
             "note": "SURVEY 8(d) B_alg = 24 R + 16 X + 4 L + 16 P per string (exact, from the "
                     "kernel's work counters); these reads hit the L2-resident rhs mirror and "
                     "LDS, not HBM, so they are priced against L2 as well"}
    sq = issue_profile(args, sem)
    blk = {"kernel": EAGER_KERNEL if sem else LAZY_KERNEL, "kernel_ms": avg_k_ms,
           "traffic": traffic, "hbm": hbm, "b_alg": b_alg,
           "relaxations_per_s": float(work[1::2].astype(np.int64).sum()) / ks,
           "compulsory_bytes_per_string": float((4 * lengths + 16 * plen + 24).sum()) / n}
    if sq is not None:
        ps = sq["per_string"]
        busy_cyc = 4.0 * ps["SQ_ACTIVE_INST_VALU"]          # quad-cycles -> cycles
        ach = busy_cyc * n / ks / 1e9
        blk.update({"bound": "valu", "achieved": ach, "peak": VALU_PEAK_GCYC,
                    "unit": "G SIMD-cycles/s (VALU busy)", "frac": ach / VALU_PEAK_GCYC,
                    "valu_insts_per_string": ps.get("SQ_INSTS_VALU"),
                    "valu_busy_cycles_per_string": busy_cyc,
                    "salu_insts_per_string": ps.get("SQ_INSTS_SALU"),
                    "lds_insts_per_string": ps.get("SQ_INSTS_LDS"),
                    "issue_source": sq.get("source", ISSUE_FILES[sem])})
    elif hbm is not None:
        blk.update({"bound": "hbm", "achieved": hbm["achieved"], "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": hbm["frac"]})
    else:  # no counters for this workload: the logical bytes against HBM (may exceed 1)
        blk.update({"bound": "hbm", "achieved": logical, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": logical / HBM_PEAK_GBS,
                    "note": "no PMC/SQ profile for this workload: B_alg logical bytes"})
    return blk


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--scaling", choices=["strong", "weak"], default="weak",
                   help="strong: --global-batch strings per step split over the ranks (the "
                        "metric's batch=1M at 1/2/4/8 GPUs); weak: --batch strings per rank")
    p.add_argument("--global-batch", type=int, default=1 << 20,
                   help="strong scaling: strings per step over all GPUs")
    p.add_argument("--batch", type=int, default=1 << 20,
                   help="weak scaling: strings per GPU per step")
    p.add_argument("--backend", default="nccl",
                   help="torch.distributed backend (nccl = RCCL; gloo for ranks sharing a GPU "
                        "in tests)")
    p.add_argument("--no-f64", dest="f64", action="store_false",
                   help="skip the f64-cell and fractional-weight legs")
    p.add_argument("--len", type=int, default=64)
    p.add_argument("--transducer-len", type=int, default=4096)
    p.add_argument("--branches", type=int, default=12)
    p.add_argument("--semantics", choices=["eager", "lazy"], default="eager")
    p.add_argument("--no-varied", dest="varied", action="store_false",
                   help="skip the varied batch (lengths 1..len, 10%% dead strings)")
    p.add_argument("--no-e2e", dest="e2e", action="store_false",
                   help="profiling runs only: skip the host-entry headline (value is then the "
                        "kernel-resident rate, and the line says so)")
    p.add_argument("--lazy-batch", type=int, default=-1,
                   help="also time the lazy engine on this many metric strings "
                        "(-1 = the eager batch size, 0 = off)")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget")
    p.add_argument("--cpu-threads", type=int, default=0, help="0 = nproc (the affinity mask)")
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


def check_sample(batch, blob_bytes, sem, n=256, threads=1):
    """Bit-compares the first n strings of the last run with the oracle (compose.zig +
    shortest-path.zig, or compose-shortest-path.zig): status, path labels, arc weights and
    final weight, f64 bit patterns.  The oracle is the checker here, never the thing timed."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ffi as O  # checker / CPU baseline only

    n = min(n, batch.num)
    offs = batch.offsets[: n + 1].cpu().numpy().astype(np.uint64)
    labels = batch.labels[: int(offs[-1])].cpu().numpy().astype(np.uint32)
    ref = O.batch_run(blob_bytes, labels, offs, 1 if sem == F.FST_SEM_EAGER else 0, 1, threads)
    return compare_with_ref(batch, ref, n)


def compare_with_ref(batch, ref, n):
    """Asserts that the first n strings of a DeviceBatch equal an oracle BatchResult."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ffi as O  # checker only

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
        el = max_over_ranks(el, dev_index)
    return el, kms, st


def max_over_ranks(x, dev_index):
    on = f"cuda:{dev_index}" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=on)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def nproc():
    """What GNU `nproc` prints: OMP_NUM_THREADS when set, else the CPUs of this process's
    affinity mask.  On the GPU box that is its CPU share (16: OMP_NUM_THREADS, and the cgroup
    quota cpu.max), while the affinity mask and os.cpu_count() show the whole host (256)."""
    try:
        v = int(os.environ.get("OMP_NUM_THREADS", "0"))
        if v > 0:
            return v
    except ValueError:
        pass
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def cgroup_cpu_limit():
    """CPUs the cgroup quota allows (cpu.max), or None when unlimited / unknown."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        return None


def cpu_baseline(args, blob_bytes, sem, seconds=None):
    """The CPU port (oracle/fst_oracle.c -O3, the reference's algorithm) on nproc host
    threads, each composing its share of a bounded sample of the same strings."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ffi as O  # checker / CPU baseline only

    threads = args.cpu_threads or nproc()
    L = args.len

    def run(n, th):
        labels = np.ones(n * L, np.uint32)
        offs = (np.arange(n + 1, dtype=np.uint64) * L)
        secs, _ = O.batch_time(blob_bytes, labels, offs, sem, th)
        return secs

    probe = 64
    s = run(probe, 1)
    single = probe / s
    # all threads on a small sample first: a cgroup quota below nproc would otherwise make
    # the main run many times longer than its budget
    n0 = threads * 4
    agg0 = n0 / run(n0, threads)
    budget = args.cpu_seconds if seconds is None else seconds
    n = int(max(n0, min(4_000_000, agg0 * budget)))
    s = run(n, threads)
    return {"value": n / s, "unit": "strings/s", "cores": threads, "kind": "port",
            "nproc": nproc(), "os_cpu_count": os.cpu_count(),
            "cgroup_cpu_limit": cgroup_cpu_limit(),
            "single_thread_value": single,
            "sample": f"{n} strings (1^{L} vs ambiguous T={args.transducer_len} B={args.branches}, "
                      f"{'eager compose+shortestPath' if sem else 'lazy composeShortestPath'}) "
                      f"on {threads} host threads (= nproc), oracle/fst_oracle.c -O3, {s:.1f} s"}


def fractional_ambiguous(T, B, delta=0.5, table=None):
    """The metric's ambiguous-chain rhs (bench/optimize-bench.zig:250-277) with every arc
    weight + delta (a WeText-like fractional grammar weight): built through the library's
    MutableFst API and frozen (fst_freeze).  Distances stop being integers: a dyadic delta
    (0.5) keeps the pull tiers' integer records (weights scaled by 2, exact), any other
    (0.1) takes their f64 cells (src/weight.zig:15-37 semantics throughout).  table: the
    arcs' weights drawn from these values instead (arc b of state i: table[(5 i + b + 1) %
    len], its self-loop table[5 i % len]) -- a grammar with that many distinct costs."""
    m = F.MutableFst()
    for _ in range(T + 1):
        m.add_state()
    m.set_start(0)
    fan = max(1, min(B, 4))
    for i in range(T + 1):
        m.set_final(i, 0.0)
        m.add_arc(i, 1, 1, table[(5 * i) % len(table)] if table else 0.0 + delta, i)
        for b in range(fan):
            w = table[(5 * i + b + 1) % len(table)] if table else float(b) + delta
            m.add_arc(i, 1, ((i + b) % 255) + 1, w, min(i + b + 1, T))
    return m.freeze()


def leg(batch, rhs, sem, dev_index, world, total_per_step, blob, env=None, steps=3):
    """One extra timed leg on the metric batch (3 steps after 1 warm-up), every string OK
    and the first 256 bit-compared with the oracle.  env: variables set for the leg only
    (read by the library at each call)."""
    env = env or {}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        el, kms, st = timed(batch, rhs, sem, dev_index, steps, 1, world)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    status = batch.status.cpu().numpy()
    assert np.all(status == F.FST_PATH_OK), np.unique(status, return_counts=True)
    return {"value": total_per_step * steps / el, "kernel_ms": float(np.mean(kms)),
            "checked_vs_oracle": check_sample(batch, blob, sem)}


def host_timed(rhs, sem, dev_index, labels, offsets, steps, warmup, world):
    """Timed steps of the host batch entry fst_compose_frozen_shortest_path_batch: host
    labels in, H2D, kernels, D2H into the library's pinned result arrays, result out --
    SURVEY 8(d)'s wall time (bench/optimize-bench.zig:416-453 times the whole call).
    Barrier + synchronize on both sides, max over ranks.  Returns the last step's result."""
    def run():
        return F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem, dev_index)
    for _ in range(warmup):
        r = run()
        del r
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    kms = []
    r = None
    t0 = time.perf_counter()
    for _ in range(steps):
        r = None          # the previous result goes back to the pinned pool first
        r = run()
        kms.append(F.last_launch_stats().kernel_ms)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        el = max_over_ranks(el, dev_index)
    return el, kms, r


def check_host_result(r, labels, offsets, blob_bytes, sem, n=256):
    """Bit-compares the first n strings of a host BatchResult with the oracle (checker)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ffi as O  # checker only

    n = min(n, len(offsets) - 1)
    offs = np.asarray(offsets[: n + 1], np.uint64)
    ref = O.batch_run(blob_bytes, np.asarray(labels[: int(offs[-1])], np.uint32), offs,
                      1 if sem == F.FST_SEM_EAGER else 0, 1, 1)
    exp = np.where(ref.empty == 1, F.FST_PATH_EMPTY, F.FST_PATH_OK)
    assert np.all(ref.status == O.OR_OK) and np.array_equal(r.status[:n], exp), "status"
    a, b = int(r.offsets[0]), int(r.offsets[n])
    assert np.array_equal(r.offsets[: n + 1] - r.offsets[0], ref.offsets), "path offsets"
    assert np.array_equal(r.ilabels[a:b], ref.ilabels), "ilabels"
    assert np.array_equal(r.olabels[a:b], ref.olabels), "olabels"
    assert np.array_equal(r.weights[a:b].view(np.uint64), ref.weights.view(np.uint64)), "w"
    ok = exp == F.FST_PATH_OK
    assert np.array_equal(r.finals[:n][ok].view(np.uint64), ref.finals[ok].view(np.uint64))
    return int(n)


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """`bench.py --gpus N` without a launcher: start torchrun with N ranks (one per GPU) as
    a CHILD process -- before this process touches the GPU, never exec -- and hand back its
    exit code.  Its ranks inherit stdout, so rank 0's JSON line is this command's output."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", "--master-port",
           str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if os.environ.get("FSTAMD_BENCH_DRY_LAUNCH"):  # tests (CPU): the command only
        print(json.dumps({"launch": cmd}), flush=True)
        return 0
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    # rank topology first, before anything touches the GPU (launch_ranks runs a child)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # N ranks' host entries share the host's DRAM: each stages its labels once (into
        # the pinned result) instead of twice, ~23 % fewer host bytes per string
        os.environ.setdefault("FSTAMD_STREAM_STAGE", "1")
    # one GPU per rank; ranks beyond the visible devices share them (gloo tests only)
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)
    sem = F.FST_SEM_EAGER if args.semantics == "eager" else F.FST_SEM_LAZY
    if args.scaling == "strong":  # this rank's contiguous share of the global batch
        b0, b1 = D.shard_range(args.global_batch, rank, world)
        args.batch = b1 - b0
    total_per_step = args.global_batch if args.scaling == "strong" else args.batch * world

    # ---- rhs: built on rank 0, broadcast once over xGMI (RCCL), adopted on every rank ----
    blob_host = None
    if rank == 0:
        blob_host = D.blob_bytes(
            F.Fst.bench_transducer(F.BENCH_AMBIGUOUS, args.transducer_len, args.branches))
    if world > 1 and args.backend == "nccl":
        buf = D.broadcast_blob(blob_host, rank, dev)
    elif world > 1:  # gloo: broadcast through host memory
        buf = D.broadcast_blob(blob_host, rank, torch.device("cpu")).to(dev)
    else:
        buf = torch.frombuffer(bytearray(blob_host), dtype=torch.uint8).to(dev)
    rhs = D.adopt_on_device(buf, local)
    del buf
    blob_check = blob_host if blob_host is not None else D.blob_bytes(
        F.Fst.bench_transducer(F.BENCH_AMBIGUOUS, args.transducer_len, args.branches))

    L = args.len
    lengths = np.full(args.batch, L, np.int64)

    # ---- headline: the host entry, host arrays in and out (SURVEY 8(d) wall time) ----
    h_labels = np.ones(args.batch * L, np.uint32)          # the caller's (pageable) arrays
    h_offsets = np.arange(args.batch + 1, dtype=np.uint64) * L
    if args.e2e:
        el, hkms, res = host_timed(rhs, sem, local, h_labels, h_offsets, args.steps,
                                   args.warmup, world)
        assert np.all(res.status == F.FST_PATH_OK), np.unique(res.status, return_counts=True)
        assert int(res.offsets[-1]) == args.batch * L
        checked = check_host_result(res, h_labels, h_offsets, blob_check, sem)
        del res

    # ---- kernel-only: the same strings device-resident (fst_device_compose_shortest_path) --
    batch = DeviceBatch(lengths, lambda t: torch.ones(t, dtype=torch.int32), dev)
    kel, kms, st = timed(batch, rhs, sem, local, args.steps, args.warmup, world)
    status = batch.status.cpu().numpy()
    plen = batch.plen.cpu().numpy().astype(np.int64)
    assert np.all(status == F.FST_PATH_OK), np.unique(status, return_counts=True)
    assert np.all(plen == L)
    kchecked = check_sample(batch, blob_check, sem)
    # one untimed run with the per-string work counters (B_alg of the roofline)
    batch.run(rhs, sem, local, torch.cuda.current_stream().cuda_stream, work=True)
    torch.cuda.synchronize()
    work = batch.work.cpu().numpy().astype(np.int64)
    avg_k = float(np.mean(kms))
    balg = b_alg_bytes(work, lengths, plen)   # bytes per launch on this rank
    if not args.e2e:  # (profiling runs) the headline falls back to the kernel-resident rate
        el, hkms, checked = kel, kms, kchecked
    value = total_per_step * args.steps / el
    extra = {"value_kernel": total_per_step * args.steps / kel,
             "kernel_resident": {
                 "value": total_per_step * args.steps / kel,
                 "ms_per_step": kel / args.steps * 1e3, "kernel_ms": avg_k,
                 "checked_vs_oracle": kchecked,
                 "note": "fst_device_compose_shortest_path on device-resident labels/outputs: "
                         "kernels only, no host copies (the roofline's kernel)"},
             "end_to_end": None if not args.e2e else {"ms_per_call": el / args.steps * 1e3,
                            "kernel_ms_per_call": float(np.mean(hkms)),
                            "bytes_in_per_call": int(h_labels.nbytes + h_offsets.nbytes),
                            "note": "the headline: fst_compose_frozen_shortest_path_batch, "
                                    "pageable host labels in, pinned host result out (the "
                                    "streamed batch: labels staged into the result while the "
                                    "kernel reads them, paths copied out by the kernel)"}}

    if args.varied:
        rng = np.random.default_rng(1234 + rank)
        vl = rng.integers(1, L + 1, size=args.batch)

        def vlabels(t):
            x = torch.ones(t, dtype=torch.int32)
            kill = torch.from_numpy((rng.random(t) < (0.1 / L)).astype(np.int32))
            return x + kill
        vb = DeviceBatch(vl, vlabels, dev)
        vel, vk, _ = timed(vb, rhs, sem, local, args.steps, args.warmup, world)
        extra["varied"] = {"value": total_per_step * args.steps / vel,
                           "kernel_ms": float(np.mean(vk)),
                           "lengths": "uniform 1..%d, ~10%% strings with a dead label" % L,
                           "checked_vs_oracle": check_sample(vb, blob_check, sem)}
        del vb
    if args.lazy_batch < 0:
        args.lazy_batch = args.batch
    if args.lazy_batch and sem == F.FST_SEM_EAGER:
        lb = DeviceBatch(np.full(args.lazy_batch, L, np.int64),
                         lambda t: torch.ones(t, dtype=torch.int32), dev)
        lel, lk, _ = timed(lb, rhs, F.FST_SEM_LAZY, local, 3, 1, world)
        ls = lb.status.cpu().numpy()
        assert np.all(ls == F.FST_PATH_OK)
        lazy_total = args.lazy_batch * world
        if args.scaling == "strong" and args.lazy_batch == args.batch:
            lazy_total = total_per_step
        extra["lazy"] = {"value": lazy_total * 3 / lel, "kernel_ms": float(np.mean(lk)),
                         "batch": args.lazy_batch,
                         "checked_vs_oracle": check_sample(lb, blob_check, F.FST_SEM_LAZY),
                         "note": "fst_compose_frozen_shortest_path semantics (lazy_pull_kernel, "
                                 "exact vs the oracle), device-resident"}
        if args.lazy_batch == args.batch:
            lb.run(rhs, F.FST_SEM_LAZY, local, torch.cuda.current_stream().cuda_stream, work=True)
            torch.cuda.synchronize()
            lwork = lb.work.cpu().numpy().astype(np.int64)
            lplen = lb.plen.cpu().numpy().astype(np.int64)
            extra["lazy"]["roofline"] = roofline_block(
                args, F.FST_SEM_LAZY, float(np.mean(lk)), b_alg_bytes(lwork, lengths, lplen),
                lwork, lengths, lplen, *measured_traffic(args, F.FST_SEM_LAZY))
        del lb
        if rank == 0 and not args.no_cpu and world == 1:  # the CPU port beside it (~3 s)
            extra["lazy"]["cpu_baseline"] = cpu_baseline(args, blob_check, 0, seconds=3.0)

    if args.f64:
        # the f64-cell rates beside the headline: the integer cells above hold only because
        # the metric's weights are small integers; fractional grammar weights take f64 cells
        E, Lz = F.FST_SEM_EAGER, F.FST_SEM_LAZY
        extra["f64_cells"] = {
            "eager": leg(batch, rhs, E, local, world, total_per_step, blob_check,
                         {"FSTAMD_P_F64": "1"}),
            "lazy": leg(batch, rhs, Lz, local, world, total_per_step, blob_check,
                        {"FSTAMD_LP_F64": "1"}),
            "note": "same metric batch and rhs, the pull kernels forced to f64 cells "
                    "(FSTAMD_P_F64 / FSTAMD_LP_F64), device-resident"}
        for key, delta, how in (("fractional_weights", 0.5, "dyadic: integer records "
                                 "scaled by 2"), ("non_dyadic_weights", 0.1,
                                 "f64 cells; eager: 4-B records indexing a weight table")):
            fr = fractional_ambiguous(args.transducer_len, args.branches, delta)
            fr_blob = D.blob_bytes(fr)
            extra[key] = {
                "eager": leg(batch, fr, E, local, world, total_per_step, fr_blob),
                "lazy": leg(batch, fr, Lz, local, world, total_per_step, fr_blob),
                "rhs": f"ambiguous chain T={args.transducer_len} B={args.branches}, every arc "
                       f"weight + {delta} ({how}), device-resident"}
            del fr
        # 200 distinct non-dyadic arc weights: tier P's 4-B records index a 256-entry table
        # (RK 5, round 6; up to 64 weights the 64-entry one)
        fr = fractional_ambiguous(args.transducer_len, args.branches,
                                  table=[0.1 + k / 7.0 for k in range(200)])
        fr_blob = D.blob_bytes(fr)
        extra["wide_weight_table"] = {
            "eager": leg(batch, fr, E, local, world, total_per_step, fr_blob),
            "lazy": leg(batch, fr, Lz, local, world, total_per_step, fr_blob),
            "rhs": f"ambiguous chain T={args.transducer_len} B={args.branches}, arc weights "
                   "drawn from 200 distinct non-dyadic values (f64 cells; eager: 4-B records "
                   "indexing a 256-entry weight table), device-resident"}
        del fr
    del batch

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
            "scaling": args.scaling,
            "vs_baseline": None,
            # results and the CPU port are f64; on this integer-weight rhs the pull tiers
            # keep the cells' distances as exact integers (every distance < 2^24), so every
            # output bit equals the f64 computation (checked_vs_oracle)
            "dtype": "f64",
            "cell_dtype": "u32 (exact: integer weights, max_len * max weight < 2^24)",
            "data": "synthetic (reference bench generators: 1^64 repeat acceptors, "
                    "ambiguous-chain rhs)",
            "timed": ("host entry: pageable host labels in -> kernels -> host result "
                      "(SURVEY 8(d) wall time); kernel-only rate in value_kernel") if args.e2e
                     else "kernel-resident only (--no-e2e profiling run)",
            "config": {"workload": "compose_frozen_shortest_path_ambiguous",
                       "semantics": args.semantics, "len": L,
                       "transducer_len": args.transducer_len, "branches": args.branches,
                       "strings_per_gpu": args.batch,
                       "global_batch": total_per_step,
                       "scaling_mode": (f"strong: {total_per_step} strings per step split over "
                                        f"{world} GPU(s)" if args.scaling == "strong" else
                                        f"weak: {args.batch} strings per GPU per step"),
                       "parallelism": f"dp{world} (string shards, rhs replicated via "
                                      f"{'RCCL' if args.backend == 'nccl' else args.backend} broadcast)"},
            "roofline": roofline_block(args, sem, avg_k, balg, work, lengths, plen, traffic,
                                       traffic_src),
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
