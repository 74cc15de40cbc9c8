"""Bench-compatible CLI for the compose_frozen scenarios.

Same options and output schema as the reference's optimize-bench
(bench/optimize-bench.zig:104-158 usage, :160-328 inputs, :330-420 scenarios, :505-541
output), with the GPU engines behind the same C-ABI calls:

  python -m libfst_amd.optimize_bench --scenario compose_frozen_shortest_path_ambiguous \\
      --len 64 --transducer-len 4096 --branches 12 --iters 80 --warmup 5 --format json

One extra option, `--batch B` (default 1): B > 1 times one batched call over B copies of
the input string per iteration (fst_compose_frozen_shortest_path_batch, host buffers),
for the *_shortest_path scenarios; the JSON line then also carries "batch" and
"strings_per_s".  Scenarios off the compose_frozen path (clone, optimize, mutable compose,
rm_epsilon) are out of scope here and rejected.
"""
import argparse
import json
import sys
import time

import numpy as np

from . import fst as F

SCENARIOS = [
    "clone_acceptor", "optimize_acceptor", "optimize_transducer", "compose_acceptor",
    "compose_frozen_transducer", "compose_frozen_epsilon_dense",
    "compose_frozen_ambiguous_chain", "compose_frozen_shortest_path",
    "compose_frozen_shortest_path_ambiguous", "compose_frozen_shortest_path_epsilon_dense",
    "compose_frozen_lazy_shortest_path", "compose_frozen_lazy_shortest_path_ambiguous",
    "compose_frozen_lazy_shortest_path_epsilon_dense", "rm_epsilon_acceptor",
    "shortest_path_acceptor",
]
OUT_OF_SCOPE = {"clone_acceptor", "optimize_acceptor", "optimize_transducer",
                "compose_acceptor", "rm_epsilon_acceptor"}

# scenario -> (lhs input, rhs generator, op); optimize-bench.zig:330-420
PLAN = {
    "compose_frozen_transducer": ("branch", F.BENCH_BRANCHING, "compose"),
    "compose_frozen_epsilon_dense": ("repeat", F.BENCH_EPS_DENSE, "compose"),
    "compose_frozen_ambiguous_chain": ("repeat", F.BENCH_AMBIGUOUS, "compose"),
    "compose_frozen_shortest_path": ("branch", F.BENCH_BRANCHING, "eager"),
    "compose_frozen_shortest_path_ambiguous": ("repeat", F.BENCH_AMBIGUOUS, "eager"),
    "compose_frozen_shortest_path_epsilon_dense": ("repeat", F.BENCH_EPS_DENSE, "eager"),
    "compose_frozen_lazy_shortest_path": ("branch", F.BENCH_BRANCHING, "lazy"),
    "compose_frozen_lazy_shortest_path_ambiguous": ("repeat", F.BENCH_AMBIGUOUS, "lazy"),
    "compose_frozen_lazy_shortest_path_epsilon_dense": ("repeat", F.BENCH_EPS_DENSE, "lazy"),
    "shortest_path_acceptor": ("linear", None, "sp"),
}


def input_bytes(kind: str, n: int, branches: int) -> bytes:
    """compileString bytes (label = byte + 1) of the bench acceptors (:160-199)."""
    if kind == "repeat":
        return bytes(n)                                        # label 1 repeated
    alpha = max(1, branches) if kind == "branch" else 255
    return bytes(i % alpha for i in range(n))                 # (i % alpha) + 1


def parse_args(argv):
    ap = argparse.ArgumentParser(prog="optimize-bench (libfst_amd)")
    ap.add_argument("--scenario", choices=SCENARIOS, default="compose_frozen_shortest_path_ambiguous")
    ap.add_argument("--len", type=int, default=4096)
    ap.add_argument("--transducer-len", type=int, default=0)
    ap.add_argument("--branches", type=int, default=3)
    ap.add_argument("--iters", type=int, default=80)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--format", choices=["text", "json"], default="text")
    ap.add_argument("--per-iter", choices=["true", "false"], default="false")
    ap.add_argument("--batch", type=int, default=1)
    a = ap.parse_args(argv)
    if a.len <= 0 or a.iters <= 0:
        ap.error("--len and --iters must be positive")
    a.branches = max(1, a.branches)
    return a


def make_runner(a, transducer_len):
    kind, gen, op = PLAN[a.scenario]
    data = input_bytes(kind, a.len, a.branches)
    if op == "sp":
        acc = F.MutableFst.compile_string(data)
        return lambda: F.shortest_path(acc, 1).num_states
    rhs = F.Fst.bench_transducer(gen, transducer_len, a.branches)
    if a.batch > 1:
        if op == "compose":
            raise SystemExit("--batch applies to the *_shortest_path scenarios")
        sem = F.FST_SEM_LAZY if op == "lazy" else F.FST_SEM_EAGER
        labels = np.tile(np.frombuffer(data, np.uint8).astype(np.uint32) + 1, a.batch)
        offsets = (np.arange(a.batch + 1, dtype=np.uint64) * len(data)).astype(np.uint64)

        def run_batch():
            r = F.compose_frozen_shortest_path_batch(rhs, labels, offsets, 1, sem)
            ok = r.status == F.FST_PATH_OK
            return int((np.diff(r.offsets)[ok] + 1).sum()) // max(1, a.batch)
        return run_batch
    lhs = F.MutableFst.compile_string(data)
    if op == "compose":
        return lambda: F.compose_frozen(lhs, rhs).num_states
    if op == "lazy":
        return lambda: F.compose_frozen_shortest_path(lhs, rhs, 1).num_states
    return lambda: F.shortest_path(F.compose_frozen(lhs, rhs), 1).num_states


def main(argv=None) -> int:
    a = parse_args(sys.argv[1:] if argv is None else argv)
    if a.scenario in OUT_OF_SCOPE:
        print(f"scenario {a.scenario} is not on the compose_frozen path (see DESIGN.md §0)",
              file=sys.stderr)
        return 2
    transducer_len = max(1, a.len // 4 if a.transducer_len == 0 else a.transducer_len)
    run = make_runner(a, transducer_len)
    for _ in range(a.warmup):
        run()
    total = 0
    lo, hi, states = None, 0, 0
    per_iter = a.per_iter == "true"
    for it in range(a.iters):
        t0 = time.perf_counter_ns()
        st = run()
        ns = time.perf_counter_ns() - t0
        total += ns
        lo = ns if lo is None else min(lo, ns)
        hi = max(hi, ns)
        states += st
        if per_iter:
            if a.format == "json":
                print(json.dumps({"iter": it, "ns": ns, "states": st}, separators=(",", ":")))
            else:
                print(f"iter={it} ns={ns} states={st}")
    avg_ns = total // a.iters
    if a.format == "text":
        print(f"scenario={a.scenario} len={a.len} transducer_len={transducer_len} "
              f"branches={a.branches} warmup={a.warmup} iters={a.iters}")
        print(f"total_ns={total} avg_us={avg_ns / 1e3:.3f} min_ns={lo} max_ns={hi} "
              f"avg_states={states // a.iters}")
        if a.batch > 1:
            print(f"batch={a.batch} strings_per_s={a.batch * 1e9 / avg_ns:.1f}")
    else:
        rec = {"scenario": a.scenario, "len": a.len, "transducer_len": transducer_len,
               "branches": a.branches, "warmup": a.warmup, "iters": a.iters,
               "total_ns": total, "avg_ns": avg_ns, "min_ns": lo, "max_ns": hi,
               "avg_states": states // a.iters}
        if a.batch > 1:
            rec["batch"] = a.batch
            rec["strings_per_s"] = a.batch * 1e9 / avg_ns
        print(json.dumps(rec, separators=(",", ":")))
    return 0


if __name__ == "__main__":
    sys.exit(main())
