"""A/B timing of kernel variants on the metric shape (timing only, no oracle check).

usage: python scripts/lazy_ab.py [--sem lazy|eager] [--batch N] variant.so ...
Each variant runs in its own child process (LIBFST_AMD_LIB=...), 1 warm-up + 3 timed steps on
1^64 strings against the ambiguous T=4096 B=12 rhs; prints one JSON line per variant with the
mean kernel time (HIP events on the launch stream) and the status counts of the last step.
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(sem_name, batch):
    import numpy as np
    import torch
    sys.path.insert(0, REPO)
    import bench
    import libfst_amd as F
    from libfst_amd import dist as D

    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    sem = F.FST_SEM_LAZY if sem_name == "lazy" else F.FST_SEM_EAGER
    blob = D.blob_bytes(F.Fst.bench_transducer(F.BENCH_AMBIGUOUS, 4096, 12))
    rhs = D.adopt_on_device(torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev), 0)
    b = bench.DeviceBatch(np.full(batch, 64, np.int64), lambda t: torch.ones(t, dtype=torch.int32), dev)
    el, kms, st = bench.timed(b, rhs, sem, 0, 3, 1, 1)
    u, c = np.unique(b.status.cpu().numpy(), return_counts=True)
    print(json.dumps({"lib": os.environ.get("LIBFST_AMD_LIB", "default"), "sem": sem_name,
                      "kernel_ms": float(np.mean(kms)), "strings_per_s": batch * 3 / el,
                      "status": {int(k): int(v) for k, v in zip(u, c)}}), flush=True)


def main():
    args = sys.argv[1:]
    sem, batch = "lazy", 1 << 20
    libs = []
    i = 0
    while i < len(args):
        if args[i] == "--sem":
            sem = args[i + 1]; i += 2
        elif args[i] == "--batch":
            batch = int(args[i + 1]); i += 2
        else:
            libs.append(args[i]); i += 1
    if os.environ.get("LAZY_AB_CHILD"):
        child(sem, batch)
        return
    for lib in libs:
        env = dict(os.environ, LAZY_AB_CHILD="1", LIBFST_AMD_LIB=os.path.abspath(lib))
        r = subprocess.run([sys.executable, __file__, "--sem", sem, "--batch", str(batch)],
                           env=env, timeout=300)
        if r.returncode != 0:
            print(json.dumps({"lib": lib, "rc": r.returncode}), flush=True)
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
