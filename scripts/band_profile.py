"""Config 3's band replay alone (no CPU oracle), for rocprofv3 kernel traces and counter
passes: the full rhs (eps_dense T=65,536, B=12) and n strings of config 3's length
distribution (L uniform 11..251, seed 0x5EED), lazy, one warm-up run then one timed.
usage: python scripts/band_profile.py [--n 16384]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts"))
import bench  # noqa: E402
import libfst_amd as F  # noqa: E402
from bench_configs import dev_rhs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--T", type=int, default=65536)
    a = ap.parse_args()
    fz = F.Fst.bench_transducer(F.BENCH_EPS_DENSE, a.T, 12)
    rhs, _ = dev_rhs(fz)
    rng = np.random.default_rng(0x5EED)
    lens = rng.integers(11, 252, a.n)
    b = bench.DeviceBatch(lens, lambda t: torch.ones(t, dtype=torch.int32), "cuda:0",
                          arc_factor=4)
    s = torch.cuda.current_stream().cuda_stream
    b.run(rhs, F.FST_SEM_LAZY, 0, s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    b.run(rhs, F.FST_SEM_LAZY, 0, s)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    st = b.status.cpu().numpy()
    print(json.dumps({"n": a.n, "T": a.T, "wall_s": wall, "strings_per_s": a.n / wall,
                      "ok": int((st == 0).sum()), "mean_len": float(lens.mean())}), flush=True)


if __name__ == "__main__":
    main()
