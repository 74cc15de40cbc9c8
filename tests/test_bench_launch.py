"""bench.py's rank topology (CPU): `--gpus N` without a launcher starts torchrun with N ranks
as a child process (the driver's 1/2/4/8-GPU runs call `python bench.py --gpus N` directly),
and a WORLD_SIZE that disagrees with --gpus is refused before anything touches a GPU."""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
BENCH = os.path.join(os.path.dirname(HERE), "bench.py")


def _run(args, env_extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True,
                          text=True, timeout=120)


def test_gpus_n_launches_n_ranks():
    r = _run(["--gpus", "4", "--steps", "3", "--warmup", "1"], {"FSTAMD_BENCH_DRY_LAUNCH": "1"})
    assert r.returncode == 0, r.stderr[-2000:]
    cmd = json.loads(r.stdout.strip().splitlines()[-1])["launch"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd
    assert cmd[-6:] == ["--gpus", "4", "--steps", "3", "--warmup", "1"]
    assert os.path.samefile(cmd[-7], BENCH)


def test_world_size_mismatch_is_refused():
    r = _run(["--gpus", "2"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=3 but --gpus 2" in r.stderr
    r = _run(["--gpus", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
