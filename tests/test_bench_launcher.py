"""bench.py's multi-GPU launch contract, rehearsed on CPU with gloo
(`--gpus N` must start N ranks; the driver's
`python bench.py --gpus N` is a plain process).

* `--gpus 2` without WORLD_SIZE: the parent starts torch.distributed.run with
  2 workers as a child (never touching a GPU itself); the workers rendezvous on
  127.0.0.1, all-gather per-rank top-k-shaped tensors and take the max over
  ranks; rank 0 prints one JSON line with n_gpus = 2 and the world size seen.
* `--gpus 1`: one process, no launcher.
* WORLD_SIZE disagreeing with --gpus: exit code 2 with the launch command.
"""
import json
import os
import subprocess
import sys

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    env.update(env_extra or {})
    env["OMP_NUM_THREADS"] = "1"
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout, env=env)


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def test_gpus2_spawns_two_ranks():
    r = _run(["--gpus", "2", "--dry-run", "--steps", "1", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    assert lines[0]["n_gpus"] == 2 and lines[0]["world_size_seen"] == 2 and lines[0]["gather_ok"]


def test_gpus1_single_process():
    r = _run(["--gpus", "1", "--dry-run"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1 and lines[0]["n_gpus"] == 1 and lines[0]["world_size_seen"] == 1


def test_world_size_mismatch_is_an_error():
    r = _run(["--gpus", "4", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "torch.distributed.run" in r.stderr
