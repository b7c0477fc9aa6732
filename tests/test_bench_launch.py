"""bench.py's multi-GPU launch contract (driver: ``bench.py --gpus N``).

* CPU: ``--gpus N`` that disagrees with a launcher's WORLD_SIZE exits 2
  before touching the GPU; ``--gpus N`` started directly with fewer than N
  visible GPUs (and no CEO_BENCH_SHARE_GPU rehearsal) exits 2 -- never a
  silent one-rank run;
* GPU: ``CEO_BENCH_SHARE_GPU=1 bench.py --gpus 2`` spawns two ranks itself
  (both on the test box's GPU, gloo) and rank 0 prints one JSON line with
  n_gpus 2 and the whole job's pairs/s.
"""
import json
import os
import subprocess
import sys

import pytest
import torch

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra, timeout):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra)
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=timeout)


def test_gpus_flag_must_match_launcher_world_size():
    r = _run(["--gpus", "2"], {"WORLD_SIZE": "3", "RANK": "0"}, 120)
    assert r.returncode == 2, r.stderr[-2000:]
    assert "does not match WORLD_SIZE" in r.stderr


def test_gpus_flag_without_enough_devices_fails_loudly():
    if torch.cuda.device_count() >= 8:
        pytest.skip("enough GPUs here: the launch would really run")
    r = _run(["--gpus", "8"], {}, 120)
    assert r.returncode == 2, r.stderr[-2000:]
    assert "GPU(s) visible" in r.stderr
    assert r.stdout.strip() == ""


@pytest.mark.gpu
def test_bench_spawns_ranks_for_gpus_flag():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    r = _run(["--gpus", "2", "--steps", "6", "--warmup", "2", "--no-extras", "--no-cpu-baseline"],
             {"CEO_BENCH_SHARE_GPU": "1"}, 600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2"
    assert res["config"]["global_batch"] == 2 * 16384
    assert res["value"] > 0 and res["steps"] == 6
