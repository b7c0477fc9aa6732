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


def _json(r):
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, (r.stdout[-2000:], r.stderr[-3000:])
    return json.loads(lines[0])


def _port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return str(s.getsockname()[1])


@pytest.mark.gpu
def test_bench_dp_world1_on_rccl_and_on_the_peer_exchange():
    """The driver's ``--gpus 8`` path at world 1 on the test box: RCCL init
    (``backend="nccl"``), the data-parallel step with the RCCL all-reduce
    captured into the hipGraph chunks (CEO_TT_PEER_AR=0, the fallback the
    8-GPU run takes if the peer exchange loses its checks), and the peer
    exchange's own setup (its collective check, then the in-reduction form
    chosen by bits and timing, both timings reported).  Each run's mean loss
    equals the single-GPU run's (training.py:54-55 under DDP at world 1 is
    the plain step)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    args = ["--gpus", "1", "--steps", "8", "--warmup", "2", "--no-extras", "--no-cpu-baseline"]
    # the fewest warm replays (one chunk): the mean losses compared below are
    # of a ~20-step trajectory, not of 200+ steps over which the float-atomic
    # order's rounding noise (different in every run) has grown
    warm = {"CEO_BENCH_WARM_STEPS": "0"}
    single = _json(_run(args, dict(warm), 600))
    rccl_run = _run(args + ["--dp"], {"CEO_TT_PEER_AR": "0", "MASTER_PORT": _port(), **warm}, 600)
    assert rccl_run.returncode == 0, rccl_run.stderr[-3000:]
    rccl = _json(rccl_run)
    peer_run = _run(args + ["--dp"], {"MASTER_PORT": _port(), **warm}, 600)
    assert peer_run.returncode == 0, peer_run.stderr[-3000:]
    peer = _json(peer_run)
    assert single["config"]["parallelism"] == "single"
    assert rccl["config"]["parallelism"] == "dp1" and peer["config"]["parallelism"] == "dp1"
    assert rccl["config"]["grad_exchange"] == "rccl all-reduce", rccl["config"]
    assert rccl["config"]["graph"] is True  # the RCCL all-reduce captured with the kernels
    assert peer["config"]["grad_exchange"].startswith("peer-memory"), peer["config"]
    ft = peer["config"]["fused_vs_two_launch_us"]
    assert ft is not None and all(0 < t < 1e4 for t in ft), ft
    for res in (rccl, peer):
        assert abs(res["mean_loss"] - single["mean_loss"]) <= 1e-5 * abs(single["mean_loss"]) + 1e-5, \
            (res["mean_loss"], single["mean_loss"])
    print("rccl dp1", rccl["ms_per_step"], "peer dp1", peer["ms_per_step"], peer["config"]["grad_exchange"], ft,
          "single", single["ms_per_step"])
