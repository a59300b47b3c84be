"""bench.py plumbing on CPU: `--gpus N` self-launching (one rank per GPU through
torch.distributed.run), the loud failure without enough devices, and the
roofline pricing of the training step."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _run(args, env_extra, timeout=240):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", **env_extra)
    env.pop("WORLD_SIZE", None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          env=env, timeout=timeout, cwd=ROOT)


def test_gpus2_self_launches_two_ranks():
    r = _run(["--gpus", "2", "--steps", "3", "--warmup", "1", "--dry-run"], {"DF_DIST_BACKEND": "gloo"})
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout           # rank 0 prints ONE line
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 3 and out["warmup"] == 1 and out["dry_run"] is True


def test_gpus2_without_devices_fails_loudly():
    import torch

    if torch.cuda.device_count() >= 2:
        pytest.skip("this host has two GPUs")
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"], {"DF_DIST_BACKEND": "nccl"})
    assert r.returncode != 0
    assert "GPU(s) visible" in (r.stderr + r.stdout)
    assert '"n_gpus": 1' not in r.stdout


def test_train_split_flops_pricing():
    import bench

    cfg2 = bench.build_chain("cfg2")
    # 16 nets (in 2/3, hidden 64, out 3/2): forward first + hidden Dense, and the hidden
    # Dense's W1ᵀδ and dW1 on the split products
    hidden = 16 * 2 * 64 * 64
    first = sum(2 * D.in_dim * D.out_dim for e in cfg2 for L in (e.layer_1, e.layer_2)
                for net in (L.s_net, L.t_net) for D in net[:1])
    assert bench.train_split_flops(cfg2, 4) == first + 3 * hidden
    assert bench.train_split_flops(cfg2, 3) == 0.0
    cfg4 = bench.build_chain("cfg4")
    per_net = 2 * (24 * 256 + 256 * 256 + 256 * 16) + 2 * 2 * 256 * 256
    assert bench.train_split_flops(cfg4, 6) == 32 * per_net


def test_gpus8_dry_run_reports_every_rank():
    """the 1→8 run is self-diagnosing — 8 ranks launched by
    bench.py itself (gloo on CPU), rank 0 reports n_gpus 8 and the per-rank
    timing spread gathered from all 8."""
    r = _run(["--gpus", "8", "--steps", "2", "--warmup", "1", "--dry-run"], {"DF_DIST_BACKEND": "gloo"},
             timeout=400)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["dry_run"] is True
    ranks = out["ranks"]
    assert ranks["n"] == 8 and ranks["group_size"] == 8 and len(ranks["kernel_ms_per_rank"]) == 8
    assert ranks["wall_ms_per_step_min"] <= ranks["wall_ms_per_step_max"]
    assert ranks["process_group"] == "torch.distributed gloo"
