"""bench.py multi-rank contract and the kernel-path report (item 9), on CPU.

* ``python bench.py --gpus 2`` with no launcher starts two rank processes itself (gloo here) and reports two
  distinct ranks / devices;
* a launch whose WORLD_SIZE disagrees with ``--gpus`` fails instead of benchmarking the wrong node size;
* under RCCL (``nccl``) a rank without its own GPU is an error; GPU sharing is an explicit gloo-only opt-in.
"""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--steps", "1", "--warmup", "0", "--envs", "4", "--episode_length", "2", "--n_workers", "4", "--ppo_epoch",
         "1", "--num_mini_batch", "1", "--no_eval"]


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="1", **kw)
    return env


def test_bench_self_launches_two_ranks():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", *SMALL], cwd=ROOT, env=_env(), capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 prints ONE JSON line
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["ranks"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["backend"] == "gloo" and len(set(out["rank_devices"])) == 2
    assert out["config"]["global_batch"] == 8
    assert set(out["kernels"]) >= {"env", "encoder", "decode", "train", "gae"}
    # scaling diagnostics: per-rank ms per step and critical-path collective time per step
    assert len(out["rank_ms_per_step"]) == 2 and all(t > 0 for t in out["rank_ms_per_step"])
    assert max(out["rank_ms_per_step"]) <= out["ms_per_step"] * 1.001
    cm = out["comm_ms_per_step"]
    assert cm["grad_allreduce"] > 0 and cm["stats_allreduce"] > 0
    assert cm["grad_allreduce"] + cm["stats_allreduce"] < out["ms_per_step"]
    # SMALL = 1 epoch x 1 minibatch: one gradient average and one epoch-statistics all-reduce per step
    assert out["collectives_per_step"] == {"grad_allreduce": 1, "stats_allreduce": 1}
    # phase breakdown: separate instrumented steps after the uninstrumented timed
    # loop, every phase occurrence timed (nothing sampled / scaled): the rollout phases + update partition the step
    ph = out["phase_ms_per_step"]
    assert {"pack", "decode", "env", "insert", "update", "train_fwd", "train_bwd"} <= set(ph)
    assert all(v > 0 for v in ph.values())
    assert ph["train_fwd"] + ph["train_bwd"] <= ph["update"]
    run = out["phase_run"]
    top = sum(ph[k] for k in ("pack", "decode", "env", "insert", "update"))
    assert abs(run["phases_sum_ms"] - top) < 0.01
    assert top <= 1.02 * run["ms_per_step"]
    tk = out["train_kernels_ms_per_minibatch"]
    assert set(tk) == {"fwd", "bwd"} and abs(tk["fwd"] - ph["train_fwd"]) < 1e-2   # 1 epoch x 1 minibatch


def test_bench_rejects_world_size_mismatch():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", *SMALL], cwd=ROOT,
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "does not match" in r.stderr


@pytest.mark.parametrize("backend,share", [("nccl", "0"), ("nccl", "1"), ("gloo", "0")])
def test_rank_without_own_gpu_fails_loudly(monkeypatch, backend, share):
    from mat_dcml_amd.parallel import comm as C
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "1")
    monkeypatch.setenv("LOCAL_RANK", "1")
    monkeypatch.setenv("MAT_DCML_DIST_BACKEND", backend)
    monkeypatch.setenv("MAT_DCML_SHARE_DEVICES", share)
    with pytest.raises(RuntimeError, match="needs one GPU per rank"):
        C.init_from_env(prefer_gpu=True)


def test_bench_four_ranks_full_update_schedule():
    """``bench.py --gpus 4`` end to end through launch_ranks (gloo), with the reference's PPO
    schedule (15 epochs x 4 minibatches): 60 gradient averages and 15 epoch-statistics all-reduces per step, every
    rank timed."""
    args = ["--steps", "1", "--warmup", "0", "--envs", "8", "--episode_length", "2", "--n_workers", "4",
            "--ppo_epoch", "15", "--num_mini_batch", "4", "--no_eval", "--no_phase_timers"]
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4", *args], cwd=ROOT, env=_env(), capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["ranks"] == 4 and out["n_gpus"] == 4 and out["config"]["parallelism"] == "dp4"
    assert out["collectives_per_step"] == {"grad_allreduce": 60, "stats_allreduce": 15}
    assert len(out["rank_ms_per_step"]) == 4 and all(0 < t <= out["ms_per_step"] * 1.001 for t in out["rank_ms_per_step"])
    assert out["config"]["global_batch"] == 32
    assert "phase_ms_per_step" not in out
