#!/usr/bin/env python
"""Headline benchmark: MAT-AS PPO training throughput on 32-worker DCML (BASELINE.json).

One "step" = one full PPO iteration of the reference training loop (``dcml_runner.py:39-91``): a T=50-step
stochastic rollout over the rank's 256 vectorised envs (encoder + autoregressive MAT decode + env step per
step) followed by the complete MAT-PPO update (15 epochs x 4 minibatches, next-value + GAE recomputed each
epoch, clip / Huber / ValueNorm / grad clip / Adam, gradient all-reduce under DP).  Nothing is skipped inside
the timed region.  Weak scaling: every rank owns 256 envs, so the node runs 256·N envs.

    python bench.py --gpus 1 --steps 5 --warmup 2
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29500 \
        bench.py --gpus 8 --steps 5 --warmup 2

Rank 0 prints ONE JSON line; ``value`` = whole-node env-steps/s (max time over ranks).
Baseline = 43 env-steps/s: the reference itself on the 32-worker config (CPU, measured).
"""
import argparse
import json
import os
import sys
import time

import torch

BASELINE_ENV_STEPS_PER_S = 43.0
METRIC = "env-steps/sec (whole node) MAT-AS 32-worker DCML at 1/2/4/8 GPU; eval task time"


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--n_workers", type=int, default=32)
    p.add_argument("--envs", type=int, default=256, help="vectorised envs per GPU")
    p.add_argument("--episode_length", type=int, default=50)
    p.add_argument("--kernels", default="auto")
    p.add_argument("--dtype", default="bf16")
    p.add_argument("--phases", action="store_true")
    a = p.parse_args()

    from mat_dcml_amd.config import get_config, parse_args
    from mat_dcml_amd.parallel.comm import init_from_env
    from mat_dcml_amd.runner.dcml_runner import DCMLRunner

    comm = init_from_env(prefer_gpu=True)
    argv = ["--env_name", "DCML", "--scenario", "AS", "--algorithm_name", "mat", "--n_rollout_threads", str(a.envs),
            "--episode_length", str(a.episode_length), "--lr", "5e-5", "--ppo_epoch", "15", "--num_mini_batch", "4",
            "--gamma", "0.99", "--use_valuenorm", "--use_popart", "--entropy_coef", "0.01",
            "--n_workers", str(a.n_workers), "--kernels", a.kernels, "--dtype", a.dtype, "--seed", "1"]
    if a.phases:
        argv.append("--profile_phases")
    args = parse_args(argv, get_config(), warn=False)
    runner = DCMLRunner({"all_args": args, "device": comm.device, "run_dir": None, "comm": comm})
    runner.warmup()
    dev = comm.device

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    for _ in range(a.warmup):
        runner.train_iteration()
    if a.phases:
        runner.timers.summary()
    sync()
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        runner.train_iteration()
    sync()
    comm.barrier()
    sync()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    comm.all_reduce_max_(t)
    dt = float(t)
    n = comm.world_size
    env_steps = a.steps * a.episode_length * a.envs * n
    value = env_steps / dt
    if comm.is_main:
        if a.phases:
            print(runner.timers.summary(), file=sys.stderr)
        print(json.dumps({
            "metric": METRIC, "value": round(value, 2), "unit": "env-steps/s", "n_gpus": n, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": round(value / BASELINE_ENV_STEPS_PER_S, 2),
            "dtype": a.dtype if dev.type == "cuda" else "fp32",
            "data": "synthetic (on-device DCML env simulation, Philox streams; random-init MAT weights)",
            "config": {"model": f"MAT (2+2 blocks, d=64, 2 heads) on DCML {a.n_workers}-worker bid-first env "
                                f"({a.n_workers + 1} agents)",
                       "global_batch": a.envs * n, "seq_len": a.n_workers + 1,
                       "parallelism": f"dp{n}", "envs_per_gpu": a.envs, "episode_length": a.episode_length,
                       "ppo_epoch": 15, "num_mini_batch": 4, "kernels": a.kernels,
                       "device": torch.cuda.get_device_name(dev) if dev.type == "cuda" else "cpu"},
        }), flush=True)
    comm.destroy()


if __name__ == "__main__":
    main()
