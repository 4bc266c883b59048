#!/usr/bin/env python
"""MAT on MPE (CLI-compatible with ``mat_src/mat/scripts/train/train_mpe.py``; defaults from ``train_mpe.sh``).

All nine reference scenarios run on the on-device ``MPEVecEnv``; multi-GPU data parallelism as for DCML::

    python train_mpe.py --scenario_name simple_spread --num_agents 3 --num_landmarks 3
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 train_mpe.py --n_rollout_threads 1024
"""
import os
import sys

import numpy as np
import torch

from mat_dcml_amd.config import _MPE_FLAGS, get_config, parse_args
from mat_dcml_amd.parallel.comm import init_from_env
from mat_dcml_amd.utils.checkpoint import make_run_dir
from mat_dcml_amd.runner.mpe_runner import MPERunner

# train_mpe.sh (the reference passes --use_ReLU/--gain/--critic_lr for its baselines; MAT ignores them)
DEFAULT_ARGV = ["--env_name", "MPE", "--algorithm_name", "mat", "--experiment_name", "single",
                "--scenario_name", "simple_spread", "--num_agents", "3", "--num_landmarks", "3", "--seed", "1",
                "--n_block", "1", "--n_embd", "64", "--n_rollout_threads", "128", "--num_mini_batch", "1",
                "--episode_length", "25", "--num_env_steps", "20000000", "--ppo_epoch", "10", "--clip_param", "0.05",
                "--use_ReLU", "--gain", "0.01", "--lr", "7e-4", "--critic_lr", "7e-4", "--use_eval"]


def main(argv):
    all_args = parse_args(argv, get_config(), extra=_MPE_FLAGS)
    all_args.scenario = all_args.scenario_name
    comm = init_from_env(prefer_gpu=all_args.cuda)
    run_dir = make_run_dir(all_args, comm)
    if comm.is_main:
        with open(run_dir / "args.txt", "w") as f:
            f.write(str(argv))
    torch.manual_seed(all_args.seed)
    np.random.seed(all_args.seed)
    runner = MPERunner({"all_args": all_args, "device": comm.device, "run_dir": run_dir, "comm": comm})
    if all_args.use_render:   # render_mpe: deterministic episodes of a (restored, --model_dir) policy -> gifs/
        runner.render()
    else:
        runner.run()
    if comm.is_main:
        runner.writter.export_scalars_to_json(os.path.join(runner.log_dir, "summary.json"))
        runner.writter.close()
    comm.destroy()
    return runner


if __name__ == "__main__":
    main(DEFAULT_ARGV + sys.argv[1:])
