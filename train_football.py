#!/usr/bin/env python
"""MAT on Google Research Football (CLI-compatible with ``mat_src/mat/scripts/train/train_football.py``; defaults
from ``train_football.sh``).

The matches run on the device-batched ``SyntheticFootballEnv`` (gfootball is not installable here) with the
reference's observation / availability / reward encoders::

    python train_football.py --scenario academy_3_vs_1_with_keeper --n_agent 3
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 train_football.py --n_rollout_threads 160
"""
import os
import sys

import numpy as np
import torch

from mat_dcml_amd.config import _FOOTBALL_FLAGS, get_config, parse_args
from mat_dcml_amd.parallel.comm import init_from_env
from mat_dcml_amd.runner.football_runner import FootballRunner
from mat_dcml_amd.utils.checkpoint import make_run_dir

# train_football.sh
DEFAULT_ARGV = ["--env_name", "football", "--algorithm_name", "mat", "--experiment_name", "single",
                "--scenario", "academy_3_vs_1_with_keeper", "--n_agent", "3", "--seed", "1", "--lr", "5e-4",
                "--entropy_coef", "0.01", "--max_grad_norm", "0.5", "--eval_episodes", "32",
                "--n_training_threads", "16", "--n_rollout_threads", "20", "--num_mini_batch", "1",
                "--episode_length", "200", "--eval_interval", "25", "--num_env_steps", "10000000", "--ppo_epoch", "10",
                "--clip_param", "0.05", "--use_eval", "--use_value_active_masks", "--use_policy_active_masks"]


def main(argv):
    all_args = parse_args(argv, get_config(), extra=_FOOTBALL_FLAGS)
    comm = init_from_env(prefer_gpu=all_args.cuda)
    run_dir = make_run_dir(all_args, comm)
    if comm.is_main:
        with open(run_dir / "args.txt", "w") as f:
            f.write(str(argv))
    torch.manual_seed(all_args.seed)
    np.random.seed(all_args.seed)
    runner = FootballRunner({"all_args": all_args, "device": comm.device, "run_dir": run_dir, "comm": comm})
    runner.run()
    if comm.is_main:
        runner.writter.export_scalars_to_json(os.path.join(runner.log_dir, "summary.json"))
        runner.writter.close()
    comm.destroy()
    return runner


if __name__ == "__main__":
    main(DEFAULT_ARGV + sys.argv[1:])
