#!/usr/bin/env python
"""MAT on multi-agent MuJoCo with faulty-node injection (CLI-compatible with
``mat_src/mat/scripts/train/train_mujoco.py``; defaults from ``train_mujoco.sh``).

The robots run on the device-batched planar surrogate of ``mat_dcml_amd/envs/mujoco`` (MuJoCo is not installable
here); partitions, observation layouts, rewards and the faulty-node protocol follow the reference::

    python train_mujoco.py --scenario HalfCheetah-v2 --agent_conf 6x1 --faulty_node -1 --eval_faulty_node -1 0 1
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 train_mujoco.py --n_rollout_threads 320
"""
import os
import sys

import numpy as np
import torch

from mat_dcml_amd.config import _MUJOCO_FLAGS, get_config, parse_args
from mat_dcml_amd.parallel.comm import init_from_env
from mat_dcml_amd.runner.mujoco_runner import MujocoRunner
from mat_dcml_amd.utils.checkpoint import make_run_dir

# train_mujoco.sh
DEFAULT_ARGV = ["--env_name", "mujoco", "--algorithm_name", "mat", "--experiment_name", "single",
                "--scenario", "HalfCheetah-v2", "--agent_conf", "6x1", "--agent_obsk", "0", "--faulty_node", "-1",
                "--eval_faulty_node", "-1", "--critic_lr", "5e-5", "--lr", "5e-5", "--entropy_coef", "0.001",
                "--max_grad_norm", "0.5", "--eval_episodes", "5", "--n_training_threads", "16",
                "--n_rollout_threads", "40", "--num_mini_batch", "40", "--episode_length", "100",
                "--eval_interval", "25", "--num_env_steps", "10000000", "--ppo_epoch", "10", "--clip_param", "0.05",
                "--use_eval", "--add_center_xy", "--use_state_agent", "--use_value_active_masks",
                "--use_policy_active_masks"]


def parse(argv):
    parser = get_config()
    parser.add_argument("--eval_faulty_node", type=int, nargs="+", default=None)
    return parse_args(argv, parser, extra=_MUJOCO_FLAGS)


def main(argv):
    all_args = parse(argv)
    comm = init_from_env(prefer_gpu=all_args.cuda)
    run_dir = make_run_dir(all_args, comm)
    if comm.is_main:
        with open(run_dir / "args.txt", "w") as f:
            f.write(str(argv))
    torch.manual_seed(all_args.seed)
    np.random.seed(all_args.seed)
    runner = MujocoRunner({"all_args": all_args, "device": comm.device, "run_dir": run_dir, "comm": comm})
    runner.run()
    if comm.is_main:
        runner.writter.export_scalars_to_json(os.path.join(runner.log_dir, "summary.json"))
        runner.writter.close()
    comm.destroy()
    return runner


if __name__ == "__main__":
    main(DEFAULT_ARGV + sys.argv[1:])
