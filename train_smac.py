#!/usr/bin/env python
"""MAT on SMAC (CLI-compatible with ``mat_src/mat/scripts/train/train_smac.py``; flags as in ``train_smac.sh``).

Default map 27m_vs_30m (BASELINE config #5).  Without StarCraft II the env is the on-device SMAC-shaped synthetic
env (``--smac_backend synthetic``, the default); multi-GPU data parallelism as for DCML::

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 train_smac.py --n_rollout_threads 32
"""
import os
import sys

import numpy as np
import torch

from mat_dcml_amd.config import _SMAC_FLAGS, get_config, parse_args
from mat_dcml_amd.parallel.comm import init_from_env
from mat_dcml_amd.utils.checkpoint import make_run_dir
from mat_dcml_amd.runner.smac_runner import SMACRunner

DEFAULT_ARGV = ["--env_name", "StarCraft2", "--algorithm_name", "mat", "--experiment_name", "single",
                "--seed", "1", "--n_rollout_threads", "32", "--num_mini_batch", "1", "--episode_length", "100",
                "--num_env_steps", "10000000", "--lr", "5e-4", "--ppo_epoch", "15", "--clip_param", "0.05",
                "--save_interval", "100000", "--use_value_active_masks", "--use_eval"]


def main(argv):
    all_args = parse_args(argv, get_config(), extra=_SMAC_FLAGS)
    all_args.scenario = all_args.map_name
    comm = init_from_env(prefer_gpu=all_args.cuda)
    run_dir = make_run_dir(all_args, comm)
    if comm.is_main:
        with open(run_dir / "args.txt", "w") as f:
            f.write(str(argv))
    torch.manual_seed(all_args.seed)
    np.random.seed(all_args.seed)
    runner = SMACRunner({"all_args": all_args, "device": comm.device, "run_dir": run_dir, "comm": comm})
    runner.run()
    if comm.is_main:
        runner.writter.export_scalars_to_json(os.path.join(runner.log_dir, "summary.json"))
        runner.writter.close()
    comm.destroy()
    return runner


if __name__ == "__main__":
    main(DEFAULT_ARGV + sys.argv[1:])
