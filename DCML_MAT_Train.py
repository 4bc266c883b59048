#!/usr/bin/env python
"""MAT-AS training entry point for DCML (CLI-compatible with the reference ``DCML_MAT_Train.py``).

* Same flags (``mat_dcml_amd/config.py``) and the same default argv as the reference's hard-coded list
  (``DCML_MAT_Train.py:193``) — but real CLI arguments are appended and override it (the reference ignored
  ``sys.argv``), and the malformed ``value_loss_coef 1.5`` pair is dropped with a warning (its effective value
  in the reference is the default 1.0).
* Same run layout: ``<cwd>/results/<env_name>/<scenario>/<algorithm>/<experiment>/run{n}/`` with ``args.txt``,
  ``logs/`` (+ ``summary.json``) and ``models/transformer_{episode}.pt`` (``:116-147,182``).
* Launch one process per GPU for data parallelism::

      python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 DCML_MAT_Train.py --n_workers 32

  (``--n_rollout_threads`` is per rank; the global env set is ``world_size x n_rollout_threads``.)
"""
import os
import sys
from pathlib import Path

import numpy as np
import torch

from mat_dcml_amd.config import get_config, parse_args
from mat_dcml_amd.parallel.comm import init_from_env
from mat_dcml_amd.utils.checkpoint import make_run_dir
from mat_dcml_amd.runner.dcml_runner import DCMLRunner as Runner

DEFAULT_ARGV = ["--n_rollout_threads", "8", "--num_env_steps", "1000000", "--save_interval", "50",
                "--episode_length", "50", "--algorithm_name", "mat", "--env_name", "DCML", "--scenario", "AS",
                "--lr", "5e-5", "--critic_lr", "5e-5", "--ppo_epoch", "15", "--num_mini_batch", "4",
                "--gamma", "0.99", "--use_valuenorm", "--use_popart", "--entropy_coef", "0.01"]

SUPPORTED = ("mat", "mat_dec", "mat_encoder", "mat_decoder", "mat_gru", "momat", "dmomat", "happo", "rmappo", "ppo",
             "ippo", "hatrpo", "random")


def main(args):
    all_args = parse_args(args, get_config())
    if all_args.algorithm_name not in SUPPORTED:
        raise NotImplementedError(all_args.algorithm_name)
    if all_args.algorithm_name == "rmappo":
        all_args.use_recurrent_policy = True
    if all_args.algorithm_name in ("momat", "dmomat"):   # multi-objective MAT: (task completion time, payment)
        all_args.n_objective = max(2, all_args.n_objective)
        all_args.use_advantage_norm = all_args.use_advantage_norm or all_args.algorithm_name == "dmomat"
    if all_args.algorithm_name == "mat_dec":
        all_args.dec_actor = True
        all_args.share_actor = True
    torch.set_num_threads(all_args.n_training_threads)
    comm = init_from_env(prefer_gpu=all_args.cuda)
    device = comm.device
    if comm.is_main:
        print("choose to use gpu..." if device.type == "cuda" else "choose to use cpu...")
    if device.type == "cuda" and all_args.cuda_deterministic:   # reference DCML_MAT_Train.py:108-110
        # the eager torch parts deterministic too; the fused PPO update is bit-reproducible by construction (private
        # gradient workspace, fixed-order reductions: algos/mat_trainer.py, tests/test_gpu_determinism.py)
        torch.backends.cudnn.benchmark = False
        torch.backends.cudnn.deterministic = True
    run_dir = make_run_dir(all_args, comm)
    if comm.is_main:
        with open(run_dir / "args.txt", "w") as f:
            f.write(str(args))
    torch.manual_seed(all_args.seed)
    np.random.seed(all_args.seed)
    all_args.use_centralized_V = True
    config = {"all_args": all_args, "device": device, "run_dir": run_dir, "comm": comm}
    if all_args.algorithm_name in ("mat", "mat_dec", "mat_encoder", "mat_decoder", "mat_gru", "momat", "dmomat"):
        runner = Runner(config)
    else:
        from mat_dcml_amd.runner.baseline_runner import BaselineRunner
        runner = BaselineRunner(config)
    if all_args.resume:
        runner.resume()
    runner.run()
    if runner.heartbeat is not None:
        runner.heartbeat.stop()
    if comm.is_main:
        runner.writter.export_scalars_to_json(os.path.join(runner.log_dir, "summary.json"))
        runner.writter.close()
    comm.destroy()
    return runner


if __name__ == "__main__":
    main(DEFAULT_ARGV + sys.argv[1:])
