"""Is the bench iteration host-bound?  Host enqueue time of the rollout and of the PPO update (perf_counter without a
synchronize) against their device time, at the bench config (32 workers, 256 envs x 50 steps, 15 x 4 minibatches).
If the host time of a phase approaches its device time, the GPU idles waiting for launches.

    python scripts/host_bound_diag.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from mat_dcml_amd.config import get_config, parse_args
    from mat_dcml_amd.parallel.comm import Comm
    from mat_dcml_amd.runner.dcml_runner import DCMLRunner
    dev = torch.device("cuda:0")
    argv = ["--env_name", "DCML", "--scenario", "AS", "--algorithm_name", "mat", "--n_rollout_threads", "256",
            "--episode_length", "50", "--lr", "5e-5", "--ppo_epoch", "15", "--num_mini_batch", "4", "--gamma", "0.99",
            "--use_valuenorm", "--use_popart", "--entropy_coef", "0.01", "--n_workers", "32", "--seed", "1"]
    args = parse_args(argv, get_config(), warn=False)
    r = DCMLRunner({"all_args": args, "device": dev, "run_dir": None, "comm": Comm(device=dev)})
    r.warmup()
    for _ in range(2):
        r.train_iteration()
    torch.cuda.synchronize()
    for it in range(3):
        t0 = time.perf_counter()
        r.rollout()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        r.compute()
        r.train()
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        print(f"iter {it}: rollout host {1e3 * (t1 - t0):.2f} ms, rollout until idle {1e3 * (t2 - t0):.2f} ms; "
              f"update host {1e3 * (t3 - t2):.2f} ms, update until idle {1e3 * (t4 - t2):.2f} ms", flush=True)


def profile_rollout():
    """cProfile of the rollout's host side (top functions by own time)."""
    import cProfile
    import pstats
    from mat_dcml_amd.config import get_config, parse_args
    from mat_dcml_amd.parallel.comm import Comm
    from mat_dcml_amd.runner.dcml_runner import DCMLRunner
    dev = torch.device("cuda:0")
    argv = ["--env_name", "DCML", "--scenario", "AS", "--algorithm_name", "mat", "--n_rollout_threads", "256",
            "--episode_length", "50", "--use_valuenorm", "--use_popart", "--n_workers", "32", "--seed", "1"]
    args = parse_args(argv, get_config(), warn=False)
    r = DCMLRunner({"all_args": args, "device": dev, "run_dir": None, "comm": Comm(device=dev)})
    r.warmup()
    r.rollout()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(4):
        r.rollout()
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
    if "--profile" in sys.argv:
        profile_rollout()
