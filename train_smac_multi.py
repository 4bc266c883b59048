#!/usr/bin/env python
"""Multi-map MAT on SMAC (CLI-compatible with ``mat_src/mat/scripts/train/train_smac_multi.py``; defaults from
``train_smac_multi.sh``): unified 27-agent / 2029-feature / 38-action layout with task embeddings
(``envs/smac/multi.py``), envs split evenly over ``--train_maps``."""
import sys

import train_smac

MAPS = ["3s_vs_3z", "3s_vs_4z", "3m", "MMM", "3s5z", "8m_vs_9m", "25m", "10m_vs_11m", "2s3z"]
DEFAULT_ARGV = ["--env_name", "StarCraft2_multi", "--algorithm_name", "mat", "--experiment_name", "multi_task",
                "--train_maps", *MAPS, "--eval_maps", *MAPS, "--seed", "1", "--n_eval_rollout_threads", "36",
                "--n_rollout_threads", "36", "--num_mini_batch", "1", "--episode_length", "100",
                "--num_env_steps", "10000000", "--lr", "5e-4", "--ppo_epoch", "10", "--clip_param", "0.05",
                "--use_value_active_masks", "--use_eval", "--map_name", "multi"]


def main(argv):
    return train_smac.main(argv)


if __name__ == "__main__":
    main(DEFAULT_ARGV + sys.argv[1:])
