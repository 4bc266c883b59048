"""Flag-compatible configuration.

Every flag of the reference's ``get_config()`` (``mat_src/mat/config.py:156-315``) and of the DCML entry's
``parse_args`` (``DCML_MAT_Train.py:61-78``) parses here with the same name, type and default, including the
inverted ``store_false`` booleans (``--cuda``, ``--use_huber_loss``, ``--use_valuenorm`` is store_true, …), so
every reference argv still works.  New MI355X-side flags are grouped under "framework".

Differences: ``parse`` uses ``parse_known_args`` like the reference but *warns* about dropped
tokens instead of silently ignoring them (the reference argv's ``value_loss_coef 1.5`` typo, §2.7 #5).
"""
from __future__ import annotations

import argparse
import sys

T, F = True, False

# (name, kind, default, help) — kind: type object, "true" (store_true) or "false" (store_false)
_FLAGS = [
    # prepare
    ("algorithm_name", str, "mat", "mat|mat_dec|mat_encoder|mat_decoder|mat_gru|momat|happo|rmappo|random|hatrpo|ppo|ippo"),
    ("experiment_name", str, "check", "identifier of the experiment"),
    ("seed", int, 1, "random seed for torch / env Philox streams"),
    ("cuda", "false", T, "use the GPU (store_false, as in the reference)"),
    ("cuda_deterministic", "false", T, "deterministic kernels (store_false, as in the reference)"),
    ("n_training_threads", int, 1, "torch CPU threads"),
    ("n_rollout_threads", int, 10, "parallel training envs (per rank)"),
    ("n_eval_rollout_threads", int, 1, "parallel eval envs"),
    ("n_render_rollout_threads", int, 1, "parallel render envs"),
    ("n_objective", int, 1, "number of objectives (multi-objective MAT)"),
    ("num_env_steps", float, 7e5, "total env steps to train"),
    ("user_name", str, "xxx", "wandb user"),
    ("use_wandb", "true", F, "log to wandb (unavailable offline; falls back to the local writer)"),
    # env
    ("env_name", str, "StarCraft2", "environment name"),
    ("use_obs_instead_of_state", "true", F, "use concatenated obs as state"),
    # buffer
    ("episode_length", int, 200, "rollout length T"),
    # network
    ("share_policy", "false", T, "agents share a policy"),
    ("use_centralized_V", "false", T, "centralised value function"),
    ("stacked_frames", int, 1, "stacked frames"),
    ("use_stacked_frames", "true", F, "use stacked frames"),
    ("hidden_size", int, 64, "hidden width of baseline actor/critic nets"),
    ("layer_N", int, 2, "layers of baseline actor/critic nets"),
    ("use_ReLU", "false", T, "ReLU in baseline nets"),
    ("use_popart", "true", F, "PopArt value normalisation"),
    ("use_advantage_norm", "true", F, "normalised-value advantages (DMO buffer)"),
    ("use_valuenorm", "true", F, "running mean/std value normalisation"),
    ("use_feature_normalization", "false", T, "LayerNorm on inputs of baseline nets"),
    ("use_orthogonal", "false", T, "orthogonal init"),
    ("gain", float, 0.01, "gain of the last action layer"),
    # recurrent
    ("use_naive_recurrent_policy", "true", F, "naive recurrent policy"),
    ("use_recurrent_policy", "true", F, "recurrent policy"),
    ("recurrent_N", int, 1, "recurrent layers"),
    ("data_chunk_length", int, 10, "recurrent chunk length"),
    # optimizer
    ("lr", float, 1e-3, "learning rate"),
    ("critic_lr", float, 5e-4, "critic learning rate (baselines)"),
    ("opti_eps", float, 1e-5, "Adam epsilon"),
    ("weight_decay", float, 0.0, "weight decay"),
    ("std_x_coef", float, 1.0, "std x coef"),
    ("std_y_coef", float, 0.5, "std y coef"),
    # trpo
    ("kl_threshold", float, 0.01, "HATRPO KL threshold"),
    ("ls_step", int, 10, "HATRPO line-search steps"),
    ("accept_ratio", float, 0.5, "HATRPO accept ratio"),
    # ppo
    ("ppo_epoch", int, 15, "PPO epochs"),
    ("use_clipped_value_loss", "false", T, "clip the value loss"),
    ("clip_param", float, 0.2, "PPO clip"),
    ("num_mini_batch", int, 4, "PPO minibatches"),
    ("entropy_coef", float, 0.01, "entropy coefficient"),
    ("value_loss_coef", float, 1.0, "value loss coefficient"),
    ("use_max_grad_norm", "false", T, "clip gradients"),
    ("max_grad_norm", float, 10.0, "max gradient norm"),
    ("use_gae", "false", T, "GAE"),
    ("gamma", float, 0.99, "discount"),
    ("gae_lambda", float, 0.95, "GAE lambda"),
    ("use_proper_time_limits", "true", F, "time-limit aware returns"),
    ("use_huber_loss", "false", T, "Huber value loss"),
    ("use_value_active_masks", "false", T, "mask the value loss"),
    ("use_policy_active_masks", "false", T, "mask the policy loss"),
    ("use_actor_masks", "true", F, "mask disabled actors"),
    ("huber_delta", float, 10.0, "Huber delta"),
    # run
    ("use_linear_lr_decay", "true", F, "linear LR decay"),
    ("use_cent_local_observe", "true", F, "(reference flag, unused)"),
    ("save_interval", int, 100, "episodes between checkpoints"),
    ("log_interval", int, 5, "episodes between logs"),
    ("use_eval", "true", F, "evaluate during training"),
    ("eval_interval", int, 25, "episodes between evaluations"),
    ("eval_episodes", int, 32, "episodes per evaluation"),
    ("save_gifs", "true", F, "save render gifs"),
    ("use_render", "true", F, "render"),
    ("render_episodes", int, 5, "render episodes"),
    ("ifi", float, 0.1, "render frame interval"),
    ("model_dir", str, None, "pretrained transformer_{ep}.pt to restore"),
    # transformer
    ("encode_state", "true", F, "encode share_obs instead of obs"),
    ("n_block", int, 2, "transformer blocks"),
    ("n_embd", int, 64, "embedding width"),
    ("n_head", int, 2, "attention heads"),
    ("dec_actor", "true", F, "decentralised actor (MAT-Dec)"),
    ("share_actor", "true", F, "share the decentralised actor"),
]

# DCML_MAT_Train.parse_args extras (DCML_MAT_Train.py:61-78)
_DCML_FLAGS = [
    ("scenario", str, "DCML_MAT", "scenario name"),
    ("n_agent", int, 101, "agents (informational: the env defines it)"),
    ("add_move_state", "true", F, ""), ("add_local_obs", "true", F, ""), ("add_distance_state", "true", F, ""),
    ("add_enemy_action_state", "true", F, ""), ("add_agent_id", "true", F, ""), ("add_visible_state", "true", F, ""),
    ("add_xy_state", "true", F, ""), ("use_state_agent", "true", F, ""), ("use_mustalive", "false", T, ""),
    ("add_center_xy", "true", F, ""),
]

# SMAC entry extras (mat_src/mat/scripts/train/train_smac.py:65-78)
_SMAC_FLAGS = [
    ("map_name", str, "27m_vs_30m", "SMAC map"), ("eval_map_name", str, None, "SMAC eval map"),
    ("run_dir", str, "", ""), ("add_move_state", "true", F, ""), ("add_local_obs", "true", F, ""),
    ("add_distance_state", "true", F, ""), ("add_enemy_action_state", "true", F, ""), ("add_agent_id", "true", F, ""),
    ("add_visible_state", "true", F, ""), ("add_xy_state", "true", F, ""), ("use_state_agent", "false", T, ""),
    ("use_mustalive", "false", T, ""), ("add_center_xy", "false", T, ""), ("random_agent_order", "true", F, ""),
    ("smac_backend", str, "synthetic", "synthetic (on-device SMAC-shaped env) | sc2 (StarCraft II via process pool)"),
    ("n_env_workers", int, None, "worker processes of the CPU env pool (sc2 backend)"),
]

# MPE (``mat_src/mat/scripts/train/train_mpe.py:53-60`` + the scenario args the scenarios read)
_MPE_FLAGS = [
    ("scenario_name", str, "simple_spread", "MPE scenario"), ("num_landmarks", int, 3, ""),
    ("num_agents", int, 3, "agents (spread / reference / speaker_listener / push / adversary / crypto)"),
    ("num_good_agents", int, 1, "good agents (tag / world_comm / attack)"),
    ("num_adversaries", int, 3, "adversaries (tag / world_comm / attack)"),
]

# MA-MuJoCo (``mat_src/mat/scripts/train/train_mujoco.py:64-86`` + the env_args it builds, ``:20-27``)
_MUJOCO_FLAGS = [
    ("scenario", str, "Hopper-v2", "MuJoCo robot (HalfCheetah-v2, Ant-v2, Hopper-v2, Walker2d-v2, Swimmer-v2, "
                                   "Reacher-v2, coupled_half_cheetah, manyagent_swimmer, manyagent_ant)"),
    ("agent_conf", str, "3x1", "joint partition, e.g. 6x1 / 2x3 / 2x4 / 4x2"),
    ("agent_obsk", int, 0, "observe joints within k hops of the agent's own"),
    ("k_categories", str, None, "per-hop observed categories, e.g. 'qpos,qvel|qpos'"),
    ("global_categories", str, None, "categories of the global joints"),
    ("episode_limit", int, 1000, "env time limit"),
    ("faulty_node", int, -1, "agent whose actions are zeroed during training (-1: none)"),
    ("random_agent_order", "true", F, "RandomMujocoMulti: permute the agents every episode"),
    ("add_move_state", "true", F, ""), ("add_local_obs", "true", F, ""), ("add_distance_state", "true", F, ""),
    ("add_enemy_action_state", "true", F, ""), ("add_agent_id", "true", F, ""), ("add_visible_state", "true", F, ""),
    ("add_xy_state", "true", F, ""), ("use_state_agent", "true", F, ""), ("use_mustalive", "false", T, ""),
    ("add_center_xy", "true", F, ""),
]

# Google Research Football (``mat_src/mat/scripts/train/train_football.py:64-86``)
_FOOTBALL_FLAGS = [
    ("scenario", str, "academy_3_vs_1_with_keeper", "GRF academy scenario"),
    ("n_agent", int, 3, "controlled left-team players"),
    ("add_move_state", "true", F, ""), ("add_local_obs", "true", F, ""), ("add_distance_state", "true", F, ""),
    ("add_enemy_action_state", "true", F, ""), ("add_agent_id", "true", F, ""), ("add_visible_state", "true", F, ""),
    ("add_xy_state", "true", F, ""), ("use_state_agent", "true", F, ""), ("use_mustalive", "false", T, ""),
    ("add_center_xy", "true", F, ""),
]

# framework (new)
_FRAMEWORK_FLAGS = [
    ("n_workers", int, 100, "DCML worker count W (agents = W + 1); 4 / 32 / 100 / 128 in the BASELINE configs"),
    ("shannon", "true", F, "Shannon-capacity links in the DCML env (shannon_enable, Shannon.py)"),
    ("reward_alpha", float, 99.0, "DCML reward = -(alpha * completion time + beta * payment); 99 / 1 = the reference "
     "(DCML_ENV_Functions.py:15-17)"),
    ("reward_beta", float, 1.0, "payment weight of the DCML reward (see reward_alpha)"),
    ("central_execution", int, 1, "1: one Semi_Discrete space for all agents; 0: per-agent spaces (Env(central_execution=False))"),
    ("kernels", str, "auto", "auto|hip|torch — fused HIP kernels on GPU (auto) or the PyTorch reference path"),
    ("dtype", str, "bf16", "bf16|fp32 compute dtype (master weights and optimizer state are fp32)"),
    ("train_stride", int, 1, "decision stride for rollouts (1 = exact per-agent sampling, the reference)"),
    ("rollout_groups", int, 1, "env groups of the rollout, each on its own HIP stream: one group's env step / insert / "
     "encoder overlap the other groups' decode (SURVEY §2.4); the rollout is identical for any group count"),
    ("eval_stride", int, 2, "batch decision stride for evaluation (dcml_runner.py:320)"),
    ("grad_overlap", "true", F, "data parallelism: all-reduce the decoder's gradient slice asynchronously while the "
     "encoder backward runs (two collectives per minibatch instead of one blocking all-reduce)"),
    ("recompute_gae_every_epoch", "false", T, "recompute next-value/GAE every PPO epoch (reference semantics)"),
    ("results_dir", str, None, "root of results/ (default: ./results)"),
    ("resume", "true", F, "resume from the latest trainer_state_*.pt in the run dir"),
    ("save_trainer_state", "false", T, "write trainer_state_{ep}.pt next to transformer_{ep}.pt"),
    ("max_restarts", int, 0, "elastic relaunches after a rank failure (launcher)"),
    ("fault_inject", str, None, "test hook: 'nan@<it>' or 'kill@<rank>:<it>'"),
    ("heartbeat_s", float, 0.0, "rank heartbeat period in seconds (0 = off)"),
    ("profile_phases", "true", F, "print per-phase timers"),
]


def _add(parser, flags):
    for name, kind, default, hlp in flags:
        if kind == "true":
            parser.add_argument(f"--{name}", action="store_true", default=default, help=hlp)
        elif kind == "false":
            parser.add_argument(f"--{name}", action="store_false", default=default, help=hlp)
        else:
            parser.add_argument(f"--{name}", type=kind, default=default, help=hlp)


def get_config() -> argparse.ArgumentParser:
    parser = argparse.ArgumentParser(description="mat_dcml_amd", formatter_class=argparse.RawDescriptionHelpFormatter)
    _add(parser, _FLAGS)
    parser.add_argument("--train_maps", type=str, nargs="+", default=None)
    parser.add_argument("--eval_maps", type=str, nargs="+", default=None)
    _add(parser, _FRAMEWORK_FLAGS)
    return parser


def parse_args(argv, parser=None, extra=_DCML_FLAGS, warn=True):
    parser = parser or get_config()
    existing = {a.dest for a in parser._actions}
    _add(parser, [f for f in extra if f[0] not in existing])
    args, unknown = parser.parse_known_args(argv)
    if unknown and warn:
        print(f"[config] ignoring unrecognised arguments: {unknown}", file=sys.stderr)
    args.num_env_steps = int(args.num_env_steps)
    return args
