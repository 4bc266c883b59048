"""Flag compatibility with the reference argvs (DCML_MAT_Train.py:193, DCML_MAT_ALT_Benchmark.py:80)."""
from mat_dcml_amd.config import get_config, parse_args

REF_TRAIN_ARGV = ["--n_rollout_threads", "8", "--num_env_steps", "1000000", "--save_interval", "50",
                  "--episode_length", "50", "--algorithm_name", "mat", "--env_name", "DCML", "--scenario", "AS",
                  "--lr", "5e-5", "--critic_lr", "5e-5", "--ppo_epoch", "15", "--num_mini_batch", "4", "--gamma",
                  "0.99", "--use_valuenorm", "--use_popart", "value_loss_coef", "1.5", "--entropy_coef", "0.01"]
REF_BENCH_ARGV = ["--use_eval", "--n_eval_rollout_threads", "2", "--algorithm_name", "mat", "--model_dir",
                  "./results/DCML/AS/mat/check/run1/models/transformer_1900.pt"]


def test_reference_train_argv():
    a = parse_args(REF_TRAIN_ARGV, get_config(), warn=False)
    assert a.n_rollout_threads == 8 and a.num_env_steps == 1000000 and a.episode_length == 50
    assert a.lr == 5e-5 and a.ppo_epoch == 15 and a.num_mini_batch == 4
    assert a.use_valuenorm and a.use_popart
    assert a.value_loss_coef == 1.0  # the malformed pair is dropped, exactly like the reference
    assert a.scenario == "AS" and a.env_name == "DCML"


def test_reference_benchmark_argv():
    a = parse_args(REF_BENCH_ARGV, get_config(), warn=False)
    assert a.use_eval and a.n_eval_rollout_threads == 2 and a.model_dir.endswith("transformer_1900.pt")


def test_inverted_booleans():
    a = parse_args([], get_config(), warn=False)
    assert a.cuda and a.use_huber_loss and a.use_clipped_value_loss and a.use_max_grad_norm
    a = parse_args(["--cuda", "--use_huber_loss", "--use_policy_active_masks"], get_config(), warn=False)
    assert not a.cuda and not a.use_huber_loss and not a.use_policy_active_masks


def test_defaults_match_reference():
    a = parse_args([], get_config(), warn=False)
    expect = dict(algorithm_name="mat", seed=1, n_rollout_threads=10, episode_length=200, lr=1e-3, opti_eps=1e-5,
                  ppo_epoch=15, clip_param=0.2, num_mini_batch=4, entropy_coef=0.01, value_loss_coef=1.0,
                  max_grad_norm=10.0, gamma=0.99, gae_lambda=0.95, huber_delta=10.0, n_block=2, n_embd=64,
                  n_head=2, save_interval=100, log_interval=5, eval_interval=25, eval_episodes=32, n_agent=101)
    for k, v in expect.items():
        assert getattr(a, k) == v, k
