"""Multi-objective MAT (momat / dmomat): vector value head over (-completion time, -payment)."""
import pytest
import torch

import DCML_MAT_Train


@pytest.mark.parametrize("algo", ["momat", "dmomat"])
def test_multi_objective_training(algo, tmp_path):
    argv = DCML_MAT_Train.DEFAULT_ARGV + ["--algorithm_name", algo, "--n_workers", "4", "--n_rollout_threads", "3",
                                          "--episode_length", "5", "--num_env_steps", "30", "--ppo_epoch", "2",
                                          "--num_mini_batch", "3", "--n_embd", "32", "--cuda", "--log_interval", "1",
                                          "--results_dir", str(tmp_path)]
    r = DCML_MAT_Train.main(argv)
    b = r.buffer
    assert b.rewards.shape[-1] == 2 and r.policy.transformer.encoder.head[-1].out_features == 2
    # objectives are the negated delay and payment of the same steps
    assert torch.all(b.rewards[..., 0] < 0) and torch.all(b.rewards[..., 1] <= 0)
    assert r.trainer.value_normalizer.running_mean.shape == (2,)
    assert torch.isfinite(b.returns).all() and torch.isfinite(b.advantages).all()
    logs = list((tmp_path / "DCML").rglob("scalars.jsonl")) + list((tmp_path / "DCML").rglob("*.csv"))
    text = "".join(p.read_text() for p in logs)
    assert "average_step_objective_1" in text
