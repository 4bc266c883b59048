"""MAT variants (mat_encoder / mat_decoder / mat_gru / mat_dec): API, exact incremental decode, DCML training."""
import pytest
import torch

from mat_dcml_amd.models import act as act_mod
from mat_dcml_amd.models.variants import MultiAgentDecoder, MultiAgentEncoder, MultiAgentGRU

B, L, OBS = 5, 9, 7


def _mk(cls):
    torch.manual_seed(0)
    m = cls(10, OBS, 2, L, n_block=2, n_embd=32, n_head=2, action_type="Semi_Discrete", semi_index=-1)
    for p in m.parameters():   # break the 0.01-gain init so every row matters
        p.data.add_(0.05 * torch.randn_like(p))
    return m


@pytest.mark.parametrize("cls", [MultiAgentEncoder, MultiAgentDecoder, MultiAgentGRU])
def test_variant_logprob_consistency(cls):
    """Sampled actions' log-probs from the incremental decode == teacher-forced evaluation of the same actions."""
    m = _mk(cls)
    obs = torch.rand(B, L, OBS)
    ava = torch.ones(B, L, 2)
    ava[:, 2, 1] = 0
    with torch.no_grad():
        a, lp, v = m.get_actions(None, obs, ava, deterministic=False)
        lp2, v2, ent = m(None, obs, a, ava)
    assert a.shape == (B, L, 1) and v.shape == (B, L, 1) and ent.shape == (B, L, 1)
    assert torch.allclose(lp, lp2, atol=1e-4), (lp - lp2).abs().max()
    assert torch.allclose(v, v2, atol=1e-5)
    assert torch.all(a[:, 2, 0] == 0)   # masked action never chosen


@pytest.mark.parametrize("cls", [MultiAgentDecoder, MultiAgentGRU])
def test_variant_stride_blocks_match_full_recompute(cls):
    """Deterministic stride decode == the reference's block loop of FULL decoder passes (transformer_act.py:37-75)."""
    m = _mk(cls)
    obs = torch.rand(B, L, OBS)
    with torch.no_grad():
        a, lp, _ = m.get_actions(None, obs, None, deterministic=True, stride=3)
        rep = m.encoder(None, obs)[1] if cls is MultiAgentGRU else m.decoder.obs_encoder(obs)
        n_disc = L - 1
        sh = torch.zeros(B, L, 3)
        sh[:, 0, 0] = 1
        ref = torch.zeros(B, L)
        for (s, e) in act_mod.block_schedule(L, n_disc, 3):
            logits = m.decoder(sh, rep, obs)
            for i in range(s, e):
                if i < n_disc:
                    ai = logits[:, i].argmax(-1)
                    ref[:, i] = ai.float()
                    if i + 1 < L:
                        sh[:, i + 1, 1:] = torch.nn.functional.one_hot(ai, 2).float()
                else:
                    ref[:, i] = logits[:, i, -1]
    assert torch.allclose(a[..., 0], ref, atol=1e-5)


@pytest.mark.parametrize("algo", ["mat_encoder", "mat_decoder", "mat_gru", "mat_dec"])
def test_variant_trains_on_dcml(algo, tmp_path):
    import DCML_MAT_Train
    argv = DCML_MAT_Train.DEFAULT_ARGV + ["--algorithm_name", algo, "--n_workers", "4", "--n_rollout_threads", "2",
                                          "--episode_length", "4", "--num_env_steps", "16", "--ppo_epoch", "2",
                                          "--num_mini_batch", "2", "--n_embd", "32", "--results_dir", str(tmp_path),
                                          "--cuda", "--log_interval", "1"]
    runner = DCML_MAT_Train.main(argv)
    files = list((tmp_path / "DCML").rglob("transformer_*.pt"))
    assert files, "no checkpoint written"
    sd = torch.load(files[0], weights_only=True)
    assert set(sd) == set(runner.policy.transformer.state_dict())
