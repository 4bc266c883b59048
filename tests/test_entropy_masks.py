"""Entropy reduction of TransformerPolicy.evaluate_actions under policy active masks for a multi-dimensional
continuous action (A = 3): the reference computes (entropy(N, A) * active_masks(N, 1)).sum() / active_masks.sum()
(transformer_policy.py:212-213) — summed over the action dimensions, per active token — and entropy.mean() without
the masks.  The reference's own Continuous branch cannot run evaluate_actions (act_prob_dim is never set for Box
spaces, transformer_policy.py:55-58), so the formula is the oracle."""
import torch

from mat_dcml_amd.algos.policy import TransformerPolicy
from mat_dcml_amd.config import get_config, parse_args
from mat_dcml_amd.envs.mujoco.multi import Box


def _policy(pam):
    argv = ["--algorithm_name", "mat", "--n_block", "1"] + (["--use_policy_active_masks"] if pam else [])
    args = parse_args(argv, get_config(), warn=False)
    args.use_policy_active_masks = pam
    torch.manual_seed(0)
    return TransformerPolicy(args, [5], [5], Box(-1.0, 1.0, 3), 4)


def test_entropy_sums_action_dims_under_policy_active_masks():
    B, L, A = 6, 4, 3
    g = torch.Generator().manual_seed(0)
    obs = torch.rand(B, L, 5, generator=g)
    act = torch.rand(B, L, A, generator=g) * 2 - 1
    am = (torch.rand(B * L, 1, generator=g) > 0.3).float()
    for pam in (True, False):
        pol = _policy(pam)
        with torch.no_grad():
            _, _, ent = pol.evaluate_actions(None, obs, act, None, am)
            m = pol.transformer
            v, rep = m.encoder(None, obs)
            from mat_dcml_amd.models import act as act_mod
            _, ent_tok = act_mod.parallel_act(m, rep, obs, act, None)
        e = ent_tok.reshape(B * L, A)
        want = (e * am).sum() / am.sum() if pam else e.mean()
        assert torch.allclose(ent, want, rtol=1e-5), (pam, float(ent), float(want))
    # the two reductions differ by the dimension count on an all-active batch
    assert A > 1
