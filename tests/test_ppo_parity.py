"""Golden parity of one PPO iteration (GAE per epoch, advantage normalisation, clipped policy loss, clipped Huber
value loss with ValueNorm, entropy bonus, grad clipping, Adam) against the reference MATTrainer itself
(mat_src/mat/algorithms/mat/mat_trainer.py:96-217) on the same weights and the same recorded buffer.

One minibatch per epoch, so the reference's random minibatch order cannot change the result."""
import numpy as np
import pytest
import torch

import ref_oracle as ro

W, E, T = 4, 3, 5
A = W + 1

pytestmark = pytest.mark.skipif(not ro.available(), reason="reference not mounted")


def _argv():
    return ["--n_rollout_threads", str(E), "--episode_length", str(T), "--ppo_epoch", "3", "--num_mini_batch", "1",
            "--algorithm_name", "mat", "--lr", "5e-3", "--use_valuenorm", "--entropy_coef", "0.01",
            "--use_value_active_masks", "--use_policy_active_masks", "--seed", "1"]


def test_ppo_iteration_matches_reference(tmp_path):
    ro.install_stubs()
    with ro.ref_cwd(tmp_path):
        from mat.config import get_config as ref_get_config
        from mat.algorithms.mat.algorithm.transformer_policy import TransformerPolicy as RefPolicy
        from mat.algorithms.mat.mat_trainer import MATTrainer as RefTrainer
        from mat.utils.shared_buffer import SharedReplayBuffer
        from DCML_ENVs.DCML_utils.DCML_ActionSpace import Action_Space as RefSpace
        ref_args = ref_get_config().parse_known_args(_argv())[0]
        ref_space = RefSpace(2, semi_index=-1, extra=True)
        torch.manual_seed(0)
        ref_pol = RefPolicy(ref_args, [7], [2 + W], ref_space, A, device=torch.device("cpu"))
        ref_tr = RefTrainer(ref_args, ref_pol, A, device=torch.device("cpu"))
        ref_buf = SharedReplayBuffer(ref_args, A, [7], [2 + W], ref_space, "DCML")

    from mat_dcml_amd.algos.buffer import RolloutBuffer
    from mat_dcml_amd.algos.mat_trainer import MATTrainer
    from mat_dcml_amd.algos.policy import TransformerPolicy
    from mat_dcml_amd.config import get_config, parse_args
    from mat_dcml_amd.envs.dcml.spaces import dcml_action_spaces
    from mat_dcml_amd.parallel.comm import Comm
    args = parse_args(_argv(), get_config(), warn=False)
    pol = TransformerPolicy(args, [7], [2 + W], dcml_action_spaces(W)[0], A)
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():   # a non-trivial common starting point
        for p in pol.transformer.parameters():
            p.add_(0.05 * torch.randn(p.shape, generator=g))
    ref_pol.transformer.load_state_dict(pol.transformer.state_dict())
    comm = Comm()
    comm.attach_flat_grads(pol.transformer.parameters())
    tr = MATTrainer(args, pol, A, comm=comm)
    buf = RolloutBuffer(T, E, A, 7, 2 + W, 2, use_valuenorm=True)

    # recorded rollout
    obs = torch.rand(T + 1, E, A, 7, generator=g)
    ava = torch.ones(T + 1, E, A, 2)
    ava[:, :, 1::2, 1] = (torch.rand(T + 1, E, (W + 1) // 2, generator=g) > 0.3).float()
    act = (torch.rand(T, E, A, 1, generator=g) < 0.5).float() * ava[:-1, :, :, 1:]
    act[:, :, -1, 0] = torch.rand(T, E, generator=g)
    with torch.no_grad():
        v, lp, _ = pol.evaluate_actions(None, obs[:-1].reshape(T * E, A, 7), act.reshape(T * E, A, 1),
                                        ava[:-1].reshape(T * E, A, 2))
    lp = lp.reshape(T, E, A, 1) + 0.05 * torch.randn(T, E, A, 1, generator=g)
    vp = torch.cat([v.reshape(T, E, A, 1), torch.zeros(1, E, A, 1)])
    rew = -torch.rand(T, E, 1, 1, generator=g).expand(T, E, A, 1) * 20
    masks = torch.ones(T + 1, E, A, 1)
    masks[2, 1] = 0
    masks[4, 0] = 0
    share = torch.rand(T + 1, E, 2 + W, generator=g)
    for name, val in (("obs", obs), ("available_actions", ava), ("actions", act), ("action_log_probs", lp),
                      ("value_preds", vp), ("rewards", rew), ("masks", masks)):
        getattr(buf, name).copy_(val)
    buf.share_obs.copy_(share)
    ref_buf.obs[:] = obs.numpy()
    ref_buf.share_obs[:] = share.unsqueeze(2).expand(T + 1, E, A, 2 + W).numpy()
    ref_buf.available_actions[:] = ava.numpy()
    ref_buf.actions[:] = act.numpy()
    ref_buf.action_log_probs[:] = lp.numpy()
    ref_buf.value_preds[:] = vp.numpy()
    ref_buf.rewards[:] = rew.numpy()
    ref_buf.masks[:] = masks.numpy()

    info_ref = ref_tr.train(ref_buf)
    info = tr.train(buf)
    for (k, a), (k2, b) in zip(ref_pol.transformer.state_dict().items(), pol.transformer.state_dict().items()):
        assert k == k2
        assert torch.allclose(a.float(), b.float(), rtol=2e-4, atol=2e-6), (k, (a - b).abs().max())
    assert np.allclose(ref_buf.returns[:-1], buf.returns[:-1].numpy(), rtol=1e-4, atol=1e-4)
    for k in ("value_loss", "policy_loss", "dist_entropy", "ratio"):
        r, m = float(torch.as_tensor(info_ref[k]).detach()), float(torch.as_tensor(info[k]).detach())
        assert abs(r - m) <= 1e-4 * max(1.0, abs(r)), (k, r, m)
