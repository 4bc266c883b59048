"""Random-policy baseline (reference ``mat_src/mat/algorithms/random/algorithm/random_policy.py:61-109`` and
``random/random_trainer.py``), device-side.

Every discrete agent picks uniformly among its available actions; the ratio agent of a Semi_Discrete space
draws U(0,1).  (The reference's ratio branch ``i > semi_index + num_agents`` can never be true, so its ratio
agent picks 0 or 1 uniformly instead; ``ratio_quirk=True`` reproduces that.)  Values and log-probs are zero,
training is a no-op that reports zero losses.
"""
from __future__ import annotations

import torch


class RandomPolicy:
    def __init__(self, args, obs_space, cent_obs_space, act_space, num_agents, device=torch.device("cpu"),
                 ratio_quirk: bool = False):
        self.device = torch.device(device)
        self.num_agents = num_agents
        self.act_space = act_space
        self.semi_index = getattr(act_space, "semi_index", 0)
        self.act_dim = getattr(act_space, "n", 2)
        self.ratio_quirk = ratio_quirk
        self.n_objective = getattr(args, "n_objective", 1)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(int(getattr(args, "seed", 1)))

    def lr_decay(self, episode, episodes):
        pass

    @torch.no_grad()
    def get_actions(self, cent_obs, obs, available_actions=None, deterministic=False, stride=1, rand=None):
        B, A = obs.shape[0], obs.shape[1]
        if available_actions is None:
            available_actions = torch.ones(B, A, self.act_dim, device=obs.device)
        w = available_actions.float()
        u = torch.rand(B, A, 1, device=obs.device, generator=self.gen)
        # inverse-CDF pick among the available actions
        cdf = torch.cumsum(w, -1) / w.sum(-1, keepdim=True).clamp(min=1)
        act = (u >= cdf).sum(-1, keepdim=True).clamp(max=self.act_dim - 1).float()
        if self.semi_index != 0 and not self.ratio_quirk:
            act[:, self.semi_index:] = torch.rand(B, -self.semi_index, 1, device=obs.device, generator=self.gen)
        z = torch.zeros(B, A, 1, device=obs.device)
        return torch.zeros(B, A, self.n_objective, device=obs.device), act, z

    def get_values(self, cent_obs, obs, available_actions=None):
        return torch.zeros(obs.shape[0], obs.shape[1], self.n_objective, device=obs.device)

    def act(self, cent_obs, obs, available_actions=None, deterministic=True, stride=1):
        return self.get_actions(cent_obs, obs, available_actions)[1]

    def save(self, save_dir, episode):
        return None

    def restore(self, model_dir):
        pass

    def train(self):
        pass

    def eval(self):
        pass


class RandomTrainer:
    """``random_trainer.py``: nothing to learn; returns the standard info dict with zeros."""

    def __init__(self, args, policy, num_agents, device=torch.device("cpu"), comm=None):
        self.policy = policy

    def prep_training(self):
        pass

    def prep_rollout(self):
        pass

    def train(self, buffer):
        keys = ("value_loss", "policy_loss", "dist_entropy", "actor_grad_norm", "critic_grad_norm", "ratio")
        return {k: 0.0 for k in keys}
