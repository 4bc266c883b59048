"""Baseline MARL algorithms on agent-batched actor-critics: HAPPO, R-MAPPO, IPPO, HATRPO and single-agent PPO.

Behavioural contract (reference ``mat_src/mat``):

* Policies (``happo_policy.py``, ``rMAPPOPolicy.py``, ``ippo_policy.py``, ``hatrpo_policy.py``,
  ``ppo_policy.py``): an actor and a critic per agent, actor lr ``--lr``, critic lr ``--critic_lr``, Adam
  (eps ``--opti_eps``), linear LR decay, actor input = obs or concat(share_obs, obs) with
  ``--use_cent_local_observe``.
* Separated buffers (``utils/separated_buffer.py``): per-agent GAE on (PopArt|ValueNorm)-denormalised values,
  advantage normalisation over active entries, feed-forward / naive-recurrent / chunked-recurrent
  (``--data_chunk_length``) minibatch generators, the HAPPO ``factor``.
* PPO update (``happo_trainer.py:88-166``, ``r_mappo.py``, ``ippo_trainer.py``, ``ppo_trainer.py``):
  importance weight = prod over action dims of exp(new − old), clipped surrogate times ``factor``, policy
  loss masked by active masks, entropy bonus, per-net grad clipping, clipped + Huber value loss with the value
  normaliser; infos averaged over ``ppo_epoch × num_mini_batch`` updates.
* Sequential update (``base_runner.py:327-417``): agents in ``torch.randperm`` order; after agent k is trained,
  ``factor ← sqrt(factor · prod exp(new_logp − old_logp))`` (the reference's square root is kept; pass
  ``happo_factor_sqrt=False`` for the paper's plain product).
* HATRPO (``hatrpo_trainer.py:181-348``): critic Adam step, then natural-gradient actor step — conjugate
  gradient (10 iterations) on the Fisher-vector product of the mean KL, step size sqrt(2·δ / sᵀFs), backtracking
  line search (``--ls_step``, ``--accept_ratio``) accepting when the KL stays under ``--kl_threshold`` and the
  surrogate improves.

MI355X design: rollout inference runs all agents in one batched pass; algorithms whose agents are independent
(IPPO; R-MAPPO, whose update ignores the factor) also *train* all agents in one batched pass with per-agent
grad clipping and per-agent Adam state (``algos/stacked_adam.py``), instead of the reference's per-agent Python
loop.  HAPPO / HATRPO keep the sequential per-agent order because it is the algorithm.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..models.ac import Actor, Critic, space_of
from .stacked_adam import StackedAdam


def _huber(e, d):
    a = e.abs()
    return torch.where(a <= d, 0.5 * e * e, d * (a - 0.5 * d))


class StackedValueNorm:
    """ValueNorm (``utils/valuenorm.py``) with one set of statistics per agent; stats shaped (M, 1)."""

    def __init__(self, M, device, beta=0.99999, eps=1e-5):
        self.beta, self.eps = beta, eps
        self.mean = torch.zeros(M, 1, device=device)
        self.mean_sq = torch.zeros(M, 1, device=device)
        self.debias = torch.zeros(M, 1, device=device)

    def _mv(self, idx=None):
        d = self.debias.clamp(min=self.eps)
        mean = self.mean / d
        var = (self.mean_sq / d - mean ** 2).clamp(min=1e-2)
        if idx is not None:
            return mean[idx], var[idx]
        return mean, var

    @torch.no_grad()
    def update(self, x, idx=None):
        """x: (N, M, 1) for all agents or (N, 1) for agent idx."""
        if idx is None:
            x = x.float().reshape(-1, *self.mean.shape)
            bm, bsq = x.mean(0), (x ** 2).mean(0)
            self.mean.mul_(self.beta).add_(bm * (1 - self.beta))
            self.mean_sq.mul_(self.beta).add_(bsq * (1 - self.beta))
            self.debias.mul_(self.beta).add_(1 - self.beta)
        else:
            bm, bsq = x.float().mean(), (x.float() ** 2).mean()
            self.mean[idx] = self.mean[idx] * self.beta + bm * (1 - self.beta)
            self.mean_sq[idx] = self.mean_sq[idx] * self.beta + bsq * (1 - self.beta)
            self.debias[idx] = self.debias[idx] * self.beta + (1 - self.beta)

    def normalize(self, x, idx=None):
        m, v = self._mv(idx)
        return (x - m) / v.sqrt()

    def denormalize(self, x, idx=None):
        m, v = self._mv(idx)
        return x * v.sqrt() + m


class AgentGroups:
    """Agents partitioned into runs of identical action spaces; each run is one stacked actor."""

    def __init__(self, act_spaces):
        kinds = [space_of(s) for s in act_spaces]
        self.groups = []            # (start, end, space)
        s = 0
        for i in range(1, len(kinds) + 1):
            if i == len(kinds) or kinds[i] != kinds[s]:
                self.groups.append((s, i, kinds[s]))
                s = i
        self.A = len(kinds)

    def locate(self, k):
        for g, (s, e, _) in enumerate(self.groups):
            if s <= k < e:
                return g, k - s
        raise IndexError(k)


class ACPolicy:
    """Per-agent actors/critics (agent-batched) + per-agent Adam; the policy surface of ``rMAPPOPolicy``."""

    def __init__(self, args, obs_dim, share_dim, act_spaces, num_agents, device=torch.device("cpu"), obs_shape=None):
        self.args, self.device = args, torch.device(device)
        self.lr, self.critic_lr = args.lr, args.critic_lr
        self.A = num_agents
        self.groups = AgentGroups(act_spaces)
        self.cent_local = bool(getattr(args, "use_cent_local_observe", False))
        in_dim = obs_dim + (share_dim if self.cent_local else 0)
        self.actors = torch.nn.ModuleList([Actor(e - s, in_dim, sp, args, obs_shape) for s, e, sp in self.groups.groups])
        self.critic = Critic(num_agents, share_dim, args, popart=args.use_popart)
        self.actors.to(self.device)
        self.critic.to(self.device)
        self.actor_opt = [StackedAdam(a.parameters(), e - s, self.lr, args.opti_eps, weight_decay=args.weight_decay)
                          for a, (s, e, _) in zip(self.actors, self.groups.groups)]
        self.critic_opt = StackedAdam(self.critic.parameters(), num_agents, self.critic_lr, args.opti_eps,
                                      weight_decay=args.weight_decay)
        self.act_dim = max(a.act.act_dim for a in self.actors)
        self.recurrent = args.use_recurrent_policy or args.use_naive_recurrent_policy
        self.N, self.H = args.recurrent_N, args.hidden_size

    # ---------------------------------------------------------------------------------- helpers
    def actor_in(self, share, obs):
        if self.cent_local:
            return torch.cat([share.expand(*obs.shape[:-1], share.shape[-1]), obs], -1)
        return obs

    def lr_decay(self, episode, episodes):
        f = 1 - episode / float(episodes)
        for o in self.actor_opt:
            o.set_lr(self.lr * f)
        self.critic_opt.set_lr(self.critic_lr * f)

    # ---------------------------------------------------------------------------------- rollout (all agents)
    @torch.no_grad()
    def get_actions(self, share, obs, rnn_a, rnn_c, masks, ava=None, deterministic=False):
        """(B, A, ·) tensors; rnn_* (B, A, N, H).  Returns values (B,A,1), actions (B,A,adim), logp (B,A,adim),
        rnn_a, rnn_c."""
        B = obs.shape[0]
        x = self.actor_in(share, obs)
        acts = torch.zeros(B, self.A, self.act_dim, device=obs.device)
        lps = torch.zeros(B, self.A, self.act_dim, device=obs.device)
        rnn_a = rnn_a.clone()
        for actor, (s, e, sp) in zip(self.actors, self.groups.groups):
            av = None if ava is None else ava[:, s:e, : _ava_dim(sp)]
            a, lp, h = actor(x[None, :, s:e], rnn_a[:, s:e], masks[None, :, s:e], av, deterministic)
            acts[:, s:e, : a.shape[-1]] = a[0]
            lps[:, s:e, : lp.shape[-1]] = lp[0]
            rnn_a[:, s:e] = h
        v, hc = self.critic(share.expand(B, self.A, share.shape[-1])[None], rnn_c, masks[None])
        return v[0], acts, lps, rnn_a, hc

    @torch.no_grad()
    def get_values(self, share, rnn_c, masks):
        B = share.shape[0]
        v, _ = self.critic(share.expand(B, self.A, share.shape[-1])[None], rnn_c, masks[None])
        return v[0]

    def act(self, share, obs, rnn_a, masks, ava=None, deterministic=True):
        B = obs.shape[0]
        rnn_c = torch.zeros(B, self.A, self.N, self.H, device=obs.device)
        return self.get_actions(share, obs, rnn_a, rnn_c, masks, ava, deterministic)[1]

    # ---------------------------------------------------------------------------------- save / restore
    def state_dict(self):
        return {"actors": self.actors.state_dict(), "critic": self.critic.state_dict()}

    def load_state_dict(self, sd):
        self.actors.load_state_dict(sd["actors"])
        self.critic.load_state_dict(sd["critic"])


def _ava_dim(space):
    kind, dims = space
    if kind == "discrete":
        return dims
    if kind == "mixed":
        return dims[0] * dims[1]
    return 1


class SeparatedBuffer:
    """(T+1, E, A, ·) rollout storage with per-agent returns and the HAPPO factor (``separated_buffer.py``)."""

    def __init__(self, args, E, A, obs_dim, share_dim, act_dim, ava_dim, device):
        T = args.episode_length
        self.T, self.E, self.A = T, E, A
        self.gamma, self.lam = args.gamma, args.gae_lambda
        self.N, self.H = args.recurrent_N, args.hidden_size
        dev, f = torch.device(device), torch.float32
        self.share_obs = torch.zeros(T + 1, E, share_dim, dtype=f, device=dev)
        self.obs = torch.zeros(T + 1, E, A, obs_dim, dtype=f, device=dev)
        self.rnn_states = torch.zeros(T + 1, E, A, self.N, self.H, dtype=f, device=dev)
        self.rnn_states_critic = torch.zeros_like(self.rnn_states)
        self.value_preds = torch.zeros(T + 1, E, A, 1, dtype=f, device=dev)
        self.returns = torch.zeros_like(self.value_preds)
        self.advantages = torch.zeros(T, E, A, 1, dtype=f, device=dev)
        self.actions = torch.zeros(T, E, A, act_dim, dtype=f, device=dev)
        self.action_log_probs = torch.zeros(T, E, A, act_dim, dtype=f, device=dev)
        self.rewards = torch.zeros(T, E, A, 1, dtype=f, device=dev)
        self.masks = torch.ones(T + 1, E, A, 1, dtype=f, device=dev)
        self.active_masks = torch.ones_like(self.masks)
        self.available_actions = torch.ones(T + 1, E, A, ava_dim, dtype=f, device=dev)
        self.factor = torch.ones(T, E, 1, dtype=f, device=dev)
        self.step = 0

    def insert(self, share, obs, rnn_a, rnn_c, actions, logp, values, rewards, masks, active_masks=None, ava=None):
        t = self.step
        self.share_obs[t + 1].copy_(share)
        self.obs[t + 1].copy_(obs)
        self.rnn_states[t + 1].copy_(rnn_a)
        self.rnn_states_critic[t + 1].copy_(rnn_c)
        self.actions[t].copy_(actions)
        self.action_log_probs[t].copy_(logp)
        self.value_preds[t].copy_(values)
        self.rewards[t].copy_(rewards.expand_as(self.rewards[t]))
        self.masks[t + 1].copy_(masks.expand_as(self.masks[t + 1]))
        if active_masks is not None:
            self.active_masks[t + 1].copy_(active_masks.expand_as(self.active_masks[t + 1]))
        if ava is not None:
            self.available_actions[t + 1, ..., : ava.shape[-1]].copy_(ava)
        self.step = (t + 1) % self.T

    def after_update(self):
        for n in ("share_obs", "obs", "rnn_states", "rnn_states_critic", "masks", "active_masks", "available_actions"):
            b = getattr(self, n)
            b[0].copy_(b[-1])

    @torch.no_grad()
    def compute_returns(self, next_value, denorm=None):
        """GAE per agent on denormalised values (``separated_buffer.py:compute_returns``)."""
        self.value_preds[-1].copy_(next_value)
        v = denorm(self.value_preds) if denorm is not None else self.value_preds
        g = torch.zeros_like(self.rewards[0])
        for t in reversed(range(self.T)):
            delta = self.rewards[t] + self.gamma * v[t + 1] * self.masks[t + 1] - v[t]
            g = delta + self.gamma * self.lam * self.masks[t + 1] * g
            self.returns[t] = g + v[t]

    def sequences(self, L):
        """Reshape (T, E, ...) time-major data into (L, T/L·E, ...) chunks (L = 1: feed-forward samples)."""
        T, E = self.T, self.E
        n = T // L

        def chunk(x):  # (T, E, ...) → (L, n*E, ...)
            return x[: n * L].reshape(n, L, E, *x.shape[2:]).transpose(0, 1).reshape(L, n * E, *x.shape[2:])

        def first(x):  # state at each chunk start: (n*E, ...)
            return x[: n * L: L].reshape(n * E, *x.shape[2:])
        return chunk, first, n * E


class BaselineTrainer:
    """One trainer for every baseline; ``mode`` picks the update schedule (see module docstring)."""

    def __init__(self, args, policy: ACPolicy, mode="rmappo", device=torch.device("cpu")):
        self.args, self.policy, self.mode = args, policy, mode
        self.device = torch.device(device)
        self.clip = args.clip_param
        self.ppo_epoch, self.num_mini_batch = args.ppo_epoch, args.num_mini_batch
        self.data_chunk_length = args.data_chunk_length
        self.value_loss_coef, self.entropy_coef = args.value_loss_coef, args.entropy_coef
        self.max_grad_norm, self.huber_delta = args.max_grad_norm, args.huber_delta
        self.use_max_grad_norm = args.use_max_grad_norm
        self.use_clipped_value_loss, self.use_huber_loss = args.use_clipped_value_loss, args.use_huber_loss
        self.use_popart, self.use_valuenorm = args.use_popart, args.use_valuenorm
        self.use_value_active_masks = args.use_value_active_masks
        self.use_policy_active_masks = args.use_policy_active_masks
        self.recurrent = args.use_recurrent_policy
        self.naive_recurrent = args.use_naive_recurrent_policy
        self.factor_sqrt = getattr(args, "happo_factor_sqrt", True)
        A = policy.A
        self.value_normalizer = None
        if self.use_popart:
            self.value_normalizer = policy.critic.v_out
        elif self.use_valuenorm:
            self.value_normalizer = StackedValueNorm(A, self.device)

    # ---------------------------------------------------------------------------------- helpers
    def denorm(self, x, idx=None):
        if self.value_normalizer is None:
            return x
        if idx is None:   # x (..., A, 1)
            return self.value_normalizer.denormalize(x)
        return self.value_normalizer.denormalize(x, idx)

    def prep_training(self):
        self.policy.actors.train()
        self.policy.critic.train()

    def prep_rollout(self):
        self.policy.actors.eval()
        self.policy.critic.eval()

    def value_loss(self, values, old_values, returns, active, idx=None):
        """``cal_value_loss`` (``happo_trainer.py:51-86``) for all agents (idx None) or one agent."""
        clipped = old_values + (values - old_values).clamp(-self.clip, self.clip)
        if self.value_normalizer is not None:
            self.value_normalizer.update(returns, idx)
            target = self.value_normalizer.normalize(returns, idx)
        else:
            target = returns
        ec, eo = target - clipped, target - values
        if self.use_huber_loss:
            lc, lo = _huber(ec, self.huber_delta), _huber(eo, self.huber_delta)
        else:
            lc, lo = 0.5 * ec ** 2, 0.5 * eo ** 2
        loss = torch.max(lo, lc) if self.use_clipped_value_loss else lo
        return _masked_mean(loss, active if self.use_value_active_masks else None, idx is None)

    def _advantages(self, buf):
        """Per-agent normalisation over active entries (each reference agent normalises its own buffer)."""
        adv = buf.returns[:-1] - self.denorm(buf.value_preds[:-1])
        m = (buf.active_masks[:-1] != 0).float()
        n = m.sum((0, 1), keepdim=True).clamp(min=1)
        mean = (adv * m).sum((0, 1), keepdim=True) / n
        var = (((adv - mean) ** 2) * m).sum((0, 1), keepdim=True) / n
        return (adv - mean) / (var.sqrt() + 1e-5)

    def _next_values(self, buf):
        return self.policy.get_values(buf.share_obs[-1][:, None].expand(buf.E, buf.A, -1), buf.rnn_states_critic[-1],
                                      buf.masks[-1])

    # ---------------------------------------------------------------------------------- train
    def train(self, buf, order=None):
        """Full PPO/TRPO iteration over the buffer; returns averaged infos."""
        buf.compute_returns(self._next_values(buf), self.denorm)
        adv = self._advantages(buf)
        self.prep_training()
        infos = {k: 0.0 for k in ("value_loss", "policy_loss", "dist_entropy", "actor_grad_norm",
                                  "critic_grad_norm", "ratio")}
        if self.mode in ("ippo", "rmappo", "ppo"):
            buf.factor.fill_(1.0)
            self._epochs(buf, adv, None, infos)
            n = self.ppo_epoch * self.num_mini_batch
        else:   # sequential: happo / hatrpo
            buf.factor.fill_(1.0)
            order = order if order is not None else torch.randperm(buf.A).tolist()
            for k in order:
                old = self._agent_logp(buf, k)
                self._epochs(buf, adv, k, infos)
                new = self._agent_logp(buf, k)
                r = torch.prod(torch.exp(new - old), -1, keepdim=True).reshape(buf.T, buf.E, 1)
                f = buf.factor * r
                buf.factor.copy_(f.clamp(min=0).sqrt() if self.factor_sqrt else f)
            n = self.ppo_epoch * self.num_mini_batch * len(order)
            if self.mode == "hatrpo":
                n = self.num_mini_batch * len(order)
        return {k: float(v) / max(n, 1) for k, v in infos.items()}

    @torch.no_grad()
    def _agent_logp(self, buf, k):
        p = self.policy
        g, j = p.groups.locate(k)
        actor = p.actors[g]
        s, e, sp = p.groups.groups[g]
        L = buf.T if (self.recurrent or self.naive_recurrent) else 1
        chunk, first, n = buf.sequences(L)
        obs = p.actor_in(chunk(buf.share_obs[:-1])[..., None, :].expand(L, n, buf.A, -1), chunk(buf.obs[:-1]))[:, :, k]
        ava = chunk(buf.available_actions[:-1])[:, :, k, : _ava_dim(sp)] if sp[0] in ("discrete", "mixed") else None
        lp, _, _ = actor.evaluate_actions(obs, first(buf.rnn_states[:-1])[:, k], chunk(buf.actions)[:, :, k, : actor.act.act_dim],
                                          chunk(buf.masks[:-1])[:, :, k], ava, idx=j)
        return lp.reshape(L, -1, lp.shape[-1]).reshape(-1, lp.shape[-1]) if L == 1 else \
            lp.reshape(L, buf.T // L, buf.E, -1).transpose(0, 1).reshape(-1, lp.shape[-1])

    def _epochs(self, buf, adv, k, infos):
        L = self.data_chunk_length if self.recurrent else (buf.T if self.naive_recurrent else 1)
        chunk, first, n = buf.sequences(L)
        data = dict(share=chunk(buf.share_obs[:-1]), obs=chunk(buf.obs[:-1]), actions=chunk(buf.actions),
                    old_lp=chunk(buf.action_log_probs), values=chunk(buf.value_preds[:-1]),
                    returns=chunk(buf.returns[:-1]), masks=chunk(buf.masks[:-1]), active=chunk(buf.active_masks[:-1]),
                    ava=chunk(buf.available_actions[:-1]), adv=chunk(adv),
                    factor=chunk(buf.factor), h_a=first(buf.rnn_states[:-1]), h_c=first(buf.rnn_states_critic[:-1]))
        epochs = 1 if self.mode == "hatrpo" else self.ppo_epoch
        for _ in range(epochs):
            perm = torch.randperm(n, device=buf.obs.device)
            mb = max(1, n // self.num_mini_batch)
            for i in range(self.num_mini_batch):
                ids = perm[i * mb:(i + 1) * mb]
                sample = {key: (v[ids] if key in ("h_a", "h_c") else v[:, ids]) for key, v in data.items()}
                if self.mode == "hatrpo":
                    out = self._trpo_update(sample, k)
                else:
                    out = self._ppo_update(sample, k)
                for key, v in out.items():
                    infos[key] += float(v)

    # ---------------------------------------------------------------------------------- one minibatch
    def _eval(self, s, k):
        """Evaluate actors (one agent k, or every agent) and critics on a minibatch of sequences."""
        p = self.policy
        Lc, B = s["obs"].shape[:2]
        share_a = s["share"][..., None, :].expand(Lc, B, p.A, s["share"].shape[-1])
        x = p.actor_in(share_a, s["obs"])
        if k is None:
            lps, ents = [], []
            for actor, (st, en, sp) in zip(p.actors, p.groups.groups):
                ava = s["ava"][:, :, st:en, : _ava_dim(sp)] if sp[0] in ("discrete", "mixed") else None
                lp, ent, _ = actor.evaluate_actions(x[:, :, st:en], s["h_a"][:, st:en],
                                                    s["actions"][:, :, st:en, : actor.act.act_dim],
                                                    s["masks"][:, :, st:en], ava)
                lps.append(F.pad(lp, (0, p.act_dim - lp.shape[-1])))
                ents.append(ent)
            lp, ent, dist = torch.cat(lps, 2), torch.cat(ents, 2), None
            v, _ = p.critic(share_a, s["h_c"], s["masks"])
            return lp, ent, v, dist
        g, j = p.groups.locate(k)
        actor = p.actors[g]
        sp = p.groups.groups[g][2]
        ava = s["ava"][:, :, k, : _ava_dim(sp)] if sp[0] in ("discrete", "mixed") else None
        lp, ent, dist = actor.evaluate_actions(x[:, :, k], s["h_a"][:, k], s["actions"][:, :, k, : actor.act.act_dim],
                                               s["masks"][:, :, k], ava, idx=j)
        v, _ = p.critic(share_a[:, :, k], s["h_c"][:, k], s["masks"][:, :, k], idx=k)
        return lp, ent, v, dist

    def _sel(self, s, key, k):
        x = s[key]
        if key == "factor":
            return x[:, :, None, :] if k is None else x
        return x if k is None else x[:, :, k]

    def _critic_step(self, v, s, k):
        vl = self.value_loss(v, self._sel(s, "values", k), self._sel(s, "returns", k), self._sel(s, "active", k), k)
        p = self.policy
        p.critic_opt.zero_grad()
        (vl * self.value_loss_coef).backward()
        cn = p.critic_opt.clip_(self.max_grad_norm, k) if self.use_max_grad_norm else p.critic_opt.grad_norms(k)
        p.critic_opt.step(k)
        return vl, cn

    def _ppo_update(self, s, k):
        p = self.policy
        lp, ent, v, _ = self._eval(s, k)
        old = self._sel(s, "old_lp", k)
        if k is not None:
            old = old[..., : lp.shape[-1]]
        imp = torch.prod(torch.exp(lp - old), -1, keepdim=True)
        adv = self._sel(s, "adv", k)
        surr = torch.min(imp * adv, imp.clamp(1 - self.clip, 1 + self.clip) * adv) * self._sel(s, "factor", k)
        active = self._sel(s, "active", k)
        pol = -_masked_mean(surr, active if self.use_policy_active_masks else None, k is None)
        ent_m = _masked_mean(ent, active if self.use_policy_active_masks else None, k is None)
        opts = p.actor_opt if k is None else [p.actor_opt[p.groups.locate(k)[0]]]
        for o in opts:
            o.zero_grad()
        (pol - ent_m * self.entropy_coef).backward()
        gn = 0.0
        for o in opts:
            idx = None if k is None else p.groups.locate(k)[1]
            n = o.clip_(self.max_grad_norm, idx) if self.use_max_grad_norm else o.grad_norms(idx)
            o.step(idx)
            gn += float(n.mean())
        vl, cn = self._critic_step(v, s, k)
        return {"value_loss": vl.detach(), "policy_loss": pol.detach(), "dist_entropy": ent_m.detach(),
                "actor_grad_norm": gn / len(opts), "critic_grad_norm": cn.mean().detach(), "ratio": imp.mean().detach()}

    # ---------------------------------------------------------------------------------- HATRPO
    def _trpo_update(self, s, k):
        p = self.policy
        g, j = p.groups.locate(k)
        actor = p.actors[g]
        lp, ent, v, dist = self._eval(s, k)
        vl, cn = self._critic_step(v, s, k)
        old = self._sel(s, "old_lp", k)[..., : lp.shape[-1]]
        adv, fac, active = self._sel(s, "adv", k), self._sel(s, "factor", k), self._sel(s, "active", k)
        am = active if self.use_policy_active_masks else None

        def surrogate(lp_):
            r = torch.prod(torch.exp(lp_ - old), -1, keepdim=True)
            return _masked_mean(r * fac * adv, am, False), r

        loss, ratio = surrogate(lp)
        params = [q for q in actor.parameters()]
        grads = torch.autograd.grad(loss, params, allow_unused=True)
        gvec = _flat_slice(grads, params, j)
        old_dist = _detach_dist(dist)

        def fvp(vec):
            lp2, _, _, d2 = self._eval(s, k)
            kl = _masked_mean(d2.kl(old_dist), am, False)
            gkl = torch.autograd.grad(kl, params, create_graph=True, allow_unused=True)
            gk = _flat_slice(gkl, params, j)
            hv = torch.autograd.grad((gk * vec).sum(), params, allow_unused=True)
            return _flat_slice(hv, params, j).detach() + 0.1 * vec

        step_dir = _conjugate_gradient(fvp, gvec.detach(), 10)
        shs = 0.5 * (step_dir * fvp(step_dir)).sum()
        step_size = 1.0 / torch.sqrt(shs.clamp(min=1e-12) / self.args.kl_threshold)
        full = step_size * step_dir
        base = _get_slice(params, j)
        expected = (gvec * full).sum()
        accepted = False
        frac = 1.0
        with torch.no_grad():
            for _ in range(self.args.ls_step):
                _set_slice(params, j, base + frac * full)
                lp_n, _, _, d_n = self._eval(s, k)
                new_loss, _ = surrogate(lp_n)
                kl = _masked_mean(d_n.kl(old_dist), am, False)
                improve = new_loss - loss
                if kl < self.args.kl_threshold and improve / (expected * frac + 1e-12) > self.args.accept_ratio \
                        and improve > 0:
                    accepted = True
                    break
                frac *= 0.5
            if not accepted:
                _set_slice(params, j, base)
        ent_m = _masked_mean(ent, am, False)
        return {"value_loss": vl.detach(), "policy_loss": loss.detach(), "dist_entropy": ent_m.detach(),
                "actor_grad_norm": float(gvec.norm()), "critic_grad_norm": cn.mean().detach(),
                "ratio": ratio.mean().detach()}


def _masked_mean(x, mask, per_agent_sum):
    """Masked mean; for an all-agent batch (…, A, d) the loss is the SUM over agents of per-agent means so each
    agent's gradient equals the one its own trainer would compute."""
    if per_agent_sum:
        red = tuple(range(x.dim() - 2)) + (x.dim() - 1,)
        if mask is None:
            return x.mean(dim=red).sum()
        m = mask.expand_as(x)
        return ((x * m).sum(dim=red) / m.sum(dim=red).clamp(min=1)).sum()
    if mask is None:
        return x.mean()
    m = mask.expand_as(x)
    return (x * m).sum() / m.sum().clamp(min=1)


def _flat_slice(grads, params, j):
    return torch.cat([(g[j] if g is not None else torch.zeros_like(p[j])).reshape(-1) for g, p in zip(grads, params)])


def _get_slice(params, j):
    return torch.cat([p.data[j].reshape(-1) for p in params]).clone()


def _set_slice(params, j, vec):
    o = 0
    for p in params:
        n = p[j].numel()
        p.data[j].copy_(vec[o:o + n].view_as(p[j]))
        o += n


def _conjugate_gradient(Avp, b, nsteps, tol=1e-10):
    x = torch.zeros_like(b)
    r, p = b.clone(), b.clone()
    rr = r @ r
    for _ in range(nsteps):
        Ap = Avp(p)
        alpha = rr / (p @ Ap + 1e-12)
        x += alpha * p
        r -= alpha * Ap
        new_rr = r @ r
        if new_rr < tol:
            break
        p = r + (new_rr / rr) * p
        rr = new_rr
    return x


def _detach_dist(d):
    from ..models import ac
    if isinstance(d, ac.CatDist):
        return ac.CatDist(d.d.logits.detach())
    if isinstance(d, ac.MultiCatDist):
        return ac.MultiCatDist(d.d.logits.detach())
    if isinstance(d, ac.NormalDist):
        return ac.NormalDist(d.d.mean.detach(), d.d.stddev.detach())
    if isinstance(d, ac.BernDist):
        return ac.BernDist(d.d.logits.detach())
    if isinstance(d, ac.ProductDist):
        return ac.ProductDist([_detach_dist(q) for q in d.parts], d.sizes, d.ent_scale, d.ent_mean_cat)
    raise TypeError(type(d))
