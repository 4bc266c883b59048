"""Vectorised multi-agent MuJoCo env on device (``MujocoMulti`` / ``RandomMujocoMulti`` semantics, E envs at once).

Reference: ``mat_src/mat/envs/ma_mujoco/multiagent_mujoco/mujoco_multi.py:39-265`` and
``random_mujoco_multi.py:39-303``, run through the vec-env worker (auto-reset when done, ``env_wrappers.py``).

* agents = the joint partition of ``graph.parts_and_edges(scenario, agent_conf)``; agent i's action vector is
  padded to ``n_actions = max partition size`` and the env keeps its first ``len(part_i)`` entries, concatenated
  in agent order into the robot's actuator vector (``:123-126``) — NOT reordered by the joints' actuator ids
  (so Ant 2x4's agent 0 drives actuators hip4, ankle4, hip1, ankle1 while observing hip1..ankle2, as upstream);
* observation of agent i: ``agent_obsk=None`` → the robot's full ``_get_obs()``; else ``graph.build_obs`` over the
  joints within ``agent_obsk`` hops, zero-padded to the largest agent; then the one-hot agent id, then
  standardised per vector ``(x - mean) / std`` (``:166-177``);
* share obs of agent i: ``_get_obs()`` + one-hot id, standardised (``:203-214``);
* reward: the robot's scalar reward replicated to every agent; dones: all agents share the robot's done or the
  ``episode_limit`` time-out, with ``info["bad_transition"]`` = timed out (``:137-141``);
* ``random_agent_order``: a fresh agent permutation at every reset; obs / share / rewards / dones come out
  permuted and the policy's actions are mapped back (``random_mujoco_multi.py:128-175, 265-281``);
* available actions: all ones (continuous actions).
"""
from __future__ import annotations

import torch

from . import graph
from .physics import PlanarSim, make_model


class Box:
    def __init__(self, low, high, shape):
        self.low, self.high, self.shape = low, high, (int(shape),)


class _Data:
    """Batched ``env.sim.data`` view built from the simulator state (gym qpos / qvel layouts)."""

    def __init__(self, env):
        s, m = env.sim, env.sim.m
        E, tw = s.E, s.twins
        self.E = E
        z = torch.zeros(s.B, 1, device=s.dev)
        if m.layout == "slide3":
            qp = torch.cat([s.p[:, :1], s.p[:, 1:] - m.z_offset, s.th[:, None], s.q], 1)
            qv = torch.cat([s.v, s.w[:, None], s.qd], 1)
        elif m.layout == "free":
            half = 0.5 * s.th[:, None]
            qp = torch.cat([s.p[:, :1], z, s.p[:, 1:], torch.cos(half), z, -torch.sin(half), z, s.q], 1)
            qv = torch.cat([s.v[:, :1], z, s.v[:, 1:], z, -s.w[:, None], z, s.qd], 1)
        elif m.layout == "swim":
            qp = torch.cat([s.p, s.th[:, None], s.q], 1)
            qv = torch.cat([s.v, s.w[:, None], s.qd], 1)
        else:   # fixed-base arm + target slides
            qp = torch.cat([s.q, s.target], 1)
            qv = torch.cat([s.qd, torch.zeros(s.B, 2, device=s.dev)], 1)
        self.qpos = qp.reshape(E, -1)
        self.qvel = qv.reshape(E, -1)
        nv = self.qvel.shape[1]
        self.qfrc_actuator = torch.zeros(E, nv, device=s.dev)
        nroot = self.qvel.shape[1] // tw - s.J
        self.qfrc_actuator.view(E, tw, -1)[:, :, nroot:] = s.tau.view(E, tw, -1)
        nb = max(m.nbody, 1)
        cf = torch.zeros(s.B, nb, 6, device=s.dev)
        if m.nbody:
            if m.nbody > 1:
                cf[:, 1, 3], cf[:, 1, 5] = s.f_root[:, 0], s.f_root[:, 1]
            for l, b in enumerate(s.body_of_link):
                if 0 <= b < nb:
                    cf[:, b, 3] += s.f_end[:, l, 0]
                    cf[:, b, 5] += s.f_end[:, l, 1]
        self.cfrc_ext = cf.reshape(E, tw * nb, 6)
        self.cvel = torch.zeros(E, tw * nb, 6, device=s.dev)
        self.cinert = torch.zeros(E, tw * nb, 10, device=s.dev)
        if tw == 2:
            J = s.J
            q0 = s.q.view(E, 2, J)[:, :, 0]
            qd0 = s.qd.view(E, 2, J)[:, :, 0]
            self.ten_length = (q0[:, 0] - q0[:, 1])[:, None]
            self.ten_velocity = (qd0[:, 0] - qd0[:, 1])[:, None]
            tj = torch.zeros(E, 1, nv, device=s.dev)
            half = nv // 2
            tj[:, 0, 3], tj[:, 0, half + 3] = 1.0, -1.0
            self.ten_J = tj
        self._env = env

    def fingertip_dist(self):
        s = self._env.sim
        d = s.fingertip() - s.target
        return torch.cat([d, torch.zeros(s.B, 1, device=s.dev)], 1)


def robot_obs(env, d):
    """the robot's own ``_get_obs()`` (gym v2 layouts)"""
    sc = env.scenario
    if sc in ("HalfCheetah-v2", "half_cheetah", "coupled_half_cheetah"):
        return torch.cat([d.qpos[:, 1:], d.qvel], 1)
    if sc in ("Hopper-v2", "Walker2d-v2"):
        return torch.cat([d.qpos[:, 1:], d.qvel.clamp(-10, 10)], 1)
    if sc in ("Swimmer-v2", "manyagent_swimmer"):
        return torch.cat([d.qpos[:, 2:], d.qvel], 1)
    if sc in ("Ant-v2", "manyagent_ant"):
        return torch.cat([d.qpos[:, 2:], d.qvel, d.cfrc_ext.clamp(-1, 1).reshape(d.E, -1)], 1)
    if sc in ("Humanoid-v2", "HumanoidStandup-v2"):   # humanoid.py _get_obs: 22 + 23 + 140 + 84 + 23 + 84 = 376
        return torch.cat([d.qpos[:, 2:], d.qvel, d.cinert.reshape(d.E, -1), d.cvel.reshape(d.E, -1),
                          d.qfrc_actuator, d.cfrc_ext.reshape(d.E, -1)], 1)
    if sc == "Reacher-v2":
        th = d.qpos[:, :2]
        return torch.cat([torch.cos(th), torch.sin(th), d.qpos[:, 2:], d.qvel[:, :2], d.fingertip_dist()], 1)
    raise NotImplementedError(sc)


def _standardise(x):
    return (x - x.mean(-1, keepdim=True)) / x.std(-1, unbiased=False, keepdim=True)


class MujocoMultiVec:
    def __init__(self, scenario, agent_conf, n_envs, agent_obsk=None, k_categories=None, global_categories=None,
                 episode_limit=1000, device="cpu", seed=1, random_agent_order=False):
        self.scenario, self.agent_conf = scenario, agent_conf
        self.device = torch.device(device)
        self.E = int(n_envs)
        self.parts, self.edges, self.globals = graph.parts_and_edges(scenario, agent_conf)
        self.A = len(self.parts)
        self.acdims = [len(p) for p in self.parts]
        self.n_actions = graph.n_actions(self.parts)
        self.agent_obsk = agent_obsk
        if agent_obsk is not None:
            self.k_cats = graph.k_categories(scenario, agent_obsk, k_categories)
            self.global_cats = global_categories.split(",") if global_categories else self.k_cats[0]
            self.k_dicts = [graph.joints_at_kdist(i, self.parts, self.edges, k=agent_obsk) for i in range(self.A)]
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(int(seed))
        self.sim = PlanarSim(make_model(scenario, agent_conf), self.E, self.device, self.gen)
        if self.sim.m.layout != "fixed":
            nu = len(self.sim.m.act_joint) * self.sim.twins
            assert nu == sum(self.acdims), (scenario, agent_conf, nu, self.acdims)
        self.episode_limit = int(episode_limit)
        self.random_agent_order = bool(random_agent_order)
        self.steps = torch.zeros(self.E, dtype=torch.long, device=self.device)
        self.perm = torch.arange(self.A, device=self.device).repeat(self.E, 1)
        self.sim.reset()
        self._obs_size = None
        d = _Data(self)
        self._obs_size = max(o.shape[1] for o in self._agent_obs(d))
        self.obs_dim = self._obs_size + self.A
        self.state_dim = robot_obs(self, d).shape[1] + self.A
        self._eye = torch.eye(self.A, device=self.device)

    # ---------------------------------------------------------------------------------- spaces
    @property
    def n_agents(self):
        return self.A

    @property
    def observation_space(self):
        return [[self.obs_dim]] * self.A

    @property
    def share_observation_space(self):
        return [[self.state_dim]] * self.A

    @property
    def action_space(self):
        return [Box(-1.0, 1.0, n) for n in self.acdims]

    @property
    def policy_action_space(self):
        """what the MAT decodes per agent: the widest partition (padded entries are dropped by ``step``)"""
        return Box(-1.0, 1.0, self.n_actions)

    # ---------------------------------------------------------------------------------- observation
    def _agent_obs(self, d):
        if self.agent_obsk is None:
            o = robot_obs(self, d)
            return [o] * self.A
        return [graph.build_obs(d, self.k_dicts[i], self.k_cats, self.globals, self.global_cats,
                                vec_len=self._obs_size) for i in range(self.A)]

    def _observe(self):
        d = _Data(self)
        E, A = self.E, self.A
        eye = self._eye[None].expand(E, A, A)
        obs = torch.stack(self._agent_obs(d), 1)                                  # (E, A, n)
        obs = _standardise(torch.cat([obs, eye], -1))
        st = robot_obs(self, d)[:, None].expand(E, A, -1)
        share = _standardise(torch.cat([st, eye], -1))
        ava = torch.ones(E, A, self.n_actions, device=self.device)
        if self.random_agent_order:
            idx = self.perm[:, :, None]
            obs = obs.gather(1, idx.expand(-1, -1, obs.shape[-1]))
            share = share.gather(1, idx.expand(-1, -1, share.shape[-1]))
        return obs, share, ava

    def _new_perm(self, mask):
        if self.random_agent_order:
            r = torch.rand(self.E, self.A, generator=self.gen, device=self.device).argsort(1)
            self.perm = torch.where(mask[:, None], r, self.perm)

    def reset(self):
        m = torch.ones(self.E, dtype=torch.bool, device=self.device)
        self.sim.reset(m)
        self.steps.zero_()
        self._new_perm(m)
        return self._observe()

    # ---------------------------------------------------------------------------------- step
    def _reward_done(self, a, x0):
        s, sc = self.sim, self.scenario
        d = _Data(self)
        x1 = s.root_x()
        fwd = ((x1 - x0) / s.dt_env).mean(1)
        ctrl = (a * a).sum(1)
        qp = d.qpos
        finite = torch.isfinite(torch.cat([qp, d.qvel], 1)).all(1)
        if sc in ("HalfCheetah-v2", "half_cheetah"):
            return fwd - 0.1 * ctrl, ~finite
        if sc == "coupled_half_cheetah":
            return fwd - 0.1 * ctrl / 2.0, ~finite
        if sc == "Hopper-v2":
            st = torch.cat([qp, d.qvel], 1)[:, 2:]
            ok = finite & (st.abs() < 100).all(1) & (qp[:, 1] > 0.7) & (qp[:, 2].abs() < 0.2)
            return fwd + 1.0 - 1e-3 * ctrl, ~ok
        if sc == "Walker2d-v2":
            ok = finite & (qp[:, 1] > 0.8) & (qp[:, 1] < 2.0) & (qp[:, 2] > -1.0) & (qp[:, 2] < 1.0)
            return fwd + 1.0 - 1e-3 * ctrl, ~ok
        if sc in ("Swimmer-v2", "manyagent_swimmer"):
            return fwd - 1e-4 * ctrl, ~finite
        if sc in ("Ant-v2", "manyagent_ant"):
            contact = 0.5e-3 * d.cfrc_ext.clamp(-1, 1).square().sum((1, 2))
            ok = finite & (qp[:, 2] >= 0.2) & (qp[:, 2] <= 1.0)
            return fwd - 0.5 * ctrl - contact + 1.0, ~ok
        if sc == "Humanoid-v2":     # humanoid.py: 1.25 * COM velocity + 5 alive - 0.1 ctrl - contact cost
            contact = (5e-7 * d.cfrc_ext.square().sum((1, 2))).clamp(max=10.0)
            ok = finite & (qp[:, 2] > 1.0) & (qp[:, 2] < 2.0)
            return 1.25 * fwd + 5.0 - 0.1 * ctrl - contact, ~ok
        if sc == "HumanoidStandup-v2":   # uphill reward (z / dt) - ctrl - impact + 1, never terminates
            impact = (0.5e-6 * d.cfrc_ext.square().sum((1, 2))).clamp(max=10.0)
            return qp[:, 2] / s.dt_env - 0.1 * ctrl - impact + 1.0, ~finite
        if sc == "Reacher-v2":
            dist = (s.fingertip() - s.target).norm(dim=-1)
            return -dist - ctrl, ~finite
        raise NotImplementedError(sc)

    def step(self, actions):
        """actions (E, A, n_actions) in the (possibly permuted) agent order -> obs, share, rewards (E, A, 1),
        dones (E, A) bool, info, ava"""
        E, A = self.E, self.A
        act = actions.reshape(E, A, self.n_actions).float()
        if self.random_agent_order:
            rec = self.perm.argsort(1)                                            # agent_recovery
            act = act.gather(1, rec[:, :, None].expand(-1, -1, self.n_actions))
        flat = torch.cat([act[:, i, :self.acdims[i]] for i in range(A)], 1)
        x0 = self.sim.root_x().clone()
        self.sim.step(flat)
        self.steps += 1
        reward, term = self._reward_done(flat.clamp(-1, 1), x0)
        timeout = self.steps >= self.episode_limit
        done = term | timeout
        info = {"bad_transition": done & timeout & ~term, "terminated": term, "reward": reward}
        self.sim.reset(done)            # masked (no host sync on done.any())
        self.steps = torch.where(done, torch.zeros_like(self.steps), self.steps)
        self._new_perm(done)
        obs, share, ava = self._observe()
        rewards = reward.float()[:, None, None].expand(E, A, 1).contiguous()
        dones = done[:, None].expand(E, A).contiguous()
        return obs, share, rewards, dones, info, ava
