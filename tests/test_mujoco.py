"""Multi-agent MuJoCo: partition graphs / k-hop observations against the reference ``obsk.py``, the batched
surrogate env's multi-agent semantics, and the faulty-node runner.

The reference module (``mat_src/mat/envs/ma_mujoco/multiagent_mujoco/obsk.py``) needs only numpy, so it is loaded
straight from its file and fed a fake ``env.sim.data`` holding the same random arrays our batched ``_Data``
carries: partitions, edges, k-hop joint sets and the observation vectors must match exactly.  (The robots'
dynamics are a documented surrogate — MuJoCo is not installable — so no trajectory parity is claimed.)
"""
import importlib.util
import os
import types

import numpy as np
import pytest
import torch

import ref_oracle

from mat_dcml_amd.envs.mujoco import graph
from mat_dcml_amd.envs.mujoco.multi import MujocoMultiVec
from mat_dcml_amd.runner.mujoco_runner import faulty_action

CONFS = [("HalfCheetah-v2", "2x3"), ("HalfCheetah-v2", "6x1"), ("Ant-v2", "2x4"), ("Ant-v2", "2x4d"),
         ("Ant-v2", "4x2"), ("Ant-v2", "8x1"), ("Hopper-v2", "3x1"), ("Humanoid-v2", "9|8"), ("Humanoid-v2", "17x1"),
         ("Reacher-v2", "2x1"), ("Swimmer-v2", "2x1"), ("Walker2d-v2", "2x3"), ("Walker2d-v2", "6x1"),
         ("coupled_half_cheetah", "1p1"), ("manyagent_swimmer", "4x2"), ("manyagent_swimmer", "10x2"),
         ("manyagent_ant", "2x3"), ("manyagent_ant", "3x1")]

SIM_CONFS = [("HalfCheetah-v2", "6x1"), ("HalfCheetah-v2", "2x3"), ("Hopper-v2", "3x1"), ("Walker2d-v2", "2x3"),
             ("Swimmer-v2", "2x1"), ("Ant-v2", "2x4"), ("Ant-v2", "4x2"), ("Reacher-v2", "2x1"),
             ("coupled_half_cheetah", "1p1"), ("manyagent_swimmer", "4x2"), ("manyagent_ant", "2x2"),
             ("Humanoid-v2", "9|8"), ("HumanoidStandup-v2", "17x1")]


def _ref_obsk():
    path = os.path.join(ref_oracle.REF, "mat_src/mat/envs/ma_mujoco/multiagent_mujoco/obsk.py")
    spec = importlib.util.spec_from_file_location("_ref_obsk", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


needs_ref = pytest.mark.skipif(not ref_oracle.available(), reason="reference not present")


class _FakeData:
    """batched data (E = 1) + the reference-shaped numpy view of the same arrays"""

    def __init__(self, rng):
        self.E = 1
        a = lambda *s: rng.standard_normal(s).astype(np.float32) * 3
        self.np = dict(qpos=a(64), qvel=a(64), qfrc_actuator=a(64), cfrc_ext=a(64, 6), cvel=a(64, 6),
                       cinert=a(64, 10), ten_J=a(1, 64), ten_length=a(1), ten_velocity=a(1))
        for k, v in self.np.items():
            setattr(self, k, torch.from_numpy(v)[None])
        self.tip = a(3)

    def fingertip_dist(self):
        return torch.from_numpy(self.tip)[None]

    def ref_env(self):
        env = types.SimpleNamespace(sim=types.SimpleNamespace(data=types.SimpleNamespace(**self.np)))
        tip = self.tip
        env.get_body_com = lambda name: tip if name == "fingertip" else np.zeros(3, np.float32)
        return env


def _labels(nodes):
    return [n.label for n in nodes]


@needs_ref
@pytest.mark.parametrize("scenario,conf", CONFS)
def test_partition_graph_matches_reference(scenario, conf):
    ref = _ref_obsk()
    rp, re_, rg = ref.get_parts_and_edges(scenario, conf)
    mp, me, mg = graph.parts_and_edges(scenario, conf)
    assert [_labels(p) for p in rp] == [_labels(p) for p in mp]
    assert sorted(sorted(_labels(e.edges)) for e in re_) == sorted(sorted(_labels(e.edges)) for e in me)
    for key in ("joints", "bodies"):
        r, m = rg.get(key, []), mg.get(key, [])
        if key == "joints":
            assert _labels(r) == _labels(m)
            assert [(j.qpos_ids, j.qvel_ids, j.act_ids) for j in r] == [(j.qpos_ids, j.qvel_ids, j.act_ids) for j in m]
        else:
            assert list(r) == list(m)
    # ids of every partition joint
    for a, b in zip(rp, mp):
        assert [(j.qpos_ids, j.qvel_ids, j.act_ids) for j in a] == [(j.qpos_ids, j.qvel_ids, j.act_ids) for j in b]


@needs_ref
@pytest.mark.parametrize("scenario,conf", CONFS)
@pytest.mark.parametrize("k", [0, 1, 2])
def test_kdist_and_obs_match_reference(scenario, conf, k, capsys):
    ref = _ref_obsk()
    rp, re_, rg = ref.get_parts_and_edges(scenario, conf)
    mp, me, mg = graph.parts_and_edges(scenario, conf)
    cats = graph.k_categories(scenario, k)
    data = _FakeData(np.random.default_rng(k))
    for agent in range(len(mp)):
        rk = ref.get_joints_at_kdist(agent, rp, re_, k=k)
        mk = graph.joints_at_kdist(agent, mp, me, k=k)
        assert {h: _labels(v) for h, v in rk.items()} == {h: _labels(v) for h, v in mk.items()}
        mine = graph.build_obs(data, mk, cats, mg, cats[0])[0].numpy()
        try:
            theirs = ref.build_obs(data.ref_env(), rk, cats, rg, cats[0])
        except TypeError:
            # Reacher: the reference appends qpos[body].tolist() (a float) for the global bodies and raises
            assert scenario == "Reacher-v2"
            continue
        np.testing.assert_allclose(mine, np.asarray(theirs, dtype=np.float32), rtol=0, atol=0)
    capsys.readouterr()   # the reference prints its hyper-edges for k > 0


@pytest.mark.parametrize("scenario,conf", SIM_CONFS)
def test_env_semantics(scenario, conf):
    E = 6
    env = MujocoMultiVec(scenario, conf, E, agent_obsk=1, episode_limit=20, seed=3)
    obs, share, ava = env.reset()
    A = env.n_agents
    assert obs.shape == (E, A, env.obs_dim) and share.shape == (E, A, env.state_dim)
    assert ava.shape == (E, A, env.n_actions) and bool((ava == 1).all())
    # standardised per vector, one-hot id in the last A entries before standardisation
    torch.testing.assert_close(obs.mean(-1), torch.zeros(E, A), atol=1e-5, rtol=0)
    torch.testing.assert_close(obs.std(-1, unbiased=False), torch.ones(E, A), atol=1e-4, rtol=0)
    g = torch.Generator().manual_seed(0)
    n_done = 0
    for t in range(45):
        act = torch.rand(E, A, env.n_actions, generator=g) * 2 - 1
        obs, share, rew, dones, info, ava = env.step(act)
        assert torch.isfinite(obs).all() and torch.isfinite(share).all() and torch.isfinite(rew).all()
        assert rew.shape == (E, A, 1) and bool((rew == rew[:, :1]).all())
        assert bool((dones == dones[:, :1]).all())
        n_done += int(dones[:, 0].sum())
        if t == 19:   # every env has hit the 20-step limit (or terminated earlier) by now
            assert bool((env.steps <= 20).all())
    assert n_done >= E * 2           # time-limit auto-reset happened


def test_action_layout_and_faulty_node():
    env = MujocoMultiVec("Ant-v2", "2x4", 2, agent_obsk=0, seed=0)
    seen = {}
    orig = env.sim.step
    env.sim.step = lambda a: (seen.__setitem__("a", a.clone()), orig(a))
    act = torch.arange(16, dtype=torch.float32).view(1, 2, 8).expand(2, 2, 8)[:, :, :4].contiguous() / 20
    env.step(act)
    # agents' actions are concatenated in agent order — not reordered by their joints' actuator ids
    torch.testing.assert_close(seen["a"][0], torch.cat([act[0, 0], act[0, 1]]))
    f = faulty_action(act, 1)
    assert bool((f[:, 1] == 0).all()) and bool((f[:, 0] == act[:, 0]).all()) and bool((act[:, 1] != 0).any())
    assert faulty_action(act, -1) is act


def test_random_agent_order_is_a_consistent_permutation():
    a = MujocoMultiVec("HalfCheetah-v2", "6x1", 4, agent_obsk=1, seed=5)
    b = MujocoMultiVec("HalfCheetah-v2", "6x1", 4, agent_obsk=1, seed=5, random_agent_order=True)
    oa, _, _ = a.reset()
    ob, _, _ = b.reset()
    perm = b.perm
    assert not bool((perm == torch.arange(6)).all())
    torch.testing.assert_close(ob, oa.gather(1, perm[:, :, None].expand_as(oa)))
    # a permuted action for permuted agent j must reach the robot as canonical agent perm[j]'s action
    act = torch.rand(4, 6, 1)
    seen = {}
    orig = b.sim.step
    b.sim.step = lambda x: (seen.__setitem__("a", x.clone()), orig(x))
    b.step(act)
    canon = torch.empty_like(act)
    canon.scatter_(1, perm[:, :, None], act)
    torch.testing.assert_close(seen["a"], canon[:, :, 0])


def test_mujoco_runner_trains_on_cpu(tmp_path):
    import train_mujoco
    argv = train_mujoco.DEFAULT_ARGV + [
        "--cuda", "--n_rollout_threads", "4", "--episode_length", "20", "--num_env_steps", "160",
        "--num_mini_batch", "2", "--ppo_epoch", "2", "--eval_episodes", "2", "--eval_interval", "1",
        "--eval_faulty_node", "-1", "0", "--faulty_node", "1", "--episode_limit", "15", "--scenario",
        "HalfCheetah-v2", "--agent_conf", "2x3", "--agent_obsk", "1", "--results_dir", str(tmp_path)]
    runner = train_mujoco.main(argv)
    assert runner.policy.action_type == "Continuous"
    for p in runner.policy.transformer.parameters():
        assert torch.isfinite(p).all()
    res = runner.eval(0, n_steps=16)
    assert set(res) == {-1, 0}
    assert (tmp_path / "mujoco" / "HalfCheetah-v2" / "mat" / "single" / "run1" / "models").exists()


@pytest.mark.gpu
def test_mujoco_env_and_policy_on_gpu():
    env = MujocoMultiVec("Ant-v2", "4x2", 64, agent_obsk=1, device="cuda", seed=1)
    obs, share, ava = env.reset()
    for _ in range(10):
        obs, share, rew, dones, info, ava = env.step(torch.rand(64, 4, 2, device="cuda") * 2 - 1)
    torch.cuda.synchronize()
    assert torch.isfinite(obs).all() and obs.device.type == "cuda"


@pytest.mark.gpu
@pytest.mark.parametrize("scenario,conf", [("HalfCheetah-v2", "6x1"), ("Ant-v2", "2x4"), ("Reacher-v2", "2x1"),
                                           ("coupled_half_cheetah", "1p1"), ("manyagent_swimmer", "4x2"),
                                           ("Humanoid-v2", "9|8")])
def test_graph_captured_step_matches_eager(scenario, conf, monkeypatch):
    """the hipGraph replay of the sub-step loop must give the eager result (same kernels, same order)"""
    envs = []
    monkeypatch.setenv("MAT_DCML_ENV_FUSED", "0")
    for graphs in ("1", "0"):
        monkeypatch.setenv("MAT_DCML_ENV_GRAPHS", graphs)
        envs.append(MujocoMultiVec(scenario, conf, 32, agent_obsk=1, device="cuda", seed=4))
    assert envs[0].sim.use_graph and not envs[1].sim.use_graph
    g = torch.Generator(device="cuda").manual_seed(0)
    for t in range(12):
        act = torch.rand(32, envs[0].A, envs[0].n_actions, device="cuda", generator=g) * 2 - 1
        outs = [e.step(act) for e in envs]
        torch.testing.assert_close(outs[0][0], outs[1][0], rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(outs[0][2], outs[1][2], rtol=1e-4, atol=1e-4)
    for k in ("p", "th", "q", "qd"):
        torch.testing.assert_close(getattr(envs[0].sim, k), getattr(envs[1].sim, k), rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("scenario,conf", [("HalfCheetah-v2", "6x1"), ("Ant-v2", "2x4"), ("Reacher-v2", "2x1"),
                                           ("manyagent_swimmer", "4x2"), ("Swimmer-v2", "2x1"), ("Hopper-v2", "3x1"),
                                           ("Humanoid-v2", "9|8")])
def test_fused_planar_step_matches_torch(scenario, conf, monkeypatch):
    """csrc/planar_sim.hip (all sub-steps in one launch) vs the torch sub-step loop, one env step at a time from
    the same state (the torch state is copied into the fused sim before every step, so contact chaos cannot
    amplify rounding differences across steps)"""
    from mat_dcml_amd.ops import kernels
    kernels.lib()   # the fused path must be the native one
    envs = []
    for fused in ("1", "0"):
        monkeypatch.setenv("MAT_DCML_ENV_FUSED", fused)
        envs.append(MujocoMultiVec(scenario, conf, 96, agent_obsk=1, device="cuda", seed=4))
    assert envs[0].sim.use_fused and not envs[1].sim.use_fused
    fs, ts = envs[0].sim, envs[1].sim
    g = torch.Generator(device="cuda").manual_seed(0)
    for t in range(20):
        for k in fs._STATE:
            getattr(fs, k).copy_(getattr(ts, k))
        before = {k: getattr(fs, k) for k in fs._STATE}
        act = torch.rand(96, envs[0].A, envs[0].n_actions, device="cuda", generator=g) * 2 - 1
        outs = [e.step(act) for e in envs]
        # a contact point sitting exactly at zero penetration switches its damping term on or off depending on
        # the last bit of its height (fn = max(k pen - c vy, 0) * (pen > 0)), so an env may legitimately diverge
        # in a step; require nearly every env to agree and none to go non-finite
        ok = torch.ones(fs.B, dtype=torch.bool, device="cuda")
        err = torch.zeros(fs.B, device="cuda")
        for k in fs._STATE:
            a, b = getattr(fs, k), getattr(ts, k)
            assert a.data_ptr() == before[k].data_ptr()
            assert torch.isfinite(a).all()
            d = ((a - b).abs() / (1.0 + b.abs())).reshape(fs.B, -1).amax(1)
            ok &= d <= 2e-3
            err = torch.maximum(err, d)
        frac = ok.float().mean().item()
        if fs.m.kind == "ground":   # the contact switch exists only for ground models
            assert frac >= 0.9, f"step {t}: only {frac:.3f} of envs match"
        else:                           # fluid (swimmers) / arm (Reacher): smooth dynamics, every env must match
            assert frac == 1.0, f"step {t}: {fs.m.kind} model, only {frac:.3f} of envs match"
        assert err.median().item() < 1e-4, f"step {t}: median per-env error {err.median().item():.2e}"


def test_humanoid_layout():
    """Humanoid surrogate: gym's 376-dim observation, 17 actuators in the XML order, 9|8 partition"""
    env = MujocoMultiVec("Humanoid-v2", "9|8", 2, agent_obsk=None, seed=0)
    assert env.state_dim == 376 + 2 and env.acdims == [9, 8]
    d_qpos = env.sim.q.shape[1] + 7
    assert d_qpos == 24
