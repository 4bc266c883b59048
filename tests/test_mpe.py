"""MPE parity: the batched device env against the reference's per-object ``MultiAgentEnv`` (gym stubbed).

For every scenario the reference world is built and reset with numpy's RNG, its state (positions, velocities,
comm, goal / key choices) is copied into world 0 of a ``MPEVecEnv``, and both step with the same random joint
actions: observations (padded + agent id), rewards (shared when collaborative) and dones must match
(``mat_src/mat/envs/mpe/environment.py:122-170``).  ``simple_attack``'s reference reward raises ``NameError``
(``simple_attack.py:92``), so there only the physics and observations are compared.
"""
import types

import numpy as np
import pytest
import torch

import ref_oracle

from mat_dcml_amd.envs.mpe.env import MPEVecEnv

CASES = {
    "simple_spread": dict(num_agents=3, num_landmarks=3),
    "simple_reference": dict(num_agents=2, num_landmarks=3),
    "simple_speaker_listener": dict(num_agents=2, num_landmarks=3),
    "simple_push": dict(num_agents=2, num_landmarks=2),
    "simple_adversary": dict(num_agents=3, num_landmarks=2),
    "simple_tag": dict(num_adversaries=3, num_good_agents=1, num_landmarks=2),
    "simple_world_comm": dict(num_adversaries=4, num_good_agents=2, num_landmarks=1),
    "simple_crypto": dict(num_agents=3, num_landmarks=2),
    "simple_attack": dict(num_adversaries=2, num_good_agents=1, num_landmarks=3),
}


def _args(name, **kw):
    a = dict(scenario_name=name, episode_length=25, num_agents=3, num_landmarks=3, num_good_agents=1,
             num_adversaries=3)
    a.update(kw)
    return types.SimpleNamespace(**a)


def _ref_env(name, args):
    ref_oracle.install_stubs()
    ref_oracle.install_gym_stub()
    from mat.envs.mpe.environment import MultiAgentEnv
    from mat.envs.mpe.scenarios import load
    scn = load(name + ".py").Scenario()
    world = scn.make_world(args)
    return MultiAgentEnv(world, scn.reset_world, scn.reward, scn.observation, scn.info), scn


def _sync(env, world, name):
    w = env.world
    ents = world.agents + world.landmarks
    for i, e in enumerate(ents):
        w.pos[0, i] = torch.as_tensor(e.state.p_pos, dtype=w.dtype)
        w.vel[0, i] = torch.as_tensor(e.state.p_vel, dtype=w.dtype)
    for i, a in enumerate(world.agents):
        if w.dim_c and a.state.c is not None:
            w.c[0, i] = torch.as_tensor(a.state.c, dtype=w.dtype)
    lm = world.landmarks
    s = env.scenario
    if name == "simple_reference":
        s.goal_b[0] = torch.tensor([lm.index(world.agents[0].goal_b), lm.index(world.agents[1].goal_b)])
    elif name == "simple_speaker_listener":
        s.goal[0] = lm.index(world.agents[0].goal_b)
    elif name in ("simple_push", "simple_adversary"):
        s.goal[0] = lm.index(world.agents[0].goal_a)
    elif name == "simple_crypto":
        s.goal[0] = lm.index(world.agents[0].goal_a)
        s.key[0] = int(np.argmax(world.agents[2].key))


def _ref_action(env, i, a):
    nm, ns = int(env.n_move[i]), int(env.n_say[i])
    mv, sy = a // ns, a % ns
    parts = []
    if nm > 1:
        parts.append(np.eye(5)[mv])
    if bool(env.has_say[i]):
        parts.append(np.eye(env.world.dim_c)[sy])
    return np.concatenate(parts)


@pytest.mark.skipif(not ref_oracle.available(), reason="reference not mounted")
@pytest.mark.parametrize("name", list(CASES))
def test_mpe_matches_reference(name):
    np.random.seed(3)
    args = _args(name, **CASES[name])
    ref, scn = _ref_env(name, args)
    ref_obs = ref.reset()
    env = MPEVecEnv(args, n_envs=2, device="cpu", seed=0)
    env.world.dtype = torch.float64
    env.world.pos, env.world.vel, env.world.c = (x.double() for x in (env.world.pos, env.world.vel, env.world.c))
    _sync(env, ref.world, name)
    obs, share, ava = env._observe()
    assert obs.shape == (2, env.A, env.obs_dim) and share.shape == (2, env.A, env.obs_dim * env.A)
    for i, o in enumerate(ref_obs):
        n = len(o) - env.A
        np.testing.assert_allclose(obs[0, i, :n].numpy(), o[:n], atol=1e-9)
        np.testing.assert_allclose(obs[0, i, -env.A:].numpy(), o[n:])
    rng = np.random.RandomState(7)
    n_i = (env.n_move * env.n_say).tolist()
    for t in range(env.world_length):
        acts = [int(rng.randint(n_i[i])) for i in range(env.A)]
        a = torch.tensor([acts, acts])
        if name == "simple_attack":
            for i, agent in enumerate(ref.agents):
                ref._set_action(_ref_action(env, i, acts[i]), agent, ref.action_space[i])
            ref.world.step()
            ref.current_step += 1
            robs = [np.concatenate([ref._get_obs(ag), np.eye(env.A)[i]]) for i, ag in enumerate(ref.agents)]
            rrew = rdone = None
        else:
            robs, rrew, rdone, _ = ref.step([_ref_action(env, i, acts[i]) for i in range(env.A)])
        obs, share, rew, dones, info, ava = env.step(a)
        if t == env.world_length - 1:
            assert bool(dones.all())
            break
        assert not bool(dones.any())
        for i, o in enumerate(robs):
            np.testing.assert_allclose(obs[0, i, :len(o) - env.A].numpy(), o[:-env.A], atol=1e-5, rtol=1e-5,
                                       err_msg=f"{name} obs agent {i} step {t}")
        if rrew is not None:
            np.testing.assert_allclose(rew[0, :, 0].numpy(), np.array(rrew)[:, 0], atol=1e-5, rtol=1e-5,
                                       err_msg=f"{name} reward step {t}")
            assert not any(rdone)


def test_mpe_spaces_and_autoreset():
    args = _args("simple_speaker_listener", num_agents=2, num_landmarks=3, episode_length=5)
    env = MPEVecEnv(args, n_envs=4, seed=1)
    # speaker: Discrete(3) say; listener: Discrete(5) move → joint space 5, speaker masked to 3
    assert env.n_actions == 5
    assert env.ava.tolist() == [[1, 1, 1, 0, 0], [1, 1, 1, 1, 1]]
    assert type(env.agent_spaces[0]).__name__ == "Discrete" and env.agent_spaces[0].n == 3
    obs, share, ava = env.reset()
    p0 = env.world.pos.clone()
    for t in range(5):
        obs, share, r, d, info, ava = env.step(torch.zeros(4, 2, dtype=torch.long))
    assert bool(d.all()) and int(env.ep_step.max()) == 0
    assert not torch.allclose(env.world.pos, p0)          # fresh episode sampled
    assert torch.equal(r[:, 0], r[:, 1])                  # collaborative: shared reward


def test_mpe_onehot_step_equals_index_step():
    args = _args("simple_world_comm", num_adversaries=4, num_good_agents=2, num_landmarks=1)
    e1, e2 = MPEVecEnv(args, 3, seed=5), MPEVecEnv(args, 3, seed=5)
    leader = e1.agent_spaces[0]
    assert type(leader).__name__ == "MultiDiscrete" and leader.n == 20
    g = torch.Generator().manual_seed(0)
    for _ in range(4):
        n_i = (e1.n_move * e1.n_say)
        a = (torch.rand(3, e1.A, generator=g) * n_i).long()
        oh = []
        for i in range(e1.A):
            mv, sy = a[:, i] // e1.n_say[i], a[:, i] % e1.n_say[i]
            parts = [torch.nn.functional.one_hot(mv, 5).float()]
            if bool(e1.has_say[i]):
                parts.append(torch.nn.functional.one_hot(sy, 4).float())
            x = torch.cat(parts, 1)
            oh.append(torch.nn.functional.pad(x, (0, 9 - x.shape[1])))
        r1 = e1.step(a)
        r2 = e2.step_onehot(torch.stack(oh, 1))
        assert torch.equal(r1[0], r2[0]) and torch.equal(r1[2], r2[2])


def _runner_args(scenario, **kw):
    from mat_dcml_amd.config import _MPE_FLAGS, get_config, parse_args
    argv = ["--env_name", "MPE", "--scenario_name", scenario, "--n_block", "1", "--n_rollout_threads", "4",
            "--episode_length", "25", "--num_env_steps", "200", "--ppo_epoch", "2", "--num_mini_batch", "1",
            "--lr", "7e-4", "--clip_param", "0.05", "--n_eval_rollout_threads", "2", "--use_eval"]
    for k, v in kw.items():
        argv += [f"--{k}", str(v)]
    a = parse_args(argv, get_config(), extra=_MPE_FLAGS, warn=False)
    a.scenario = a.scenario_name
    return a


@pytest.mark.parametrize("scenario,kw", [("simple_spread", {}),
                                         ("simple_speaker_listener", {"num_agents": 2}),
                                         ("simple_world_comm", {"num_adversaries": 2, "num_good_agents": 1,
                                                                "num_landmarks": 1})])
def test_mpe_runner_trains_cpu(scenario, kw):
    from mat_dcml_amd.runner.mpe_runner import MPERunner
    torch.manual_seed(0)
    a = _runner_args(scenario, **kw)
    r = MPERunner({"all_args": a, "device": "cpu", "run_dir": None})
    r.warmup()
    p0 = torch.cat([p.detach().flatten().clone() for p in r.policy.transformer.parameters()])
    infos = r.train_iteration()
    p1 = torch.cat([p.detach().flatten() for p in r.policy.transformer.parameters()])
    assert torch.isfinite(p1).all() and not torch.equal(p0, p1)
    assert all(np.isfinite(float(v)) for v in infos.values())
    # masked joint actions never exceed an agent's own action count
    n_i = (r.envs.n_move * r.envs.n_say).view(1, 1, -1, 1)
    assert bool((r.buffer.actions < n_i).all())
    assert np.isfinite(r.eval())


@pytest.mark.gpu
def test_mpe_spread_learns_gpu(gpu):
    """MAT on simple_spread (train_mpe.sh hyper-parameters, fused HIP path) improves the episode return."""
    from mat_dcml_amd.runner.mpe_runner import MPERunner
    torch.manual_seed(1)
    a = _runner_args("simple_spread", n_rollout_threads=128, ppo_epoch=10)
    r = MPERunner({"all_args": a, "device": gpu, "run_dir": None})
    assert r.policy._fused()
    r.warmup()
    first = None
    for it in range(40):
        r.train_iteration()
        ret = float(r.buffer.rewards.mean()) * 25
        first = ret if first is None else first
    assert ret > first + 20, (first, ret)


def test_render_gif(tmp_path):
    """MPE runner render (mpe_runner.py:193-254): deterministic episodes, one frame per step plus the reset frame,
    written as an animated GIF"""
    from PIL import Image
    from mat_dcml_amd.config import _MPE_FLAGS, get_config, parse_args
    from mat_dcml_amd.runner.mpe_runner import MPERunner
    args = parse_args(["--env_name", "MPE", "--scenario_name", "simple_spread", "--num_agents", "3",
                       "--num_landmarks", "3", "--n_rollout_threads", "2", "--episode_length", "5", "--n_block", "1",
                       "--use_render", "--save_gifs", "--render_episodes", "2"], get_config(), extra=_MPE_FLAGS,
                      warn=False)
    args.scenario = args.scenario_name
    r = MPERunner({"all_args": args, "device": torch.device("cpu"), "run_dir": tmp_path})
    frames = r.render()
    assert len(frames) == 2 * (5 + 1) and frames[0].shape == (400, 400, 3)
    agent_px = (frames[0] == (89, 89, 217)).all(-1).sum()      # AGENT_RGB
    assert agent_px > 0
    gif = Image.open(tmp_path / "gifs" / "render.gif")
    assert gif.n_frames >= 2
