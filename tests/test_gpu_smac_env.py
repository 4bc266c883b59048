"""SMAC-shaped env kernel (csrc/smac_env.hip: step + battle reset + observation build, one launch) vs the torch
env (envs/smac/synthetic.py) on identical Philox draws and identical actions."""
import pytest
import torch

from mat_dcml_amd.envs.smac.synthetic import SyntheticSMACEnv

pytestmark = pytest.mark.gpu


def _feat_close(a, b):
    """Observation / state features: the unit distances go through a square root whose last bit differs between
    the device and torch's kernels (measured: 1 ulp on ~2 % of the distance features); everything else — the
    battle state, masks, availability, dones, rewards' inputs — is compared exactly."""
    torch.testing.assert_close(a, b, rtol=3e-7, atol=0.0)
    assert ((a != b).float().mean() < 0.05), float((a != b).float().mean())


@pytest.mark.parametrize("map_name,rao", [("27m_vs_30m", False), ("27m_vs_30m", True), ("3m", True), ("MMM", False),
                                          ("2c_vs_64zg", False)])
def test_smac_env_kernel_matches_torch(gpu, map_name, rao):
    E = 24
    hip = SyntheticSMACEnv(E, map_name, device=gpu, seed=11, random_agent_order=rao, env_id_offset=5, backend="hip")
    ref = SyntheticSMACEnv(E, map_name, device=gpu, seed=11, random_agent_order=rao, env_id_offset=5, backend="torch")
    assert hip._kern is not None and ref._kern is None
    o1, o2 = hip.reset(), ref.reset()
    _feat_close(o1[0], o2[0])
    _feat_close(o1[1], o2[1])
    assert torch.equal(o1[2], o2[2])
    g = torch.Generator(device=gpu).manual_seed(0)
    ava = o2[2]
    A, nA = hip.A, hip.n_actions
    steps = 250 if map_name == "3m" else 120
    n_done = 0
    for t in range(steps):
        # mostly attacks / moves among the available actions (battles end inside the test)
        w = ava * torch.where(torch.arange(nA, device=gpu) >= 6, 4.0, 1.0)
        act = torch.multinomial(w.reshape(-1, nA), 1, generator=g).view(E, A).float()
        r1, r2 = hip.step(act), ref.step(act)
        obs1, st1, rew1, d1, inf1, av1 = r1
        obs2, st2, rew2, d2, inf2, av2 = r2
        assert torch.equal(d1, d2), t
        for k in ("won", "lost", "bad_transition"):
            assert torch.equal(inf1[k], inf2[k]), (t, k)
        for k in ("battles_won", "battles_game", "dead_allies", "dead_enemies"):
            assert torch.equal(inf1[k].float(), inf2[k].float()), (t, k)
        torch.testing.assert_close(rew1, rew2, rtol=1e-6, atol=1e-7)   # Σ damage: reduction order differs
        assert torch.equal(av1, av2), t
        _feat_close(obs1, obs2)
        _feat_close(st1, st2)
        for name in ("apos", "ahp", "epos", "ehp", "perm", "last", "t", "ep_ctr"):
            assert torch.equal(getattr(hip, name), getattr(ref, name)), (t, name)
        n_done += int(inf2["won"].sum() + inf2["lost"].sum() + inf2["bad_transition"].sum())
        ava = av2
    assert n_done > 0   # battle resets were exercised


def test_smac_env_kernel_is_one_launch_and_fast(gpu):
    E = 32
    env = SyntheticSMACEnv(E, "27m_vs_30m", device=gpu, seed=1, backend="hip")
    _, _, ava = env.reset()
    act = torch.ones(E, env.A, device=gpu)
    for _ in range(3):
        env.step(act)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        env.step(act)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / 20 * 1e3
    print(f"smac env step, 32 envs x 27 agents (obs 1288, state 1458): {us:.1f} us")
    assert us < 200


def _smac_runner(gpu, envs=8, T=6):
    from mat_dcml_amd.config import _SMAC_FLAGS, get_config, parse_args
    from mat_dcml_amd.runner.smac_runner import SMACRunner
    argv = ["--env_name", "StarCraft2", "--algorithm_name", "mat", "--map_name", "27m_vs_30m", "--n_rollout_threads",
            str(envs), "--episode_length", str(T), "--use_value_active_masks", "--seed", "2"]
    args = parse_args(argv, get_config(), extra=_SMAC_FLAGS, warn=False)
    r = SMACRunner({"all_args": args, "device": gpu, "run_dir": None})
    from mat_dcml_amd.ops import mat_fused
    mat_fused.set_sampling_key(r.policy.transformer, 2, env0=0)   # the same exploration draws in both runners
    r.warmup()
    return r


def test_smac_fused_insert_matches_torch_insert(gpu):
    """runner/smac_runner._insert_fused (one launch, csrc/rl_ops.hip smac_insert_kernel) vs the torch _track_smac +
    _insert_smac on the same rollout: identical buffers (rewards, masks, active masks, slots) and episode statistics."""
    fused, ref = _smac_runner(gpu), _smac_runner(gpu)
    ref._ins_ok = False
    for _ in range(3):   # battles finish within the episode (limit) so the done / active branches are exercised
        fused.rollout()
        ref.rollout()
        fused.buffer.after_update()
        ref.buffer.after_update()
    torch.cuda.synchronize()
    assert fused._ins_ok
    for k in ("obs", "available_actions", "actions", "action_log_probs", "value_preds", "rewards", "masks",
              "active_masks"):
        a, b = getattr(fused.buffer, k), getattr(ref.buffer, k)
        assert torch.equal(a, b), (k, (a - b).abs().max())
    assert torch.equal(fused._ep_reward, ref._ep_reward)
    torch.testing.assert_close(fused._done_stats, ref._done_stats, rtol=1e-12, atol=1e-9)
