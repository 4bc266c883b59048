"""SMAC random agent order and multi-map training (``Random_StarCraft2_Env.py``, ``Random_StarCraft2_Env_Multi.py``,
``feature_translation.py``, ``train_smac_multi.py``).

The unified-layout translation is checked against the reference's own ``single_translate_local`` /
``gen_task_embedding`` (pysc2 stubbed: only its map registry is needed) on Terran maps, where the synthetic
env's features line up with SMAC's (no shields, no unit-type bits).
"""
import sys
import types

import numpy as np
import pytest
import torch

import ref_oracle

from mat_dcml_amd.envs.smac.maps import get_map
from mat_dcml_amd.envs.smac.multi import LOCAL_DIM, TASK_DIM, UNIFIED, SyntheticSMACMultiEnv, UnifiedTranslator, \
    task_embedding
from mat_dcml_amd.envs.smac.synthetic import SyntheticSMACEnv


def _ft():
    ref_oracle.install_stubs()
    if "pysc2" not in sys.modules:
        p, m, lib = (types.ModuleType(n) for n in ("pysc2", "pysc2.maps", "pysc2.maps.lib"))
        lib.Map = type("Map", (), {})
        m.lib, p.maps = lib, m
        sys.modules.update({"pysc2": p, "pysc2.maps": m, "pysc2.maps.lib": lib})
    from mat.envs.starcraft2 import feature_translation as ft
    return ft


def _to_reference_order(obs, spec):
    """synthetic [move, enemy, ally, own, id] -> SMAC [ally, enemy, move, own+id] (Terran, u=0)"""
    A, N, nA = spec.n_agents, spec.n_enemies, spec.n_actions
    o = 0
    move = obs[..., :4]
    o = 4
    enemy = obs[..., o: o + N * 5]
    o += N * 5
    ally = obs[..., o: o + (A - 1) * (5 + nA)]
    o += (A - 1) * (5 + nA)
    own = obs[..., o:]
    return torch.cat([ally, enemy, move, own], -1)


@pytest.mark.skipif(not ref_oracle.available(), reason="reference not mounted")
def test_task_embedding_matches_reference():
    ft = _ft()
    for m in UNIFIED:
        np.testing.assert_allclose(task_embedding(m).numpy(), ft.gen_task_embedding(m), atol=1e-7, err_msg=m)


@pytest.mark.skipif(not ref_oracle.available(), reason="reference not mounted")
@pytest.mark.parametrize("map_name", ["3m", "5m_vs_6m", "8m_vs_9m"])
def test_unified_translation_matches_reference(map_name, monkeypatch):
    monkeypatch.setattr(np, "int", int, raising=False)    # the reference still uses the removed np.int alias
    ft = _ft()
    env = SyntheticSMACEnv(2, map_name, seed=3)
    tr = UnifiedTranslator(map_name, "cpu")
    spec = env.spec
    obs, _, ava = env.reset()
    for t in range(12):
        got = tr(obs)
        ref_in = _to_reference_order(obs, spec).double().numpy()
        want = ft.translate_local_obs(ref_in.reshape(-1, ref_in.shape[-1]))
        np.testing.assert_allclose(got.reshape(-1, LOCAL_DIM + TASK_DIM).numpy(), want, atol=1e-6,
                                   err_msg=f"{map_name} step {t}")
        obs, _, _, _, _, ava = env.step(torch.multinomial(ava.reshape(-1, ava.shape[-1]), 1).view(2, -1))


def test_random_agent_order_is_a_row_permutation():
    a = SyntheticSMACEnv(3, "8m", seed=5, random_agent_order=False)
    b = SyntheticSMACEnv(3, "8m", seed=5, random_agent_order=True)
    oa, sa, va = a.reset()
    ob, sb, vb = b.reset()
    perm = b.perm
    assert not torch.equal(perm, torch.arange(8).expand(3, 8))
    g = lambda x: torch.gather(x, 1, perm.view(3, 8, 1).expand_as(x))          # noqa: E731
    assert torch.equal(ob, g(oa)) and torch.equal(sb, g(sa)) and torch.equal(vb, g(va))
    act = torch.multinomial(va.reshape(-1, va.shape[-1]), 1).view(3, 8)
    ra = a.step(act)
    rb = b.step(torch.gather(act, 1, perm))        # policy row j acts for agent perm[j]
    assert torch.equal(rb[0], g(ra[0])) and torch.equal(rb[3], torch.gather(ra[3], 1, perm))
    assert torch.equal(a.apos, b.apos) and torch.equal(a.ehp, b.ehp)


def test_multi_env_padding_and_step():
    env = SyntheticSMACMultiEnv(["3m", "8m_vs_9m"], 4, seed=1)
    obs, share, ava = env.reset()
    assert obs.shape == (4, 27, LOCAL_DIM + TASK_DIM) and ava.shape == (4, 27, 38)
    D = LOCAL_DIM + TASK_DIM
    # 3m: agents 3..26 are fake: a single 1 marker, every action available
    assert torch.all(ava[:2, 3:] == 1) and torch.all(ava[:2, :3, 9:] == 0)
    assert torch.all(obs[:2, 3:].sum(-1) == 1)
    assert float(obs[0, 26, D - 1]) == 1.0 and float(obs[0, 3, D - 24]) == 1.0
    np.testing.assert_allclose(obs[:2, :3, LOCAL_DIM:].numpy(), task_embedding("3m").expand(2, 3, -1).numpy())
    for _ in range(5):
        act = torch.multinomial(ava.reshape(-1, 38), 1).view(4, 27)
        obs, share, r, d, info, ava = env.step(act)
        assert torch.all(d[:2, 3:]) and torch.all(d[2:, 8:])
        assert r.shape == (4, 27, 1) and info["won"].shape == (4,)


def test_multi_map_runner_trains_cpu(tmp_path):
    import train_smac
    argv = train_smac.DEFAULT_ARGV + ["--train_maps", "3m", "2s3z", "--random_agent_order", "--n_rollout_threads",
                                      "4", "--episode_length", "6", "--num_env_steps", "24", "--ppo_epoch", "1",
                                      "--n_embd", "32", "--cuda", "--results_dir", str(tmp_path), "--log_interval",
                                      "1", "--eval_episodes", "2", "--eval_interval", "1",
                                      "--n_eval_rollout_threads", "2", "--eval_maps", "3m", "8m"]
    runner = train_smac.main(argv)
    assert runner.num_agents == 27 and runner.envs.observation_space[0][0] == 2029
    assert isinstance(runner.eval_envs, SyntheticSMACMultiEnv) and runner.eval_envs.maps == ["3m", "8m"]
    assert torch.isfinite(torch.cat([p.flatten() for p in runner.policy.transformer.parameters()])).all()
    assert get_map("2s3z").unit_type_bits == 2
