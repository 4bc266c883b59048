"""Google Research Football: the batched observation / availability / reward encoders against the reference's
per-player numpy ``FeatureEncoder`` / ``Rewarder`` (``mat_src/mat/envs/football/encode/``), plus the synthetic
match env and runner.  gfootball itself is not installable, so the raw observations are random GRF-shaped dicts
covering every branch (ownership, set pieces, ball zones, sticky actions, time-out, yellow cards)."""
import importlib.util
import os

import numpy as np
import pytest
import torch

import ref_oracle

from mat_dcml_amd.envs.football import encode as enc
from mat_dcml_amd.envs.football.synthetic import SCENARIOS, SyntheticFootballEnv

needs_ref = pytest.mark.skipif(not ref_oracle.available(), reason="reference not present")


def _load(rel):
    path = os.path.join(ref_oracle.REF, "mat_src/mat/envs/football/encode", rel)
    spec = importlib.util.spec_from_file_location("_ref_" + rel[:-3], path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _raw(rng, E, A, NL=5, NR=3):
    f = lambda *s: rng.uniform(-1, 1, s).astype(np.float32)
    ball = np.stack([rng.choice([-0.9, -0.5, 0.0, 0.5, 0.8, 0.95], E) + rng.uniform(-0.05, 0.05, E),
                     rng.choice([0.0, 0.2, -0.35, 0.41], E), rng.uniform(0, 0.1, E)], 1).astype(np.float32)
    left = f(E, NL, 2) * np.array([1, 0.42], np.float32)
    near = rng.random(E) < 0.4          # put the ball at an active player's feet sometimes
    active = np.stack([rng.permutation(NL)[:A] for _ in range(E)])
    ball[near, :2] = left[near, active[near, 0]] + 0.01
    return {
        "left_team": left, "left_team_direction": f(E, NL, 2) * 0.01,
        "left_team_roles": rng.integers(0, 10, (E, NL)), "left_team_tired_factor": rng.uniform(0, 0.1, (E, NL)),
        "left_team_yellow_card": rng.integers(0, 2, (E, NL)).astype(np.float32),
        "right_team": f(E, NR, 2) * np.array([1, 0.42], np.float32), "right_team_direction": f(E, NR, 2) * 0.01,
        "right_team_tired_factor": rng.uniform(0, 0.1, (E, NR)),
        "right_team_yellow_card": rng.integers(0, 2, (E, NR)).astype(np.float32),
        "ball": ball, "ball_direction": f(E, 3) * 0.02, "ball_owned_team": rng.choice([-1, 0, 1], E),
        "ball_owned_player": rng.integers(0, NL, E), "game_mode": rng.choice([0, 0, 2, 4, 6], E),
        "score": rng.integers(0, 3, (E, 2)).astype(np.float32), "steps_left": rng.choice([0, 5, 100], E),
        "active": active, "sticky_actions": rng.integers(0, 2, (E, A, 10)).astype(np.float32),
    }


def _one(raw, e, a):
    d = {k: v[e] for k, v in raw.items() if k not in ("active", "sticky_actions")}
    d["active"] = int(raw["active"][e, a])
    d["sticky_actions"] = raw["sticky_actions"][e, a]
    d["ball_owned_team"] = int(d["ball_owned_team"])
    d["game_mode"] = int(d["game_mode"])
    d["steps_left"] = int(d["steps_left"])
    return d


def _t(raw):
    return {k: torch.from_numpy(np.asarray(v)) for k, v in raw.items()}


@needs_ref
@pytest.mark.parametrize("seed", range(4))
def test_feature_encoder_matches_reference(seed):
    ref = _load("obs_encode.py").FeatureEncoder()
    rng = np.random.default_rng(seed)
    E, A = 40, 3
    raw = _raw(rng, E, A)
    feats, avail = enc.encode(_t(raw))
    for e in range(E):
        for a in range(A):
            o = ref.encode(_one(raw, e, a))
            cat = np.hstack([np.array(o[k], dtype=np.float32).flatten() for k in sorted(o)])
            np.testing.assert_allclose(feats[e, a].numpy(), cat, rtol=1e-5, atol=1e-5, err_msg=f"env {e} agent {a}")
            np.testing.assert_array_equal(avail[e, a].numpy(), o["avail"])


@needs_ref
@pytest.mark.parametrize("seed", range(3))
def test_rewarder_matches_reference(seed):
    mod = _load("rew_encode.py")
    rng = np.random.default_rng(100 + seed)
    E, A = 30, 3
    prev, now = _raw(rng, E, A), _raw(rng, E, A)
    sig = rng.choice([-1.0, 0.0, 0.0, 1.0], (E, A)).astype(np.float32)
    mine = enc.reward(torch.from_numpy(sig), _t(prev), _t(now)).numpy()
    for e in range(E):
        for a in range(A):
            r = mod.Rewarder().calc_reward(float(sig[e, a]), _one(prev, e, a), _one(now, e, a))
            assert abs(mine[e, a] - r) < 1e-5, (e, a, mine[e, a], r)


@pytest.mark.parametrize("scenario", sorted(SCENARIOS))
def test_synthetic_match_runs(scenario):
    A = min(3, len(SCENARIOS[scenario]["left"]) - 1)
    env = SyntheticFootballEnv(scenario, A, 16, seed=2)
    obs, share, ava = env.reset()
    assert obs.shape == (16, A, env.obs_dim) and ava.shape == (16, A, 19)
    g = torch.Generator().manual_seed(0)
    for _ in range(120):
        act = torch.multinomial(ava.reshape(-1, 19), 1, generator=g).view(16, A)
        obs, share, r, dones, info, ava = env.step(act)
        assert torch.isfinite(obs).all() and torch.isfinite(r).all()
        assert bool((ava.sum(-1) > 0).all())
        assert bool((dones == dones[:, :1]).all())
    assert float(env.battles_game.sum()) > 0


def test_football_runner_trains_on_cpu(tmp_path):
    import train_football
    argv = train_football.DEFAULT_ARGV + [
        "--cuda", "--n_rollout_threads", "4", "--episode_length", "16", "--num_env_steps", "128", "--ppo_epoch", "2",
        "--eval_episodes", "2", "--eval_interval", "1", "--results_dir", str(tmp_path)]
    runner = train_football.main(argv)
    for p in runner.policy.transformer.parameters():
        assert torch.isfinite(p).all()
    assert (tmp_path / "football" / "academy_3_vs_1_with_keeper" / "mat" / "single" / "run1").exists()
