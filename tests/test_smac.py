"""SMAC stress config: map shapes, synthetic env contract, MAT training on it, CPU process-pool vec env."""
import numpy as np
import torch

from mat_dcml_amd.envs.smac.maps import get_map
from mat_dcml_amd.envs.smac.synthetic import SyntheticSMACEnv


def test_map_shapes_match_reference_formulas():
    s = get_map("27m_vs_30m")
    assert (s.obs_dim, s.state_dim, s.n_actions, s.limit) == (1288, 1458, 36, 180)
    m = get_map("MMM")
    assert m.n_actions == 16 and m.unit_type_bits == 3


def test_synthetic_env_contract():
    env = SyntheticSMACEnv(3, "3m", seed=0)
    obs, state, ava = env.reset()
    spec = env.spec
    assert obs.shape == (3, 3, spec.obs_dim) and state.shape == (3, 3, spec.state_dim) and ava.shape == (3, 3, 9)
    assert torch.all(ava[..., 0] == 0) and torch.all(ava[..., 1] == 1)      # alive: no-op unavailable, stop ok
    games = 0
    for t in range(200):
        act = torch.multinomial(ava.reshape(-1, 9), 1).view(3, 3)
        obs, state, r, dones, info, ava = env.step(act)
        assert torch.all(r >= 0)                                           # reward_only_positive
        dead = dones & ~dones.all(1, keepdim=True)
        if dead.any():                                                     # dead agents: only no-op available
            assert torch.all(ava[dead][:, 0] == 1) and torch.all(ava[dead][:, 1:] == 0)
    assert float(info["battles_game"].sum()) >= 3                          # limit 60: several episodes finished


def test_mat_trains_on_synthetic_smac(tmp_path):
    import train_smac
    argv = train_smac.DEFAULT_ARGV + ["--map_name", "3m", "--n_rollout_threads", "4", "--episode_length", "8",
                                      "--num_env_steps", "64", "--ppo_epoch", "2", "--n_embd", "32", "--cuda",
                                      "--results_dir", str(tmp_path), "--log_interval", "1", "--eval_episodes", "2",
                                      "--eval_interval", "1", "--n_eval_rollout_threads", "2"]
    runner = train_smac.main(argv)
    assert list((tmp_path / "StarCraft2").rglob("transformer_*.pt"))
    assert runner.buffer.active_masks.min() >= 0


class _ToyEnv:
    """Tiny CPU env with the reference wrapper contract (obs, share, ava / step 6-tuple)."""

    def __init__(self, k):
        self.k, self.t = k, 0
        self.observation_space = [[3]] * 2
        self.share_observation_space = [[4]] * 2
        self.action_space = [None] * 2
        self.n_agents = 2

    def reset(self):
        self.t = 0
        return np.full((2, 3), self.k, np.float32), np.zeros((2, 4), np.float32), np.ones((2, 5), np.float32)

    def step(self, a):
        self.t += 1
        ob = np.full((2, 3), self.k + self.t, np.float32)
        return ob, np.zeros((2, 4), np.float32), np.full((2, 1), float(a.sum())), np.array([self.t >= 3] * 2), \
            [{}, {}], np.ones((2, 5), np.float32)


def _toy(k):
    return lambda: _ToyEnv(k)


def test_process_pool_vec_env():
    from mat_dcml_amd.envs.vec.process_pool import ProcessPoolVecEnv
    pool = ProcessPoolVecEnv([_toy(k) for k in range(5)], n_workers=2, context="fork")
    try:
        obs, share, ava = pool.reset()
        assert obs.shape == (5, 2, 3) and torch.allclose(obs[:, 0, 0], torch.arange(5.0))
        acts = torch.arange(10.0).view(5, 2, 1)
        for t in range(3):
            obs, share, rew, done, info, ava = pool.step(acts)
        assert torch.allclose(rew[:, 0, 0], acts.sum((1, 2)))
        assert done.all() and torch.allclose(obs[:, 0, 0], torch.arange(5.0))   # auto-reset after 3 steps
    finally:
        pool.close()


class _FlakySC2:
    """Stand-in for smac's StarCraft2Env: raises a protocol error on chosen step calls (per game instance)."""
    launches = 0

    def __init__(self, fail_on=()):
        _FlakySC2.launches += 1
        self.fail_on, self.t = set(fail_on), 0

    def get_env_info(self):
        return {"n_agents": 3, "obs_shape": 5, "state_shape": 7, "n_actions": 4}

    def reset(self):
        self.t = 0

    def step(self, actions):
        self.t += 1
        if self.t in self.fail_on:
            raise ConnectionError("SC2 protocol error")
        return 1.0, False, {"battle_won": False}

    def get_obs(self):
        return [np.full(5, self.t, np.float32)] * 3

    def get_state(self):
        return np.zeros(7, np.float32)

    def get_avail_actions(self):
        return [[1, 1, 1, 1]] * 3

    def close(self):
        pass


def test_sc2_protocol_error_full_restart():
    """StarCraft2_Env.py:468-472,507-530: a protocol error in step relaunches the game, ends the episode (every agent
    done, zero reward) and the running restart count is in every info dict."""
    from mat_dcml_amd.envs.smac.adapter import SC2Game
    made = []

    def make_env():
        made.append(_FlakySC2(fail_on=(2,) if not made else ()))
        return made[-1]
    g = SC2Game(make_env, errors=(ConnectionError,))
    obs, state, ava = g.reset()
    assert obs.shape == (3, 5) and state.shape == (3, 7) and ava.shape == (3, 4)
    o, s, r, d, info, a = g.step([0, 1, 2])
    assert not d.any() and r[0, 0] == 1.0 and info[0]["restarts"] == 0
    o, s, r, d, info, a = g.step([0, 1, 2])          # the first game fails on its 2nd step
    assert d.all() and r[0, 0] == 0.0 and all(i["restarts"] == 1 for i in info) and len(made) == 2
    assert (o == 0).all()                             # a fresh episode of the relaunched game
    o, s, r, d, info, a = g.step([0, 1, 2])
    assert not d.any() and info[0]["restarts"] == 1


def test_sc2_restart_keeps_episode_counters():
    """a restart must not reset battles_won / battles_game / timeouts (the reference keeps its env object,
    StarCraft2_Env.py:468-472), and the error step's info carries the reference's keys (:517-524)."""
    from mat_dcml_amd.envs.smac.adapter import SC2Game
    made = []

    def make_env():
        e = _FlakySC2(fail_on=(2,) if not made else ())
        e.battles_won, e.battles_game, e.timeouts, e.win_counted = 0, 0, 0, False
        made.append(e)
        return e
    g = SC2Game(make_env, errors=(ConnectionError,))
    g.reset()
    made[0].battles_won, made[0].battles_game, made[0].timeouts = 3, 5, 1
    g.step([0, 1, 2])
    o, s, r, d, info, a = g.step([0, 1, 2])          # protocol error -> restart
    assert d.all() and len(made) == 2
    for i in info:
        assert (i["battles_won"], i["battles_game"], i["battles_draw"], i["restarts"]) == (3, 5, 1, 1)
        assert i["bad_transition"] is False and i["won"] is False
    assert (g.env.battles_won, g.env.battles_game, g.env.timeouts) == (3, 5, 1)

    class InPlace(_FlakySC2):   # smac's env: relaunches its own process, same object
        def full_restart(self):
            self.relaunched = True
            self.fail_on = ()
    e = InPlace(fail_on=(1,))
    e.battles_won, e.battles_game, e.timeouts, e.win_counted = 7, 9, 2, False
    g = SC2Game(lambda: e, errors=(ConnectionError,))
    g.reset()
    o, s, r, d, info, a = g.step([0, 1, 2])
    assert g.env is e and e.relaunched and info[0]["battles_won"] == 7 and info[0]["restarts"] == 1


def test_sc2_rebuild_reports_live_win_counted():
    """on the rebuild path the error step's ``won`` is the value the LIVE env object had when the error
    hit (StarCraft2_Env.py:517-524 reads it from the env that is still there), not the fresh object's False."""
    from mat_dcml_amd.envs.smac.adapter import SC2Game
    made = []

    def make_env():
        e = _FlakySC2(fail_on=(2,) if not made else ())
        e.battles_won, e.battles_game, e.timeouts, e.win_counted = 0, 0, 0, False
        made.append(e)
        return e
    g = SC2Game(make_env, errors=(ConnectionError,))
    g.reset()
    g.step([0, 1, 2])
    made[0].win_counted = True                        # the battle was already won when the protocol error hit
    o, s, r, d, info, a = g.step([0, 1, 2])
    assert len(made) == 2 and made[1].win_counted is False
    assert all(i["won"] is True for i in info)
