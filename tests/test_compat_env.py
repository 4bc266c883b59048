"""Reference-API ``Env`` (DCML_BID_FIRST_MA_ENV_SingleProcess.Env surface) on top of the device env."""
import numpy as np

from DCML_BID_FIRST_MA_ENV_SingleProcess import Env


def test_multi_agent_api():
    env = Env(n_workers=8, seed=3)
    obs, share, ava = env.reset()
    assert obs.shape == (9, 7) and share.shape == (9, 10) and ava.shape == (9, 2)
    assert env.n_agents == 9 and env.observation_space == [[7]] * 9 and env.share_observation_space == [[10]]
    assert env.action_space[0].semi_index == -1
    act = np.ones((9, 1))
    act[-1] = 0.5
    ob, s_ob, rew, dones, info, ava = env.step(act)
    assert rew.shape == (9, 1) and dones.shape == (9,) and set(info[0]) == {"delay", "payment"}
    assert np.allclose(rew, -(99 * info[0]["delay"] + info[0]["payment"]), rtol=1e-5)
    # standalone flag == all-zero selection (the N == 0 branch, 1.5x penalty)
    _, _, r2, _, i2, _ = env.step(act, standalone=True)
    assert np.allclose(r2, 1.5 * -(99 * i2[0]["delay"] + i2[0]["payment"]), rtol=1e-4)


def test_modes_and_arrive_time():
    env = Env(n_workers=8, seed=3, multi_agent=False)
    obs, share, ava = env.reset(arrive_time=4)
    assert obs.shape == (63,) and share.shape == (10,) and env.arrive_time == 4
    _, _, rew, dones, _, _ = env.step(np.ones(9))
    assert rew.shape == (1,) and dones.shape == (1,)
    dec = Env(n_workers=8, central_execution=False)
    assert len(dec.action_space) == 9 and dec.action_space[-1].continuous
    b = Env(n_workers=8, seed=1)
    o, s, _ = b.reset(binary=True)
    assert s.shape == (9, 64 + 8) and set(np.unique(s[0, :64])) <= {0.0, 1.0}
    sh = Env(n_workers=8, seed=1)
    o, s, _ = sh.reset(shannon_enable=True)
    assert s.shape == (9, 2 + 16)


def test_fixed_and_preset(tmp_path):
    env = Env(n_workers=100, fixed=True, preset=True, seed=1)
    env.modify_preset(disable_rate=40)
    env.reset()
    assert env.disable_rate == 40 and env.eval_episode_i == 1
    _, _, _, _, info, ava = env.step(np.zeros((101, 1)))
    assert int(ava[:100, 1].sum()) == 60 and info[0]["delay"] > 0
    m, w = env.generate_preset_data(5, dir_name=str(tmp_path) + "/S_", seed=0)
    with open(m, "rb") as f:
        assert np.load(f).shape == (5, 3)
    with open(w, "rb") as f:
        assert np.load(f).shape == (5, 100) and np.load(f).shape == (5,)
    st = env.fake_reset(2 ** 19, 2 ** 9, 0.1, 3, binary=False)
    assert st.shape == (3 + 100,)
