"""HIP DCML env kernels vs the torch implementation (same Philox draws)."""
import pytest
import torch

from mat_dcml_amd.envs.dcml.config import DCMLConfig
from mat_dcml_amd.envs.dcml.vec_env import DeviceDCMLEnv

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("W,fixed,preset,shannon", [(32, False, False, False), (100, False, False, False),
                                                    (100, True, False, False), (100, False, True, False),
                                                    (4, False, False, False), (128, False, False, False),
                                                    (32, False, False, True)])
def test_env_kernel_matches_torch(gpu, W, fixed, preset, shannon):
    """Same Philox draws on both paths, so every INTEGER quantity must match exactly — per worker the transmission
    count n (download + upload retries, DCML_Worker_TIMESLOT_MultiProcess.py:53-106) and the consumed timeslots,
    per env N, K and the standalone flag (DCML_BID_FIRST_MA_ENV_SingleProcess.py:64-105) — and the double-precision
    delays / payment / reward to 1e-6 relative.  The one legitimate exception: an env with a geometric draw whose
    log U / log Pr lies within 1e-6 of an integer (the floor may flip between libm and the device log); those envs
    are flagged from the same draws and excluded.  The standalone (N = 0) and both K-clamp branches are asserted
    on their own subsets."""
    cfg = DCMLConfig(n_workers=W, shannon=shannon)
    E = 64
    hip = DeviceDCMLEnv(E, cfg, device=gpu, seed=7, fixed=fixed, preset=preset, backend="hip")
    ref = DeviceDCMLEnv(E, cfg, device=gpu, seed=7, fixed=fixed, preset=preset, backend="torch")
    assert hip._kern is not None and ref._kern is None
    hip.record_debug = ref.record_debug = True
    o1 = hip.reset()
    o2 = ref.reset()
    for a, b in zip(o1, o2):
        assert torch.allclose(a, b, atol=1e-6, rtol=1e-6), (a - b).abs().max()
    g = torch.Generator(device=gpu).manual_seed(0)
    n_exempt = n_checked = 0
    branch = {"standalone": 0, "k_clamp_high": 0, "k_clamp_low": 0}
    for step in range(8):
        act = (torch.rand(E, W + 1, device=gpu, generator=g) < 0.4).float()
        act[:, -1] = torch.rand(E, device=gpu, generator=g) * 1.2
        act[: E // 8, :W] = 0                      # N == 0: the standalone branch
        act[E // 8: E // 4, -1] = 1.5              # K = ceil(N * 1.5) > N: clamped to N
        act[E // 4: 3 * E // 8, -1] = 0.0          # K = 0: clamped to 1
        r1 = hip.step(act)
        r2 = ref.step(act)
        obs1, _, rew1, done1, d1, p1, ava1 = r1
        obs2, _, rew2, done2, d2, p2, ava2 = r2
        assert torch.equal(done1, done2)
        assert torch.allclose(obs1, obs2, atol=1e-6)
        assert torch.equal(ava1, ava2)
        k1, k2 = hip.last_debug, ref.last_debug
        ok = ~ref.last_near_int
        n_exempt += int((~ok).sum())
        n_checked += int(ok.sum())
        a, b = k1[ok], k2[ok]
        assert torch.equal(a[:, :3], b[:, :3]), "N / K / standalone"
        assert torch.equal(a[:, 6:6 + W], b[:, 6:6 + W]), "transmission counts n"
        assert torch.equal(a[:, 6 + W:6 + 2 * W], b[:, 6 + W:6 + 2 * W]), "consumed timeslots"
        # delay, payment, reward and the per-worker delays (double on both paths; measured agreement ~1e-7 relative)
        torch.testing.assert_close(a[:, 3:6], b[:, 3:6], rtol=1e-6, atol=1e-9)
        torch.testing.assert_close(a[:, 6 + 2 * W:], b[:, 6 + 2 * W:], rtol=1e-6, atol=1e-9)
        torch.testing.assert_close(rew1[ok], rew2[ok], rtol=1e-6, atol=0.0)
        torch.testing.assert_close(d1[ok], d2[ok], rtol=1e-6, atol=0.0)
        torch.testing.assert_close(p1[ok], p2[ok], rtol=1e-6, atol=0.0)
        if not fixed:   # the branches, each on its own subset
            sa = ok & (b[:, 2] == 1)
            raw_k = torch.ceil(act[:, :W].double().sum(1) * act[:, W].double())
            hi = ok & ~(b[:, 2] == 1) & (raw_k > b[:, 0])
            lo = ok & ~(b[:, 2] == 1) & (raw_k < 1)
            for name, m in (("standalone", sa), ("k_clamp_high", hi), ("k_clamp_low", lo)):
                branch[name] += int(m.sum())
                assert torch.equal(k1[m][:, :3], k2[m][:, :3]) and torch.allclose(k1[m], k2[m], rtol=1e-6, atol=1e-9), name
            assert (k2[sa, 1] == 1).all() and (k2[hi, 1] == k2[hi, 0]).all() and (k2[lo, 1] == 1).all()
            # standalone: reward = 1.5x penalty of worker 0's solo task (ENV_SingleProcess.py:81-92)
            assert torch.equal(k2[sa, 3], k2[sa, 6 + 2 * W])
    assert n_exempt <= 0.01 * (n_exempt + n_checked), (n_exempt, n_checked)
    if not fixed:
        assert min(branch.values()) > 0, branch


def test_env_kernel_throughput(gpu):
    cfg = DCMLConfig(n_workers=32)
    env = DeviceDCMLEnv(2048, cfg, device=gpu, seed=1, backend="hip")
    env.reset()
    act = torch.ones(2048, 33, device=gpu)
    act[:, -1] = 0.7
    for _ in range(3):
        env.step(act)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        env.step(act)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 20
    print(f"dcml_env_step 2048 envs x 32 workers: {ms * 1e3:.1f} us")
    assert ms < 5.0
