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
    cfg = DCMLConfig(n_workers=W, shannon=shannon)
    E = 64
    hip = DeviceDCMLEnv(E, cfg, device=gpu, seed=7, fixed=fixed, preset=preset, backend="hip")
    ref = DeviceDCMLEnv(E, cfg, device=gpu, seed=7, fixed=fixed, preset=preset, backend="torch")
    assert hip._kern is not None and ref._kern is None
    o1 = hip.reset()
    o2 = ref.reset()
    for a, b in zip(o1, o2):
        assert torch.allclose(a, b, atol=1e-6, rtol=1e-6), (a - b).abs().max()
    g = torch.Generator(device=gpu).manual_seed(0)
    bad = 0
    for step in range(6):
        act = (torch.rand(E, W + 1, device=gpu, generator=g) < 0.4).float()
        act[:, -1] = torch.rand(E, device=gpu, generator=g) * 1.2
        act[: E // 8, :W] = 0  # exercise the standalone branch
        r1 = hip.step(act)
        r2 = ref.step(act)
        obs1, _, rew1, done1, d1, p1, ava1 = r1
        obs2, _, rew2, done2, d2, p2, ava2 = r2
        assert torch.equal(done1, done2)
        assert torch.allclose(obs1, obs2, atol=1e-6)
        assert torch.equal(ava1, ava2)
        close = torch.isclose(rew1, rew2, rtol=1e-4, atol=1e-3) & torch.isclose(d1, d2, rtol=1e-4, atol=1e-4)
        bad += int((~close).sum())
    assert bad <= 0.02 * E * 6, bad


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
