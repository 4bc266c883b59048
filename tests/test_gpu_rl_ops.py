"""HIP RL kernels vs the PyTorch fp32 reference ops."""
import pytest
import torch

from mat_dcml_amd.algos.valuenorm import ValueNorm
from mat_dcml_amd.ops import kernels, rl_ops

pytestmark = pytest.mark.gpu


def test_gae_matches_torch(gpu):
    T, E, A = 50, 64, 33
    g = torch.Generator(device=gpu).manual_seed(0)
    rew = torch.randn(T, E, A, 1, device=gpu, generator=g) * 10
    vp = torch.randn(T + 1, E, A, 1, device=gpu, generator=g)
    masks = (torch.rand(T + 1, E, A, 1, device=gpu, generator=g) > 0.2).float()
    vn = ValueNorm(1, device=gpu)
    vn.update(torch.randn(1000, 1, device=gpu) * 30 + 5)
    adv1, ret1 = torch.zeros(T, E, A, 1, device=gpu), torch.zeros(T + 1, E, A, 1, device=gpu)
    adv2, ret2 = adv1.clone(), ret1.clone()
    rl_ops.gae_torch(rew, vp, masks, 0.99, 0.95, vn, adv1, ret1)
    rl_ops.gae(rew, vp, masks, 0.99, 0.95, vn, adv2, ret2)
    assert torch.allclose(adv1, adv2, atol=1e-3, rtol=1e-4)
    assert torch.allclose(ret1[:T], ret2[:T], atol=1e-3, rtol=1e-4)


def test_gae_multi_objective_matches_torch(gpu):
    """momat / dmomat buffers: two objectives with their own ValueNorm statistics, one mask per agent."""
    T, E, A, K = 50, 32, 33, 2
    g = torch.Generator(device=gpu).manual_seed(1)
    rew = torch.randn(T, E, A, K, device=gpu, generator=g) * 10
    vp = torch.randn(T + 1, E, A, K, device=gpu, generator=g)
    masks = (torch.rand(T + 1, E, A, 1, device=gpu, generator=g) > 0.2).float()
    vn = ValueNorm(K, device=gpu)
    vn.update(torch.randn(1000, K, device=gpu) * torch.tensor([30.0, 3.0], device=gpu) + torch.tensor([5.0, -2.0], device=gpu))
    adv1, ret1 = torch.zeros(T, E, A, K, device=gpu), torch.zeros(T + 1, E, A, K, device=gpu)
    adv2, ret2 = adv1.clone(), ret1.clone()
    rl_ops.gae_torch(rew, vp, masks, 0.99, 0.95, vn, adv1, ret1)
    rl_ops.gae(rew, vp, masks, 0.99, 0.95, vn, adv2, ret2)
    assert torch.allclose(adv1, adv2, atol=1e-3, rtol=1e-4)
    assert torch.allclose(ret1[:T], ret2[:T], atol=1e-3, rtol=1e-4)


@pytest.mark.parametrize("K,nvn", [(1, 1), (2, 2), (2, 1), (1, 0)])
def test_gae_vn_kernel_matches_torch(gpu, K, nvn):
    """kernels.gae_reverse_scan_vn (buffer.compute_returns): ValueNorm statistics derived in-kernel from the running
    moments and V(T) from next_value, vs the torch statistics + scan; nvn 0 = no value normaliser."""
    T, E, A = 50, 32, 33
    g = torch.Generator(device=gpu).manual_seed(3 + K + nvn)
    rew = torch.randn(T, E, A, K, device=gpu, generator=g) * 10
    vp = torch.randn(T + 1, E, A, K, device=gpu, generator=g)
    nv = torch.randn(E, A, K, device=gpu, generator=g)
    masks = (torch.rand(T + 1, E, A, 1, device=gpu, generator=g) > 0.2).float()
    vn = None
    if nvn:
        vn = ValueNorm(nvn, device=gpu)
        vn.update(torch.randn(1000, nvn, device=gpu, generator=g) * 20 + 3)
    vp_ref = vp.clone()
    vp_ref[-1].copy_(nv)
    adv1, ret1 = torch.zeros(T, E, A, K, device=gpu), torch.zeros(T + 1, E, A, K, device=gpu)
    adv2, ret2 = adv1.clone(), ret1.clone()
    rl_ops.gae_torch(rew, vp_ref, masks, 0.99, 0.95, vn, adv1, ret1)
    kernels.gae_reverse_scan_vn(rew, vp, masks, nv.reshape(-1).contiguous(), vn, 0.99, 0.95, adv2, ret2)
    assert torch.equal(vp[-1], nv)
    assert torch.allclose(adv1, adv2, atol=1e-3, rtol=1e-4)
    assert torch.allclose(ret1[:T], ret2[:T], atol=1e-3, rtol=1e-4)


def test_train_iteration_on_gpu(gpu):
    from mat_dcml_amd.config import get_config, parse_args
    from mat_dcml_amd.runner.dcml_runner import DCMLRunner
    args = parse_args(["--env_name", "DCML", "--n_workers", "8", "--n_rollout_threads", "16", "--episode_length", "5",
                       "--ppo_epoch", "2", "--num_mini_batch", "2", "--use_valuenorm"], get_config(), warn=False)
    r = DCMLRunner({"all_args": args, "device": gpu, "run_dir": None})
    r.warmup()
    infos = r.train_iteration()
    torch.cuda.synchronize()
    assert all(torch.isfinite(torch.as_tensor(float(v))) for v in infos.values())


def test_splitk_linear_grad(gpu):
    from mat_dcml_amd.ops.linear import linear
    x = torch.randn(40000, 64, device=gpu, requires_grad=True)
    w = torch.randn(64, 64, device=gpu, requires_grad=True)
    b = torch.randn(64, device=gpu, requires_grad=True)
    y = linear(x, w, b)
    g = torch.randn_like(y)
    y.backward(g)
    x2, w2, b2 = x.detach().clone().requires_grad_(), w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    torch.nn.functional.linear(x2, w2, b2).backward(g)
    assert torch.allclose(x.grad, x2.grad, rtol=1e-3, atol=1e-2)
    assert torch.allclose(w.grad, w2.grad, rtol=1e-3, atol=1e-1)
    assert torch.allclose(b.grad, b2.grad, rtol=1e-3, atol=1e-2)


def test_mat_learns_on_dcml(gpu):
    """Integration: a short fused-kernel training run on the 32-worker env improves the mean episode reward
    (random-init MAT picks ~half the workers with ratio ~0 -> K = 1, the slowest possible plan)."""
    from mat_dcml_amd.config import get_config, parse_args
    from mat_dcml_amd.parallel.comm import Comm
    from mat_dcml_amd.runner.dcml_runner import DCMLRunner
    args = parse_args(["--n_workers", "32", "--n_rollout_threads", "128", "--episode_length", "25", "--lr", "5e-4",
                       "--ppo_epoch", "5", "--num_mini_batch", "2", "--use_valuenorm", "--entropy_coef", "0.01"],
                      get_config(), warn=False)
    r = DCMLRunner({"all_args": args, "device": gpu, "run_dir": None, "comm": Comm(device=gpu)})
    r.warmup()
    curve = []
    for it in range(30):
        r.train_iteration()
        curve.append(float(r.buffer.rewards.mean()))
    first, last = sum(curve[:5]) / 5, sum(curve[-5:]) / 5
    print(f"mean step reward: first 5 iters {first:.1f} -> last 5 iters {last:.1f}")
    assert last > first + 0.1 * abs(first), (first, last)


def test_masked_sums_and_gather_match_torch(gpu):
    """minibatch gather (+ on-the-fly advantage standardisation) and the masked fp64 statistics vs torch"""
    from mat_dcml_amd.ops import kernels, rl_ops
    g = torch.Generator(device=gpu).manual_seed(0)
    T, E, A = 50, 64, 33
    adv = torch.randn(T, E, A, 1, device=gpu, generator=g) * 3 + 1
    active = (torch.rand(T, E, A, 1, device=gpu, generator=g) < 0.8).float()
    sums = kernels.masked_sums(adv, active)
    ref = rl_ops.masked_sums(adv, active)
    torch.testing.assert_close(sums, ref, rtol=1e-12, atol=1e-9)
    assert torch.equal(sums, kernels.masked_sums(adv, active))          # fixed-order: bitwise repeatable
    # 2-objective advantages share one active mask per (t, e, agent)
    adv2 = torch.randn(T, E, A, 2, device=gpu, generator=g)
    torch.testing.assert_close(kernels.masked_sums(adv2, active), rl_ops.masked_sums(adv2, active), rtol=1e-12,
                               atol=1e-9)
    obs = torch.randn(T * E, A, 7, device=gpu, generator=g)
    act = torch.randn(T * E, A, 1, device=gpu, generator=g)
    adv_f = adv.reshape(T * E, A, 1)
    idx = torch.randperm(T * E, device=gpu, generator=g)[:800]
    wide = torch.randn(T * E, A, 12, device=gpu, generator=g)   # row width % 4 == 0: the float4 path
    out = kernels.gather_rows({"obs": obs, "actions": act, "adv": adv_f, "wide": wide}, idx, sums, ("adv",))
    assert torch.equal(out["obs"], obs[idx]) and torch.equal(out["actions"], act[idx])
    assert torch.equal(out["wide"], wide[idx])
    norm = rl_ops.normalize_from_sums(adv, ref).reshape(T * E, A, 1)[idx]
    torch.testing.assert_close(out["adv"], norm, rtol=1e-6, atol=1e-6)


def test_mb_stats_matches_torch(gpu):
    """Per-minibatch return moments of one epoch (DP statistics precompute) vs torch on the gathered rows."""
    g = torch.Generator(device=gpu).manual_seed(5)
    N, A, K = 400, 33, 2
    ret = torch.randn(N, A, K, device=gpu, generator=g) * 7
    act = (torch.rand(N, A, 1, device=gpu, generator=g) > 0.1).float()
    perm = torch.randperm(N, device=gpu, generator=g)
    out = kernels.mb_stats(ret, act, perm, 4)
    for m, idx in enumerate(perm.view(4, -1)):
        r = ret[idx].double().reshape(-1, K)
        ref = torch.cat([r.sum(0), (r * r).sum(0), torch.tensor([float(r.shape[0])], device=gpu, dtype=torch.float64),
                         act[idx].double().sum().reshape(1)])
        assert torch.allclose(out[m], ref, rtol=1e-10, atol=1e-8), (m, out[m], ref)


@pytest.mark.parametrize("n_obj", [1, 2])
def test_rollout_insert_matches_torch(gpu, n_obj):
    """the one-launch rollout bookkeeping (kernels.rollout_insert) == DCMLRunner._track + insert (torch path):
    buffer slots, agent-expanded rewards / masks, episode sums and the finished-episode statistics"""
    from mat_dcml_amd.config import get_config, parse_args
    from mat_dcml_amd.runner.dcml_runner import DCMLRunner
    argv = ["--n_workers", "8", "--n_rollout_threads", "40", "--episode_length", "6"]
    if n_obj == 2:
        argv += ["--n_objective", "2"]
    args = parse_args(argv, get_config(), warn=False)
    runs = []
    for fused in (False, True):
        torch.manual_seed(3)
        r = DCMLRunner({"all_args": args, "device": gpu, "run_dir": None})
        assert r.buffer.n_objective == n_obj
        if not fused:
            r._ins_ok = False
        r.warmup()
        r.rollout()
        torch.cuda.synchronize()
        runs.append(r)
    a, b = runs
    assert b._ins_ok
    for name in ("obs", "share_obs", "available_actions", "actions", "action_log_probs", "value_preds", "rewards",
                 "masks"):
        torch.testing.assert_close(getattr(a.buffer, name), getattr(b.buffer, name), rtol=0, atol=0, msg=name)
    assert a.buffer.step == b.buffer.step
    for name in ("_ep_reward", "_ep_delay", "_ep_pay"):
        torch.testing.assert_close(getattr(a, name), getattr(b, name), rtol=1e-6, atol=1e-4, msg=name)
    torch.testing.assert_close(a._done_stats, b._done_stats, rtol=1e-9, atol=1e-6)


@pytest.mark.gpu
def test_feistel_randperm_is_a_permutation(gpu):
    """One-launch minibatch shuffle (csrc/rl_ops.hip randperm_kernel): a bijection of [0, n) for every n, different
    per key, reproducible under torch.manual_seed, and not close to the identity."""
    from mat_dcml_amd.ops import kernels
    dev = torch.device("cuda")
    for n in (1, 2, 7, 100, 3200, 12800, 40000):
        p = kernels.randperm(n, dev).cpu()
        assert torch.equal(torch.sort(p).values, torch.arange(n)), n
    torch.manual_seed(3)
    a = kernels.randperm(12800, dev)
    torch.manual_seed(3)
    b = kernels.randperm(12800, dev)
    c = kernels.randperm(12800, dev)
    assert torch.equal(a, b) and not torch.equal(a, c)
    fixed = (a.cpu() == torch.arange(12800)).float().mean().item()
    assert fixed < 0.01
    # the first minibatch's rows spread evenly over the buffer (the T·E rows are time-major)
    first = a[:3200].cpu().float()
    assert abs(first.mean().item() / 12800 - 0.5) < 0.03
    from mat_dcml_amd.utils.philox import feistel_randperm
    for n, key in ((12800, (12345, 678)), (3200, (1, 2)), (777, (2 ** 31 - 2, 99))):
        assert torch.equal(kernels.randperm(n, dev, key=key).cpu(), feistel_randperm(n, *key)), n
