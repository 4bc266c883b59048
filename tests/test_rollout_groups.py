"""Pipelined rollout (``--rollout_groups G``, runner/dcml_runner._rollout_groups): the env groups run on their own
streams, but the rollout must be the 1-group rollout — the same env trajectories, observations, rewards, masks and
episode statistics bit for bit, the same policy outputs up to float rounding — because the sampling noise is keyed
by (step counter, global env id) and the env groups are views of the one env (SURVEY §2.4 overlap plan; §7.4 #8).
(Policy outputs: GEMM blocking on the CPU and the 32-row attention chunking of the fused encoder depend on a
sequence's position in the batch, ~1 ulp.)"""
import time

import pytest
import torch


def _runner(G, n_workers, envs, T, device, seed=3):
    from mat_dcml_amd.config import get_config, parse_args
    from mat_dcml_amd.runner.dcml_runner import DCMLRunner
    args = parse_args(["--env_name", "DCML", "--n_workers", str(n_workers), "--n_rollout_threads", str(envs),
                       "--episode_length", str(T), "--seed", str(seed), "--rollout_groups", str(G), "--use_valuenorm"],
                      get_config(), warn=False)
    r = DCMLRunner({"all_args": args, "device": device, "run_dir": None})
    r.warmup()
    return r


def _state(r):
    b = r.buffer
    out = {k: getattr(b, k).clone() for k in ("obs", "share_obs", "available_actions", "actions", "action_log_probs",
                                               "value_preds", "rewards", "masks")}
    for k in ("counter", "task_ctr", "R", "C", "worker_pr", "obs"):
        out["env_" + k] = getattr(r.envs, k).clone()
    out["ep_reward"] = r._ep_reward.clone()
    return out, r._done_stats.clone()


def _update_weights(r, it):
    """An optimizer-step stand-in that changes every weight identically in both runners (a real train() reduces
    gradients with fp32 atomics, so the two runners' weights would differ by rounding) and bumps the pack version:
    the next rollout must see every weight pack rebuilt (the groups' streams raced the lazy rebuild)."""
    from mat_dcml_amd.ops import mat_fused
    m = r.policy.transformer
    g = torch.Generator().manual_seed(100 + it)
    with torch.no_grad():
        for p_ in m.parameters():
            p_.add_(0.05 * torch.randn(p_.shape, generator=g).to(p_.device))
    mat_fused.bump_version(m)


def _compare(G, n_workers, envs, T, device, iters=1, update=False):
    ref, grp = _runner(1, n_workers, envs, T, device), _runner(G, n_workers, envs, T, device)
    assert grp._groups() == G
    for it in range(iters):
        ref.rollout()
        grp.rollout()
        ref.buffer.after_update()
        grp.buffer.after_update()
        if update:
            _update_weights(ref, it)
            _update_weights(grp, it)
    if device.type == "cuda":
        torch.cuda.synchronize()
    (a, sa), (b, sb) = _state(ref), _state(grp)
    for k in a:
        if k in ("actions", "action_log_probs", "value_preds"):
            assert torch.allclose(a[k], b[k], rtol=1e-5, atol=1e-5), (k, (a[k] - b[k]).abs().max())
        else:
            assert torch.equal(a[k], b[k]), k
    assert torch.allclose(sa, sb, rtol=1e-12, atol=0), (sa, sb)   # fp64 sums in group order
    return ref, grp


def test_group_views_step_like_the_whole_env():
    from mat_dcml_amd.envs.dcml.config import DCMLConfig
    from mat_dcml_amd.envs.dcml.vec_env import DeviceDCMLEnv
    cfg = DCMLConfig(n_workers=8)
    whole, split = DeviceDCMLEnv(6, cfg, seed=5), DeviceDCMLEnv(6, cfg, seed=5)
    whole.reset()
    split.reset()
    views = split.group_views(3)
    g = torch.Generator().manual_seed(0)
    for _ in range(4):
        act = torch.rand(6, cfg.n_agents, generator=g)
        o1, s1, r1, d1, dl1, p1, a1 = whole.step(act)
        outs = [v.step(act[2 * i:2 * i + 2]) for i, v in enumerate(views)]
        assert torch.equal(r1, torch.cat([o[2] for o in outs])) and torch.equal(dl1, torch.cat([o[4] for o in outs]))
        assert torch.equal(split.obs, whole.obs) and torch.equal(split.share, whole.share)
        assert torch.equal(split.task_ctr, whole.task_ctr)


def test_grouped_rollout_equals_single_group_cpu():
    _compare(2, 4, 4, 5, torch.device("cpu"), iters=2, update=True)


@pytest.mark.gpu
def test_grouped_rollout_equals_single_group_gpu(gpu):
    """HIP env views + fused insert per group on two streams, fused encoder / decode kernels."""
    ref, grp = _compare(2, 32, 64, 6, torch.device("cuda"), iters=3, update=True)
    from mat_dcml_amd.ops import kernels
    assert grp.envs._kern is not None and kernels.available()
    for r in (ref, grp):   # timing report (not asserted: the overlap gain is measured by bench.py)
        torch.cuda.synchronize()
        t = time.perf_counter()
        r.rollout()
        torch.cuda.synchronize()
        print(f"rollout_groups={r._groups()}: {1e3 * (time.perf_counter() - t):.2f} ms")
