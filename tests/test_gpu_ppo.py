"""Fused PPO loss / flat Adam kernels vs PyTorch fp32 references (same inputs)."""
import types

import pytest
import torch

from mat_dcml_amd.algos.valuenorm import ValueNorm

pytestmark = pytest.mark.gpu


def _args(**kw):
    d = dict(clip_param=0.2, value_loss_coef=1.0, entropy_coef=0.01, huber_delta=10.0, _use_huber_loss=True,
             _use_clipped_value_loss=True, _use_value_active_masks=True, _use_policy_active_masks=True)
    d.update(kw)
    return types.SimpleNamespace(**d)


def _torch_loss(tr, v, lp, ent, mb, vn):
    imp = torch.exp(lp - mb["old_logp"])
    s1, s2 = imp * mb["adv"], imp.clamp(1 - tr.clip_param, 1 + tr.clip_param) * mb["adv"]
    act = mb["active"]
    pl = -(torch.min(s1, s2) * act).sum() / act.sum() if tr._use_policy_active_masks else -torch.min(s1, s2).mean()
    e = (ent * act).sum() / act.sum() if tr._use_policy_active_masks else ent.mean()
    vc = mb["value_preds"] + (v - mb["value_preds"]).clamp(-tr.clip_param, tr.clip_param)
    vn.update(mb["returns"])
    tgt = vn.normalize(mb["returns"])

    def h(x):
        return torch.where(x.abs() <= tr.huber_delta, 0.5 * x * x, tr.huber_delta * (x.abs() - 0.5 * tr.huber_delta)) \
            if tr._use_huber_loss else 0.5 * x * x
    vl = torch.max(h(tgt - v), h(tgt - vc)) if tr._use_clipped_value_loss else h(tgt - v)
    vl = (vl * act).sum() / act.sum() if tr._use_value_active_masks else vl.mean()
    return pl - e * tr.entropy_coef + vl * tr.value_loss_coef, pl, vl, e, imp.mean()


@pytest.mark.parametrize("flags", [{}, {"_use_huber_loss": False, "_use_policy_active_masks": False},
                                   {"_use_clipped_value_loss": False, "_use_value_active_masks": False}])
def test_ppo_loss_grads_match_autograd(gpu, flags):
    from mat_dcml_amd.ops.ppo_fused import PPOLossFused
    g = torch.Generator(device=gpu).manual_seed(0)
    N = 5000
    r = lambda *s: torch.randn(*s, device=gpu, generator=g)  # noqa: E731
    v, lp, ent = r(N, 1), r(N, 1) * 0.3 - 0.7, r(N, 1).abs()
    mb = {"old_logp": lp + 0.3 * r(N, 1), "adv": r(N, 1), "value_preds": v + 0.3 * r(N, 1), "returns": 3 * r(N, 1) + 1,
          "active": (torch.rand(N, 1, device=gpu, generator=g) > 0.2).float()}
    tr = _args(**flags)
    tr.value_normalizer = ValueNorm(1, device=gpu)
    vn_ref = ValueNorm(1, device=gpu)
    for _ in range(2):   # second call exercises non-trivial running statistics
        fused = PPOLossFused(tr, gpu) if _ == 0 else fused
        fused.out.zero_()
        dv, dlp, dent = fused.run(v, lp, ent, mb)
        vv, ll, ee = v.clone().requires_grad_(), lp.clone().requires_grad_(), ent.clone().requires_grad_()
        loss, pl, vl, e, ratio = _torch_loss(tr, vv, ll, ee, mb, vn_ref)
        loss.backward()
        torch.cuda.synchronize()
        assert torch.allclose(dlp, ll.grad, atol=1e-7, rtol=1e-4), (dlp - ll.grad).abs().max()
        assert torch.allclose(dent, ee.grad, atol=1e-9, rtol=1e-4)
        assert torch.allclose(dv, vv.grad, atol=1e-7, rtol=1e-4), (dv - vv.grad).abs().max()
        o = fused.out
        assert torch.allclose(o, torch.stack([pl, vl, e, ratio]).detach(), rtol=1e-4, atol=1e-5), (o, pl, vl, e, ratio)
        assert torch.allclose(tr.value_normalizer.running_mean, vn_ref.running_mean, rtol=1e-5)
        assert torch.allclose(tr.value_normalizer.debiasing_term, vn_ref.debiasing_term, rtol=1e-6)


def test_flat_adam_matches_torch_adam_with_clipping(gpu):
    from mat_dcml_amd.ops.ppo_fused import FlatAdam
    g = torch.Generator(device=gpu).manual_seed(1)
    n = 151469
    p0 = torch.randn(n, device=gpu, generator=g)
    p_ref = torch.nn.Parameter(p0.clone())
    opt = torch.optim.Adam([p_ref], lr=5e-4, eps=1e-5)
    flat_p, flat_g = p0.clone(), torch.zeros(n, device=gpu)
    fa = FlatAdam(flat_p, flat_g, lr=5e-4, eps=1e-5, max_grad_norm=10.0)
    for it in range(5):
        grad = torch.randn(n, device=gpu, generator=g) * (0.01 if it % 2 else 1.0)
        p_ref.grad = grad.clone()
        norm = torch.nn.utils.clip_grad_norm_([p_ref], 10.0)
        opt.step()
        flat_g.copy_(grad)
        fa.step()
        torch.cuda.synchronize()
        assert torch.allclose(fa.grad_norm, norm, rtol=1e-4)
        assert torch.allclose(flat_p, p_ref.detach(), atol=1e-6, rtol=1e-5), (flat_p - p_ref).abs().max()


def test_workspace_reduction_with_norm_partials_matches_adam_norm(gpu):
    """The single-GPU update path: mdl_grad_reduce_norm folds the 32 gradient-workspace copies into the flat buffer
    AND leaves the optimizer's Σ g² partials, so FlatAdam.step(norm_ready=True) skips its norm launch; same grad
    norm (to fp32 summation order) and the same parameters as the unfused reduction + step."""
    from types import SimpleNamespace

    from mat_dcml_amd.ops import mat_train
    from mat_dcml_amd.ops.ppo_fused import FlatAdam
    g = torch.Generator(device=gpu).manual_seed(2)
    n, copies = 151469, 32
    p0 = torch.randn(n, device=gpu, generator=g)
    res = []
    for fused in (False, True):
        flat_p, flat_g = p0.clone(), torch.zeros(n, device=gpu)
        fa = FlatAdam(flat_p, flat_g, lr=5e-4, eps=1e-5, max_grad_norm=1.0)
        m = SimpleNamespace()
        ws = mat_train.attach_grad_workspace(m, flat_g, copies=copies)
        stride = ws.numel() // copies
        gg = torch.Generator(device=gpu).manual_seed(3)
        for it in range(3):
            for k in range(copies):
                ws[k * stride:k * stride + n].copy_(torch.randn(n, device=gpu, generator=gg) * 0.1)
            flat_g.zero_()
            ready = mat_train.reduce_grad_workspace(m, norm_into=fa.scratch if fused else None)
            assert ready == fused
            assert float(ws.abs().max()) == 0.0   # the copies are zeroed for the next minibatch
            fa.step(norm_ready=ready)
        torch.cuda.synchronize()
        res.append((flat_p.clone(), float(fa.grad_norm), flat_g.clone()))
    assert torch.equal(res[0][2], res[1][2])   # the same folded gradient
    assert abs(res[0][1] - res[1][1]) <= 1e-5 * res[0][1], (res[0][1], res[1][1])
    assert torch.allclose(res[0][0], res[1][0], atol=1e-6, rtol=1e-6), (res[0][0] - res[1][0]).abs().max()


@pytest.mark.parametrize("n_obj", [1, 2])
def test_fused_trainer_step_matches_autograd_step(gpu, n_obj):
    """One PPO minibatch: fused loss + FlatAdam vs autograd loss + torch Adam (same fused fwd/bwd kernels); n_obj = 2
    is the multi-objective MAT (vector value head, per-objective ValueNorm and advantages)."""
    from mat_dcml_amd.algos.mat_trainer import MATTrainer
    from mat_dcml_amd.algos.policy import TransformerPolicy
    from mat_dcml_amd.config import get_config, parse_args
    from mat_dcml_amd.envs.dcml.spaces import dcml_action_spaces
    from mat_dcml_amd.parallel.comm import Comm
    args = parse_args(["--n_workers", "8", "--lr", "5e-4", "--use_valuenorm", "--use_value_active_masks",
                       "--n_objective", str(n_obj)] + (["--algorithm_name", "momat"] if n_obj == 2 else []),
                      get_config(), warn=False)
    res = []
    g = torch.Generator(device=gpu).manual_seed(3)
    B, A = 96, 9
    obs = torch.rand(B, A, 7, device=gpu, generator=g)
    ava = torch.ones(B, A, 2, device=gpu)
    actions = (torch.rand(B, A, 1, device=gpu, generator=g) < 0.5).float()
    actions[:, -1] = torch.rand(B, 1, device=gpu, generator=g)
    for fused in (True, False):
        torch.manual_seed(0)
        pol = TransformerPolicy(args, [7], [10], dcml_action_spaces(8)[0], A, device=gpu)
        comm = Comm(device=gpu)
        comm.attach_flat_grads(pol.transformer.parameters())
        tr = MATTrainer(args, pol, A, device=gpu, comm=comm)
        assert tr.fused is True
        tr.fused = fused
        if not fused:
            pol.optimizer = torch.optim.Adam(pol.transformer.parameters(), lr=5e-4, eps=1e-5)
        with torch.no_grad():
            v0, lp0, _ = pol.evaluate_actions(None, obs, actions, ava)
        mb = {"obs": obs, "actions": actions, "ava": ava, "old_logp": lp0 + 0.05, "adv": torch.randn(B, A, n_obj, device=gpu, generator=torch.Generator(device=gpu).manual_seed(5)),
              "value_preds": v0, "returns": v0 + 1.0, "active": torch.ones(B, A, 1, device=gpu)}
        before = [p.detach().clone() for p in pol.transformer.parameters()]
        if fused:
            tr.loss_fused.out.zero_()
            tr.ppo_update_fused(mb)
        else:
            tr.ppo_update(mb)
        torch.cuda.synchronize()
        res.append(torch.cat([(p.detach() - b).reshape(-1) for p, b in zip(pol.transformer.parameters(), before)]))
    d_f, d_t = res
    cos = torch.nn.functional.cosine_similarity(d_f, d_t, dim=0)
    assert cos > 0.999, float(cos)
    assert torch.allclose(d_f.norm(), d_t.norm(), rtol=1e-2)


@pytest.mark.parametrize("pam", [True, False])
def test_ppo_loss_continuous_multi_dim_matches_reference_formula(gpu, pam):
    """Continuous action type with A = 3 action dimensions: (N, 3) log-probs / entropies, (N, 1) advantages and
    active masks.  Reference formulas (mat_trainer.py:129-139, transformer_policy.py:212-215): the surrogate and,
    under policy active masks, the entropy are SUMMED over the dimensions and divided by the active-token count;
    without the masks both are means over the tokens (entropy: over every (token, dim) entry)."""
    from mat_dcml_amd.ops.ppo_fused import PPOLossFused
    g = torch.Generator(device=gpu).manual_seed(7)
    N, A = 3000, 3
    r = lambda *s: torch.randn(*s, device=gpu, generator=g)  # noqa: E731
    v, lp, ent = r(N, 1), r(N, A) * 0.3 - 0.7, r(N, A).abs()
    mb = {"old_logp": lp + 0.3 * r(N, A), "adv": r(N, 1), "value_preds": v + 0.3 * r(N, 1), "returns": 3 * r(N, 1) + 1,
          "active": (torch.rand(N, 1, device=gpu, generator=g) > 0.2).float()}
    tr = _args(_use_policy_active_masks=pam)
    tr.value_normalizer = None
    fused = PPOLossFused(tr, gpu)
    fused.out.zero_()
    dv, dlp, dent = fused.run(v, lp, ent, mb)
    ll, ee = lp.clone().requires_grad_(), ent.clone().requires_grad_()
    imp = torch.exp(ll - mb["old_logp"])
    s1, s2 = imp * mb["adv"], imp.clamp(1 - tr.clip_param, 1 + tr.clip_param) * mb["adv"]
    act = mb["active"]
    if pam:
        pl = (-torch.sum(torch.min(s1, s2) * act, dim=-1, keepdim=True)).sum() / act.sum()
        e = (ee * act).sum() / act.sum()
    else:
        pl = -torch.sum(torch.min(s1, s2), dim=-1, keepdim=True).mean()
        e = ee.mean()
    (pl - e * tr.entropy_coef).backward()
    torch.cuda.synchronize()
    assert torch.allclose(dlp, ll.grad, atol=1e-8, rtol=1e-4), (dlp - ll.grad).abs().max()
    assert torch.allclose(dent, ee.grad, atol=1e-10, rtol=1e-4), (dent[:2], ee.grad[:2])
    o = fused.out
    assert torch.allclose(o[0], pl.detach(), rtol=1e-4, atol=1e-5), (o[0], pl)
    assert torch.allclose(o[2], e.detach(), rtol=1e-4, atol=1e-5), (o[2], e)
