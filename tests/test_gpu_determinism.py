"""Determinism harness for the HIP kernels (run twice with the same Philox seed, require
bitwise-equal outputs — a missing barrier or an LDS race shows up as run-to-run differences).

* DCML env reset / step kernels: bitwise equal across two envs with the same seed and actions;
* persistent decode kernel (stochastic and deterministic, stride 1 and stride blocks): bitwise equal actions /
  log-probs for the same inputs and draws, also with other work interleaved on the stream;
* fused training forward (values, log-probs, entropies): bitwise equal;
* fused backward called through autograd (no trainer workspace): weight gradients are accumulated with fp32 atomics
  straight into ``.grad``, whose summation order may differ between runs — required to agree to fp32 rounding
  (relative 1e-5), and the max deviation is printed;
* the trainer's fused PPO update (round 6, reference ``--cuda_deterministic``, DCML_MAT_Train.py:108-110): private
  per-workgroup gradient copies, 2^-32 fixed-point vector accumulators and fixed-order reductions make two whole PPO
  iterations (rollout + 2 epochs, the fused reduce + clip / Adam / repack launches included) BITWISE identical —
  parameters, Adam moments and the optimizer scratch (grad norm, skipped-step count) — with the fused and the unfused
  update alike.
"""
import os

import pytest
import torch

from mat_dcml_amd.envs.dcml.config import DCMLConfig
from mat_dcml_amd.envs.dcml.vec_env import DeviceDCMLEnv
from mat_dcml_amd.ops import mat_fused, mat_train

from test_gpu_decode import inputs as dec_inputs, make as dec_make
from test_gpu_train import make as train_make

pytestmark = pytest.mark.gpu


def _same(a, b):
    return a.shape == b.shape and torch.equal(a, b)


def test_env_kernels_bitwise_repeatable(gpu):
    cfg = DCMLConfig(n_workers=32)
    envs = [DeviceDCMLEnv(128, cfg, device=gpu, seed=11, backend="hip") for _ in range(2)]
    outs = [e.reset() for e in envs]
    assert all(_same(a, b) for a, b in zip(*outs))
    g = torch.Generator(device=gpu).manual_seed(0)
    for _ in range(8):
        act = (torch.rand(128, 33, device=gpu, generator=g) < 0.5).float()
        act[:, -1] = torch.rand(128, device=gpu, generator=g)
        r = [e.step(act) for e in envs]
        assert all(_same(a, b) for a, b in zip(*r))


@pytest.mark.parametrize("det,stride", [(False, 1), (True, 1), (True, 10)])
def test_decode_bitwise_repeatable(gpu, det, stride):
    L, B = 33, 200
    m = dec_make(L, gpu)
    obs, ava, rep, rand = dec_inputs(m, B, L, gpu)
    a1, lp1 = mat_fused.decode(m, rep, ava, det, stride, rand)
    junk = torch.randn(4096, 4096, device=gpu) @ torch.randn(4096, 4096, device=gpu)   # perturb timing / caches
    a2, lp2 = mat_fused.decode(m, rep, ava, det, stride, rand)
    torch.cuda.synchronize()
    del junk
    assert _same(a1, a2) and _same(lp1, lp2)


def test_fused_training_repeatable(gpu):
    L, B = 33, 160
    m = train_make(L, gpu, seed=5)
    g = torch.Generator(device=gpu).manual_seed(6)
    obs = torch.rand(B, L, 7, device=gpu, generator=g)
    ava = torch.ones(B, L, 2, device=gpu)
    ava[:, 2::5, 1] = 0
    actions = (torch.rand(B, L, 1, device=gpu, generator=g) < 0.5).float()
    actions[ava[..., 1:] == 0] = 0
    actions[:, -1, 0] = torch.rand(B, device=gpu, generator=g)
    w = [torch.randn(B, L, 1, device=gpu, generator=g) for _ in range(3)]
    fwd, grads = [], []
    for _ in range(2):
        for p in m.parameters():
            p.grad = torch.zeros_like(p)
        v, lp, ent = mat_train.evaluate_actions(m, obs, actions, ava)
        ((lp * w[0]).sum() + (v * w[1]).sum() + (ent * w[2]).sum()).backward()
        torch.cuda.synchronize()
        fwd.append((v.detach().clone(), lp.detach().clone(), ent.detach().clone()))
        grads.append({n: p.grad.detach().clone() for n, p in m.named_parameters()})
    assert all(_same(a, b) for a, b in zip(*fwd)), "fused forward is not bitwise repeatable"
    worst = 0.0
    # key biases get ~zero gradient (softmax is shift invariant): measure them against a floor of the global norm
    floor = 1e-3 * torch.stack([g.norm() for g in grads[0].values()]).norm()
    for n, g1 in grads[0].items():
        g2 = grads[1][n]
        d = ((g1 - g2).norm() / (g1.norm() + floor)).item()
        worst = max(worst, d)
        assert d < 1e-5, (n, d)
    print(f"max relative run-to-run gradient deviation (fp32 atomic order): {worst:.2e}")


def _ppo_run(gpu, iters=2, fused_update=True, mb_index="gather", gather_ahead=False, fused_gather=True):
    from mat_dcml_amd.config import get_config, parse_args
    from mat_dcml_amd.parallel.comm import Comm
    from mat_dcml_amd.runner.dcml_runner import DCMLRunner
    env = {"MAT_DCML_FUSED_UPDATE": "1" if fused_update else "0", "MAT_DCML_MB_INDEX": mb_index,
           "MAT_DCML_GATHER_AHEAD": "1" if gather_ahead else "0", "MAT_DCML_FUSED_GATHER": "1" if fused_gather else "0"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        args = parse_args(["--n_workers", "32", "--n_rollout_threads", "32", "--episode_length", "10", "--ppo_epoch",
                           "2", "--num_mini_batch", "2", "--use_valuenorm", "--env_name", "DCML", "--seed", "3"],
                          get_config(), warn=False)
        r = DCMLRunner({"all_args": args, "device": gpu, "run_dir": None, "comm": Comm(device=gpu)})
        tr = r.trainer
        assert tr.fused and tr.deterministic and tr._upd_fused == fused_update and tr.gather_ahead == gather_ahead
        r.warmup()
        for _ in range(iters):
            r.train_iteration()
        torch.cuda.synchronize()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    opt = r.policy.optimizer
    return {"params": torch.cat([p.detach().reshape(-1) for p in r.policy.transformer.parameters()]),
            "exp_avg": opt.m.clone(), "exp_avg_sq": opt.v.clone(), "scratch": opt.scratch[:4].clone()}


def test_fused_ppo_iteration_bitwise_repeatable(gpu):
    a, b = _ppo_run(gpu), _ppo_run(gpu)
    for k in a:
        assert torch.equal(a[k], b[k]), (k, (a[k] - b[k]).abs().max().item())
    print("two fused PPO iterations x 2 runs: parameters, Adam moments and optimizer scratch bitwise equal")


def test_fused_update_matches_unfused_update(gpu):
    """The fused reduce + clip / Adam / repack (csrc/ppo.hip mdl_update_fused: grad_reduce_priv + adam_pack) against
    the separate grad_reduce_priv + adam_step + pack_weights launches: the same norm partials in the same order, so
    the runs agree to the last bits of the Adam arithmetic (the two kernels' FMA contraction may differ)."""
    a, b = _ppo_run(gpu, fused_update=True), _ppo_run(gpu, fused_update=False)
    assert torch.equal(a["scratch"][1:3], b["scratch"][1:3]) or \
        abs(float(a["scratch"][1]) - float(b["scratch"][1])) <= 1e-6 * float(b["scratch"][1])
    d = ((a["params"] - b["params"]).norm() / b["params"].norm()).item()
    print(f"fused vs unfused update: relative parameter difference {d:.2e}")
    assert d < 1e-6, d


def test_kernel_minibatch_index_matches_gather(gpu):
    """MAT_DCML_MB_INDEX=kernel (the training kernels and the PPO loss read the buffer's rows through the epoch
    permutation, csrc/mat_train_common.h src_tok, and standardise the advantages in-kernel) against the default
    gather of each minibatch: the same rows in the same order, so the two runs agree to the advantage
    standardisation's rounding (in-kernel (a - mean) * rstd vs the gather kernel's)."""
    a, b = _ppo_run(gpu, mb_index="kernel"), _ppo_run(gpu, mb_index="gather")
    d = ((a["params"] - b["params"]).norm() / b["params"].norm()).item()
    dm = ((a["exp_avg"] - b["exp_avg"]).norm() / b["exp_avg"].norm()).item()
    print(f"in-kernel minibatch index vs gather: relative parameter difference {d:.2e}, first moment {dm:.2e}")
    assert d < 1e-5 and dm < 1e-3, (d, dm)


def test_gather_placement_is_bitwise_neutral(gpu):
    """The next minibatch's gather inside the fused update's adam_pack launch (default, csrc/gather_rows.h
    gather_rows_wavewise) and on a side stream (algos/mat_trainer._GatherAhead) against the standalone in-line
    gather: the same rows and the same standardisation arithmetic, so parameters and Adam moments are bitwise equal."""
    base = _ppo_run(gpu, gather_ahead=False, fused_gather=False)
    for kw in (dict(fused_gather=True), dict(gather_ahead=True, fused_gather=False)):
        a = _ppo_run(gpu, **kw)
        for k in a:
            assert torch.equal(a[k], base[k]), (kw, k, (a[k] - base[k]).abs().max().item())
