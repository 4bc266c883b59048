"""Rollout-vs-learner log-prob consistency.

PPO's importance weight ``exp(logp_new - logp_old)`` (reference ``mat_src/mat/algorithms/mat/mat_trainer.py:129-139``)
divides the learner's teacher-forced log-probs (``transformer_act.py:103-129``: here the fused training forward,
``csrc/mat_enc_ct.hip`` + ``csrc/mat_dec_ct.hip``) by the rollout's autoregressive ones (``transformer_act.py:76-99``:
here the production decode kernel — the speculative one-wave decode at 256 x 33 / 256 x 101, the SMAC shape too).
Both run bf16 MFMA products in different orders, so the ratio of the first minibatch of the first epoch — where the
policy has not moved — is 1 only up to that rounding.  This test rolls out with the production path, re-evaluates
the SAME observations / actions with the training forward, and bounds mean / max |Δ log-prob| and |mean ratio - 1|.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

CKPT32 = "profiles/r5_train32/transformer_500_beta3.pt"


def _dcml_runner(dev, n_workers, envs, T):
    from mat_dcml_amd.config import get_config, parse_args
    from mat_dcml_amd.parallel.comm import Comm
    from mat_dcml_amd.runner.dcml_runner import DCMLRunner
    argv = ["--env_name", "DCML", "--scenario", "AS", "--algorithm_name", "mat", "--n_rollout_threads", str(envs),
            "--episode_length", str(T), "--use_valuenorm", "--use_popart", "--n_workers", str(n_workers),
            "--dtype", "bf16", "--seed", "1"]
    args = parse_args(argv, get_config(), warn=False)
    return DCMLRunner({"all_args": args, "device": dev, "run_dir": None, "comm": Comm(device=dev)})


def _smac_runner(dev, envs, T):
    from mat_dcml_amd.config import _SMAC_FLAGS, get_config, parse_args
    from mat_dcml_amd.parallel.comm import Comm
    from mat_dcml_amd.runner.smac_runner import SMACRunner
    argv = ["--env_name", "StarCraft2", "--algorithm_name", "mat", "--map_name", "27m_vs_30m", "--n_rollout_threads",
            str(envs), "--episode_length", str(T), "--dtype", "bf16", "--seed", "1"]
    args = parse_args(argv, get_config(), extra=_SMAC_FLAGS, warn=False)
    return SMACRunner({"all_args": args, "device": dev, "run_dir": None, "comm": Comm(device=dev)})


def _consistency(runner):
    """Roll out once with the production path, then the learner's fused forward on the buffer's rows."""
    from mat_dcml_amd.ops import mat_train
    from mat_dcml_amd.ops.paths import kernel_report
    runner.warmup()
    runner.rollout()
    torch.cuda.synchronize()
    b = runner.buffer
    m = runner.policy.transformer
    obs = b.flat("obs")
    act = b.flat("actions")
    ava = b.flat("available_actions")
    old = b.flat("action_log_probs")
    enc, dec, _ = mat_train._state(m, obs.device)
    with torch.no_grad():
        _, rep = enc.forward(obs, save=True)
        new, _ = dec.forward(rep, act, ava, save=True)
    torch.cuda.synchronize()
    d = (new.reshape(old.shape) - old).float()
    ratio = torch.exp(d)
    # epoch 0, minibatch 0 of the trainer: its first quarter of the rows (a permutation does not change the statistics)
    n0 = d.shape[0] // 4
    st = {"mean_abs": d.abs().mean().item(), "max_abs": d.abs().max().item(), "p999_abs": torch.quantile(
          d.abs().flatten()[:1 << 24], 0.999).item(), "ratio_mean_m1": ratio.mean().item() - 1.0,
          "ratio_mb0_mean_m1": ratio[:n0].mean().item() - 1.0, "ratio_max": ratio.max().item(),
          "ratio_min": ratio.min().item(), "decode": kernel_report(runner).get("decode")}
    # per agent position: the ratio agent (Semi_Discrete, last row) is a Normal head with std <= 0.5
    per_row = d.abs().mean(dim=tuple(i for i in range(d.dim()) if i != 1))
    st["worst_row"] = int(per_row.argmax())
    st["worst_row_mean_abs"] = per_row.max().item()
    cont_rows = m.action_type == "Semi_Discrete"
    disc = d[:, :-1] if cont_rows else d
    st["discrete_max_abs"] = disc.abs().max().item()
    if cont_rows:
        # the Normal ratio agent: d log p = z * d mu / sigma, so a mean that agrees to bf16 rounding still moves the
        # log-prob by |z| / sigma times that; the rounding-level quantity is sigma * |d log p| (a mean error times |z|)
        sd = float(m.action_std()[-1])
        st["ratio_agent_sigma"] = sd
        st["ratio_agent_max_abs"] = d[:, -1].abs().max().item()
        st["ratio_agent_sigma_x_max_abs"] = sd * st["ratio_agent_max_abs"]
    return st


CASES = {
    "dcml32_init": dict(kind="dcml", n_workers=32, envs=256, T=8, ckpt=None),
    "dcml32_trained": dict(kind="dcml", n_workers=32, envs=256, T=8, ckpt=CKPT32),
    "dcml100_init": dict(kind="dcml", n_workers=100, envs=256, T=4, ckpt=None),
    "smac_27m": dict(kind="smac", envs=32, T=16, ckpt=None),
}


@pytest.mark.parametrize("case", list(CASES))
def test_rollout_vs_learner_logprob(gpu, case):
    import os
    cfg = CASES[case]
    if cfg["ckpt"] and not os.path.exists(cfg["ckpt"]):
        pytest.skip("checkpoint not in the tree")
    torch.manual_seed(0)
    if cfg["kind"] == "dcml":
        runner = _dcml_runner(gpu, cfg["n_workers"], cfg["envs"], cfg["T"])
    else:
        runner = _smac_runner(gpu, cfg["envs"], cfg["T"])
    if cfg["ckpt"]:
        runner.policy.restore(cfg["ckpt"])
    st = _consistency(runner)
    print(f"[logprob] {case}: " + ", ".join(f"{k}={v:.3e}" if isinstance(v, float) else f"{k}={v}"
                                            for k, v in st.items()))
    assert math.isfinite(st["max_abs"])
    # mean |d| <= 5e-3, |mean ratio - 1| <= 1e-3 (the whole buffer and the first minibatch).
    # Tails: the two paths round to bf16 at different points (different tilings / op orders, fp32 differences that
    # flip an operand's bf16 rounding), and a trained policy's logits reach ~20, so the discrete rows' worst entry
    # of 65k is 0.08 nats (p99.9 0.015; measured round 6) — bounded at 0.1, the 99.9th percentile at 0.03.  The
    # continuous ratio agent's log-prob is 1 / sigma times more sensitive (sigma = 0.05 for the trained policy):
    # bounded as sigma * max |d| <= 1e-2 (its mean agrees to ~3e-3 / |z|).
    # Round 5's speculative decode failed all of these on the trained policy (mean 0.12, max 29: its PAIR head
    # exchange swapped the two candidates' second heads, csrc/mat_decode_wave.hip sp_attn_pair).
    assert st["mean_abs"] <= 5e-3, st
    assert st["discrete_max_abs"] <= 0.1, st
    assert st["p999_abs"] <= 3e-2, st
    if "ratio_agent_sigma" in st:
        assert st["ratio_agent_sigma_x_max_abs"] <= 1e-2, st
    assert abs(st["ratio_mean_m1"]) <= 1e-3, st
    assert abs(st["ratio_mb0_mean_m1"]) <= 1e-3, st
