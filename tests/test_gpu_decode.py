"""Persistent HIP decode kernel vs the PyTorch fp32 autoregressive decode (same random draws)."""
import pytest
import torch

from mat_dcml_amd.models import act
from mat_dcml_amd.models.mat import MultiAgentTransformer
from mat_dcml_amd.ops import mat_fused

pytestmark = pytest.mark.gpu


def make(L, dev, atype="Semi_Discrete", A=2, seed=0, scale=0.3, nb=2):
    torch.manual_seed(seed)
    m = MultiAgentTransformer(L + 1, 7, A, L, nb, 64, 2, action_type=atype, semi_index=-1).to(dev)
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for p in m.parameters():
            p.copy_((torch.randn(p.shape, generator=g) * scale).to(dev))
    return m


def inputs(m, B, L, dev, A=2, seed=1):
    g = torch.Generator(device=dev).manual_seed(seed)
    obs = torch.rand(B, L, 7, device=dev, generator=g)
    ava = torch.ones(B, L, A, device=dev)
    ava[:, 1::3, -1] = 0
    with torch.no_grad():
        v, rep = m.encoder(None, obs)
    rand = {"u": torch.rand(B, L, device=dev, generator=g), "n": torch.randn(B, L, A, device=dev, generator=g)}
    return obs, ava, rep, rand


@pytest.mark.parametrize("L,B", [(33, 256), (5, 64), (101, 16), (129, 8), (33, 3)])
@pytest.mark.parametrize("det", [False, True])
def test_decode_matches_torch(gpu, L, B, det):
    m = make(L, gpu)
    assert mat_fused.supports(m)
    obs, ava, rep, rand = inputs(m, B, L, gpu)
    a_ref, lp_ref = act.autoregressive_act(m, rep, obs, ava, det, 1, rand)
    a_k, lp_k = mat_fused.decode(m, rep, ava, det, 1, rand)
    torch.cuda.synchronize()
    disc = slice(0, L - 1)
    agree = (a_ref[:, disc] == a_k[:, disc]).float().mean().item()
    assert agree > 0.97, agree
    # localised by row: the first divergence of an env propagates to its later rows, so disagreement grows with the
    # row index; a fault confined to some rows would stand out well above the average bound
    if B >= 64:
        per_row = (a_ref[:, disc] != a_k[:, disc]).float().mean(0).squeeze(-1)
        assert per_row.max().item() < 0.1, per_row.tolist()
    assert (a_k[:, disc][ava[:, disc, 1:] == 0] == 0).all()  # masked workers never selected
    # kernel log-probs are the teacher-forced log-probs of the kernel's own actions
    with torch.no_grad():
        lp_tf, _ = act.parallel_act(m, rep, obs, a_k, ava)
    err = (lp_tf - lp_k).abs()
    print(f"[decode-lp] L={L} B={B} det={det}: agree {agree:.4f} lp err mean {err.mean().item():.3e} "
          f"max {err.max().item():.3e}")
    # 1.5 x the worst measured values over these cases (round 6: mean 1.94e-3 at L = 5, max 0.139 at L = 129 with
    # random weights of scale 0.3; gpurun_out/r6_logprob.log)
    assert err.mean().item() < 3e-3 and err.max().item() < 0.21, (err.mean().item(), err.max().item())
    row_err = err.mean(0).view(-1)
    assert row_err.max().item() < 4e-2, row_err.tolist()
    if det:
        assert torch.allclose(a_ref[:, -1], a_k[:, -1], atol=5e-2)


@pytest.mark.parametrize("L", [33, 101, 129])
@pytest.mark.parametrize("stride", [2, 10])
def test_decode_stride_mode(gpu, stride, L):
    """Batch decision (``stride``, transformer_act.py:37-75): the deterministic mode behind every eval ct / payment
    number (benchmark protocol stride 10, runner eval stride 2).  B = 64 envs; the disagreement with the fp32 torch
    decode is bounded per ROW as well as on average, so a fault confined to some in-block positions would show."""
    B = 64
    m = make(L, gpu, seed=3)
    obs, ava, rep, rand = inputs(m, B, L, gpu)
    a_ref, lp_ref = act.autoregressive_act(m, rep, obs, ava, True, stride, None)
    a_k, lp_k = mat_fused.decode(m, rep, ava, True, stride, None)
    torch.cuda.synchronize()
    disc = slice(0, L - 1)
    agree = (a_ref[:, disc] == a_k[:, disc]).float().mean().item()
    assert agree > 0.97, agree
    per_row = (a_ref[:, disc] != a_k[:, disc]).float().mean(0).squeeze(-1)
    assert per_row.max().item() < 0.1, per_row.tolist()
    assert (a_k[:, disc][ava[:, disc, 1:] == 0] == 0).all()   # masked workers never selected
    assert (lp_ref - lp_k).abs().mean().item() < 3e-2
    row_err = (lp_ref - lp_k).abs().mean(0).view(-1)
    assert row_err.max().item() < 0.1, row_err.tolist()
    assert torch.allclose(a_ref[:, -1], a_k[:, -1], atol=5e-2)   # the ratio agent (deterministic mean)


@pytest.mark.parametrize("det", [False, True])
def test_decode_discrete_smac_shape(gpu, det):
    """SMAC's Discrete(36) head with availability masks: the wide fused head (lane = action, ballot argmax, prefix-scan
    inverse CDF; csrc/mat_decode.hip) against the fp32 torch decode on the same draws."""
    L, B, A = 27, 32, 36
    m = make(L, gpu, atype="Discrete", A=A, seed=5)
    obs, ava, rep, rand = inputs(m, B, L, gpu, A=A)
    g = torch.Generator(device=gpu).manual_seed(7)
    ava = (torch.rand(B, L, A, device=gpu, generator=g) < 0.6).float()
    ava[..., 0] = 1.0
    a_ref, _ = act.autoregressive_act(m, rep, obs, ava, det, 1, rand)
    a_k, lp_k = mat_fused.decode(m, rep, ava, det, 1, rand)
    # a divergence changes every later row of its env (the next token), so count only decisions taken from the
    # same prefix: the first divergences among the decisions whose earlier rows all agree (bf16 near-ties)
    eq = (a_ref == a_k).squeeze(-1).float()
    same_prefix = torch.cat([torch.ones_like(eq[:, :1]), torch.cumprod(eq, 1)[:, :-1]], 1)
    rate = ((1 - eq) * same_prefix).sum().item() / same_prefix.sum().item()
    assert (ava.gather(-1, a_k.long()) == 1).all()   # masked actions never selected
    if det:
        # argmax: bf16 operands flip near-ties, so check the regret of every kernel choice against the fp32
        # teacher-forced logits given the kernel's own earlier actions: a near-tie, never a clearly worse action
        with torch.no_grad():
            lg = m.decoder(act.shifted_from_actions(m, a_k).to(rep.dtype), rep, obs).float()
        lg = lg.masked_fill(ava == 0, -1e10)
        regret = lg.max(-1).values - lg.gather(-1, a_k.long()).squeeze(-1)
        assert regret.max().item() < 2e-2, (regret.max().item(), rate)
    else:
        assert rate < 0.02, rate
    with torch.no_grad():
        lp_tf, _ = act.parallel_act(m, rep, obs, a_k, ava)
    assert (lp_tf - lp_k).abs().mean().item() < 3e-2
    if not det:   # timing at the SMAC rollout shape
        for _ in range(3):
            mat_fused.decode(m, rep, ava, False, 1, rand)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            mat_fused.decode(m, rep, ava, False, 1, rand)
        e.record()
        torch.cuda.synchronize()
        print(f"mat_decode B=32 L=27 A=36: {s.elapsed_time(e) / 20 * 1e3:.1f} us per env step")


# 1.25 x the round-5 measurements (median of timed windows; profiles/r5_final/perf_guards.jsonl: 148.3 / 532.1 us)
DECODE_BOUND_US = {33: 185.0, 101: 665.0}


@pytest.mark.parametrize("L", [33, 101])
def test_decode_latency(gpu, L):
    B = 256
    m = make(L, gpu)
    obs, ava, rep, rand = inputs(m, B, L, gpu)
    from conftest import median_us, perf_record
    us = median_us(lambda: mat_fused.decode(m, rep, ava, False, 1, rand))
    perf_record(f"decode_256x{L}_us", us, DECODE_BOUND_US[L])
    assert us < DECODE_BOUND_US[L], us


@pytest.mark.parametrize("L,A,B", [(6, 1, 64), (2, 6, 40), (17, 3, 16), (33, 2, 8)])
@pytest.mark.parametrize("det", [False, True])
def test_decode_continuous_matches_torch(gpu, L, A, B, det):
    """"Continuous" action type (MA-MuJoCo): every agent samples act_dim Gaussians and the next row's decoder
    input is LN(GELU(W_a x + b_a)) of the sampled vector, built inside the kernel."""
    torch.manual_seed(0)
    m = MultiAgentTransformer(L + 1, 7, A, L, 2, 64, 2, action_type="Continuous").to(gpu)
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for p in m.parameters():
            p.copy_((torch.randn(p.shape, generator=g) * 0.3).to(gpu))
    assert mat_fused.supports(m)
    obs, ava, rep, rand = inputs(m, B, L, gpu, A=A)
    ava = torch.ones(B, L, A, device=gpu)
    a_ref, lp_ref = act.autoregressive_act(m, rep, obs, ava, det, 1, rand)
    a_k, lp_k = mat_fused.decode(m, rep, ava, det, 1, rand)
    torch.cuda.synchronize()
    assert a_k.shape == (B, L, A) and lp_k.shape == (B, L, A)
    # bf16 MFMA decoder vs fp32 torch: actions agree closely, and the kernel's log-probs are exact for its own
    # actions under the teacher-forced (torch) decoder
    assert (a_k - a_ref).abs().max().item() < 0.1, (a_k - a_ref).abs().max().item()
    with torch.no_grad():
        lp_tf, _ = act.parallel_act(m, rep, obs, a_k, ava)
    err = (lp_tf - lp_k).abs()
    assert err.mean().item() < 2e-2 and err.max().item() < 0.2, (err.mean().item(), err.max().item())


def test_decode_inkernel_draws(gpu):
    """rand=None: the kernel draws its own Philox noise.  Discrete rows: the frequency of action 1 matches the mean
    probability the kernel assigned to it (from its own log-probs); the continuous last row: the standardised
    samples recovered from the log-probs have E[z^2] = 1; successive calls draw fresh noise."""
    L, B = 9, 4096
    m = make(L, gpu, seed=5)
    obs, ava, rep, _ = inputs(m, B, L, gpu)
    ava = torch.ones_like(ava)
    a1, lp1 = mat_fused.decode(m, rep, ava, False, 1, None)
    a2, _ = mat_fused.decode(m, rep, ava, False, 1, None)
    torch.cuda.synchronize()
    assert not torch.equal(a1, a2)
    a, p = a1[:, :L - 1, 0], lp1[:, :L - 1, 0].exp()
    p1 = torch.where(a == 1, p, 1 - p)                      # P(action 1) of every (env, row)
    freq, mean_p = (a == 1).float().mean(0), p1.mean(0)
    se = (mean_p * (1 - mean_p) / B).sqrt()
    assert ((freq - mean_p).abs() < 5 * se + 1e-3).all(), (freq.tolist(), mean_p.tolist())
    sd = m.action_std().float()[-1]
    z2 = -2 * (lp1[:, -1, 0] + sd.log() + 0.9189385332)
    assert abs(z2.mean().item() - 1) < 5 * (2 / B) ** 0.5, z2.mean().item()


@pytest.mark.parametrize("L,A,B", [(5, 4, 64), (17, 3, 32)])
@pytest.mark.parametrize("det", [False, True])
def test_decode_available_continuous_matches_torch(gpu, L, A, B, det):
    """"Available_Continuous" (transformer_act.py:234-283): per agent a categorical over the first two logits
    (availability-masked) plus Normals over the rest; the action vector [onehot(a), x] feeds the next row."""
    torch.manual_seed(0)
    m = MultiAgentTransformer(L + 1, 7, A, L, 2, 64, 2, action_type="Available_Continuous").to(gpu)
    g = torch.Generator().manual_seed(2)
    with torch.no_grad():
        for p in m.parameters():
            p.copy_((torch.randn(p.shape, generator=g) * 0.3).to(gpu))
    assert mat_fused.supports(m), mat_fused.unsupported_reasons(m)
    obs, ava, rep, rand = inputs(m, B, L, gpu, A=A)
    ava = torch.ones(B, L, A, device=gpu)
    ava[:, 1::2, 1] = 0   # every other agent may not take option 1
    a_ref, lp_ref = act.autoregressive_act(m, rep, obs, ava, det, 1, rand)
    a_k, lp_k = mat_fused.decode(m, rep, ava, det, 1, rand)
    torch.cuda.synchronize()
    assert a_k.shape == (B, L, A) and lp_k.shape == (B, L, A - 1)
    assert (a_k[:, 1::2, 1] == 0).all()   # masked option never chosen
    agree = (a_ref[..., :2] == a_k[..., :2]).all(-1).float().mean().item()
    assert agree > 0.97, agree
    with torch.no_grad():
        lp_tf, _ = act.parallel_act(m, rep, obs, a_k, ava)
    err = (lp_tf - lp_k).abs()
    assert err.mean().item() < 2e-2 and err.max().item() < 0.2, (err.mean().item(), err.max().item())


def _both_kernels(m, rep, ava, det, rand, spec=False):
    """The same decode call on the one-wave kernel (csrc/mat_decode_wave.hip; spec: its speculative-block-0 variant
    where the configuration allows it) and on the 4-wave kernel."""
    saved = mat_fused.WAVE_DECODE, mat_fused.SPEC_DECODE
    try:
        mat_fused.WAVE_DECODE, mat_fused.SPEC_DECODE = True, spec
        a_w, lp_w = mat_fused.decode(m, rep, ava, det, 1, rand)
        path = m._mdl_decode_path
        mat_fused.WAVE_DECODE = False
        a_4, lp_4 = mat_fused.decode(m, rep, ava, det, 1, rand)
    finally:
        mat_fused.WAVE_DECODE, mat_fused.SPEC_DECODE = saved
    torch.cuda.synchronize()
    return path, a_w, lp_w, a_4, lp_4


@pytest.mark.parametrize("L,B,nb,atype,A", [(33, 256, 2, "Semi_Discrete", 2), (33, 64, 1, "Semi_Discrete", 2),
                                            (5, 64, 2, "Semi_Discrete", 2), (101, 16, 1, "Semi_Discrete", 2),
                                            (27, 32, 2, "Discrete", 36), (9, 48, 1, "Discrete", 3),
                                            # the speculative kernel's other layouts: 3..4 narrow-head candidates
                                            # (16-candidate layout, MA 1), one / two candidate waves of a wide head
                                            (9, 48, 2, "Discrete", 3), (12, 32, 2, "Discrete", 6),
                                            (10, 24, 2, "Discrete", 20)])
@pytest.mark.parametrize("det", [False, True])
@pytest.mark.parametrize("spec", [False, True])
def test_wave_decode_matches_4wave_and_torch(gpu, L, B, nb, atype, A, det, spec):
    """One-wave decode (and, n_block 2, its speculative-block-0 variant) vs the 4-wave kernel and the fp32 torch decode
    on the same draws: decisions taken from the same prefix agree (bf16 near-ties aside), the kernel's log-probs are
    the teacher-forced log-probs of its own actions, masked actions are never taken, and the launch really is the
    kernel under test."""
    m = make(L, gpu, atype=atype, A=A, seed=11, nb=nb)
    obs, ava, rep, rand = inputs(m, B, L, gpu, A=A)
    if A > 2:
        g = torch.Generator(device=gpu).manual_seed(3)
        ava = (torch.rand(B, L, A, device=gpu, generator=g) < 0.6).float()
        ava[..., 0] = 1.0
    path, a_w, lp_w, a_4, lp_4 = _both_kernels(m, rep, ava, det, rand, spec)
    assert path.startswith("spec" if spec and nb == 2 else "wave"), path
    a_ref, _ = act.autoregressive_act(m, rep, obs, ava, det, 1, rand)
    n_disc = L if atype == "Discrete" else L - 1
    for other in (a_4, a_ref):
        eq = (other[:, :n_disc] == a_w[:, :n_disc]).squeeze(-1).float()
        same_prefix = torch.cat([torch.ones_like(eq[:, :1]), torch.cumprod(eq, 1)[:, :-1]], 1)
        rate = ((1 - eq) * same_prefix).sum().item() / same_prefix.sum().item()
        assert rate < 0.02, rate
    assert (ava[:, :n_disc].gather(-1, a_w[:, :n_disc].long()) == 1).all()
    with torch.no_grad():
        lp_tf, _ = act.parallel_act(m, rep, obs, a_w, ava)
    err = (lp_tf - lp_w).abs()
    assert err.mean().item() < 2e-2 and err.max().item() < 0.2, (err.mean().item(), err.max().item())
    if n_disc < L:   # the ratio agent: same Normal draw, mean within bf16 noise of the 4-wave kernel
        same = (a_4[:, :n_disc] == a_w[:, :n_disc]).all(1).squeeze(-1)
        assert (a_4[same, -1] - a_w[same, -1]).abs().max().item() < 5e-2


@pytest.mark.parametrize("L,layout", [(101, 0), (101, 1), (101, 2), (129, 0)])
@pytest.mark.parametrize("det", [False, True])
def test_spec_decode_long_rows_token_table(gpu, det, L, layout):
    """256 x 101 with n_block 2: both blocks' K / V caches do not fit next to the speculative kernel's other operands,
    so block 0's self-attention K / V are read through the row -> token array from the token table ('tokrows'); at
    L = 129 the cross-attention queries are computed in place as well ('q2inline').  At L = 101 the plain carve fits
    with 8 register-resident main-wave matrices (the default there); layout 1 / 2 force the token-table variants
    (mdl_decode_spec_layout).  Same checks as the one-wave parity test."""
    B = 64
    m = make(L, gpu, seed=13)
    obs, ava, rep, rand = inputs(m, B, L, gpu)
    from mat_dcml_amd.ops.kernels import lib
    lib().mdl_decode_spec_layout(layout)
    try:
        path, a_s, lp_s, a_4, lp_4 = _both_kernels(m, rep, ava, det, rand, spec=True)
    finally:
        lib().mdl_decode_spec_layout(0)
    want = {0: "q2inline" if L == 129 else "", 1: "tokrows", 2: "q2inline"}[layout]
    assert path.startswith("spec") and want in path, path
    assert ("tokrows" in path) == (layout > 0 or L == 129), path
    a_ref, _ = act.autoregressive_act(m, rep, obs, ava, det, 1, rand)
    n_disc = L - 1
    for other in (a_4, a_ref):
        eq = (other[:, :n_disc] == a_s[:, :n_disc]).squeeze(-1).float()
        same_prefix = torch.cat([torch.ones_like(eq[:, :1]), torch.cumprod(eq, 1)[:, :-1]], 1)
        rate = ((1 - eq) * same_prefix).sum().item() / same_prefix.sum().item()
        assert rate < 0.02, rate
    with torch.no_grad():
        lp_tf, _ = act.parallel_act(m, rep, obs, a_s, ava)
    err = (lp_tf - lp_s).abs()
    assert err.mean().item() < 2e-2 and err.max().item() < 0.2, (err.mean().item(), err.max().item())


def test_wave_decode_inkernel_draws_match_4wave(gpu):
    """rand=None (in-kernel Philox keyed by env / row / call counter): both kernels draw the same noise, so with the
    same key they take the same decisions except at bf16 near-ties."""
    L, B = 33, 256
    m = make(L, gpu, seed=4)
    obs, ava, rep, _ = inputs(m, B, L, gpu)
    mat_fused.set_sampling_key(m, 123)
    saved = mat_fused.WAVE_DECODE
    try:
        mat_fused.WAVE_DECODE = True
        a_w, _ = mat_fused.decode(m, rep, ava, False, 1, None)
        mat_fused.set_sampling_key(m, 123)
        mat_fused.WAVE_DECODE = False
        a_4, _ = mat_fused.decode(m, rep, ava, False, 1, None)
    finally:
        mat_fused.WAVE_DECODE = saved
    eq = (a_4[:, :L - 1] == a_w[:, :L - 1]).squeeze(-1).float()   # discrete rows (the last is the ratio agent)
    same_prefix = torch.cat([torch.ones_like(eq[:, :1]), torch.cumprod(eq, 1)[:, :-1]], 1)
    rate = ((1 - eq) * same_prefix).sum().item() / same_prefix.sum().item()
    assert rate < 0.02, rate
    same = eq.all(1)
    assert (a_4[same, -1] - a_w[same, -1]).abs().max().item() < 5e-2   # same Normal draw for the ratio agent


# one-wave kernel bounds: 1.25 x the round-5 measurements (227.8 / 431.5 / 203.1 us, profiles/r5_final/perf_guards.jsonl)
WAVE_BOUND_US = {(33, 2, 2, 256): 285.0, (101, 1, 2, 256): 540.0, (27, 2, 36, 32): 254.0}
# speculative-block-0 kernel (the default rollout path at these shapes): 1.25 x 148.6 / 132.5 / 538.3 / 724.7 us
SPEC_BOUND_US = {(33, 2, 2, 256): 186.0, (27, 2, 36, 32): 166.0, (101, 2, 2, 256): 673.0, (129, 2, 2, 256): 906.0}


@pytest.mark.parametrize("L,nb,A,B", [(33, 2, 2, 256), (101, 1, 2, 256), (27, 2, 36, 32), (101, 2, 2, 256),
                                      (129, 2, 2, 256)])
def test_wave_decode_latency(gpu, L, nb, A, B):
    """Per-env-step decode time of both kernels at the rollout shapes (printed; the one-wave kernel must not be
    slower than the 4-wave one)."""
    m = make(L, gpu, nb=nb, A=A, atype="Discrete" if A > 2 else "Semi_Discrete")
    obs, ava, rep, rand = inputs(m, B, L, gpu, A=A)
    from conftest import median_us
    saved = mat_fused.WAVE_DECODE, mat_fused.SPEC_DECODE
    res, paths = {}, {}
    try:
        for kind, wave, spec in (("spec", True, True), ("wave", True, False), ("4wave", False, False)):
            mat_fused.WAVE_DECODE, mat_fused.SPEC_DECODE = wave, spec
            res[kind] = median_us(lambda: mat_fused.decode(m, rep, ava, False, 1, None))
            paths[kind] = m._mdl_decode_path
    finally:
        mat_fused.WAVE_DECODE, mat_fused.SPEC_DECODE = saved
    from conftest import perf_record
    perf_record(f"decode_4wave_{B}x{L}_nb{nb}_A{A}_us", res["4wave"], None)
    if paths["wave"].startswith("wave"):
        perf_record(f"decode_wave_{B}x{L}_nb{nb}_A{A}_us", res["wave"], WAVE_BOUND_US[(L, nb, A, B)])
        assert res["wave"] < res["4wave"] * 1.05, res
        assert res["wave"] < WAVE_BOUND_US[(L, nb, A, B)], res
    if paths["spec"].startswith("spec"):
        perf_record(f"decode_spec_{B}x{L}_nb{nb}_A{A}_us", res["spec"], SPEC_BOUND_US.get((L, nb, A, B)))
        assert res["spec"] < min(res["wave"], res["4wave"]) * 1.05, res   # relative, with a jitter tolerance
        assert res["spec"] < SPEC_BOUND_US.get((L, nb, A, B), 1e9), res
