"""FlatAdam checkpoints are torch.optim.Adam checkpoints: a fused-path trainer state resumes on the
eager path and vice versa.  CPU only (no kernel launch: the moments are set by hand)."""
import torch

from mat_dcml_amd.models.mat import MultiAgentTransformer
from mat_dcml_amd.ops.ppo_fused import FlatAdam, flatten_params, param_offsets


def _model():
    torch.manual_seed(0)
    m = MultiAgentTransformer(9, 7, 2, 8, 2, 64, 2, action_type="Semi_Discrete", semi_index=-1)
    flatten_params(m)
    return m


def test_flat_layout_is_padded_and_aligned():
    m = _model()
    for p, off in param_offsets(m):
        assert off % 16 == 0
        assert p.data_ptr() == m._mdl_flat_params.data_ptr() + 4 * off


def test_fused_state_loads_into_torch_adam_and_back():
    m = _model()
    flat = m._mdl_flat_params
    fa = FlatAdam(flat, torch.zeros_like(flat), lr=3e-4, eps=1e-5, layout=param_offsets(m))
    fa.m.copy_(torch.randn_like(flat))
    fa.v.copy_(torch.rand_like(flat))
    fa.t = 7
    sd = fa.state_dict()
    opt = torch.optim.Adam(m.parameters(), lr=1.0, eps=1e-5)
    opt.load_state_dict(sd)                      # eager resume of a fused-path checkpoint
    assert opt.param_groups[0]["lr"] == 3e-4
    for i, (p, off) in enumerate(param_offsets(m)):
        st = opt.state[p]
        assert float(st["step"]) == 7
        assert torch.equal(st["exp_avg"].reshape(-1), fa.m[off:off + p.numel()])
    fb = FlatAdam(flat, torch.zeros_like(flat), layout=param_offsets(m))
    fb.load_state_dict(opt.state_dict())         # and back (eager checkpoint -> fused resume)
    assert fb.t == 7
    mask = torch.zeros_like(flat, dtype=torch.bool)
    for p, off in param_offsets(m):
        mask[off:off + p.numel()] = True
    assert torch.equal(fb.m[mask], fa.m[mask]) and torch.equal(fb.v[mask], fa.v[mask])
    assert fb.m[~mask].abs().sum() == 0         # padding stays zero


def test_legacy_unpadded_state_is_remapped_or_reset():
    """Round-1 flat checkpoints ('m'/'v'/'t', parameters concatenated without padding): remapped through the padded
    layout; a state of any other size resets the moments AND t (zero moments with a large t would make the first
    steps ~3x too large: the bias corrections would be ~1)."""
    import pytest
    m = _model()
    flat = m._mdl_flat_params
    lay = param_offsets(m)
    n_raw = sum(p.numel() for p, _ in lay)
    raw_m, raw_v = torch.randn(n_raw), torch.rand(n_raw)
    fa = FlatAdam(flat, torch.zeros_like(flat), layout=lay)
    fa.load_state_dict({"m": raw_m, "v": raw_v, "t": 11, "param_groups": [{"lr": 1e-4}]})
    assert fa.t == 11 and fa.param_groups[0]["lr"] == 1e-4
    o = 0
    for p, off in lay:
        n = p.numel()
        assert torch.equal(fa.m[off:off + n], raw_m[o:o + n]) and torch.equal(fa.v[off:off + n], raw_v[o:o + n])
        o += n
    fb = FlatAdam(flat, torch.zeros_like(flat), layout=lay)
    with pytest.warns(UserWarning):
        fb.load_state_dict({"m": torch.randn(n_raw - 5), "v": torch.rand(n_raw - 5), "t": 11,
                            "param_groups": [{"lr": 1e-4}]})
    assert fb.t == 0 and fb.m.abs().sum() == 0 and fb.v.abs().sum() == 0
