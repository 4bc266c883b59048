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
