"""Host-side checks of the private gradient workspace layout (round 6, csrc/mat_train_common.h GradMode): the 64 x 64
weight gradients sit in each workgroup's copy in MFMA fragment order (csrc/mat_train_ct.h frag_slot with the 8-wave
block mapping wg_ct), and ``ops/mat_train._fragment_dst`` must send every copy element back to its row-major place —
a wrong map silently scrambles gradients (the GPU tests would only see it as a large numeric error)."""
import torch

from mat_dcml_amd.models.mat import MultiAgentTransformer
from mat_dcml_amd.ops import mat_train
from mat_dcml_amd.ops.ppo_fused import padded, param_offsets


def _flat_grads(m):
    lay = param_offsets(m)
    n = lay[-1][1] + padded(lay[-1][0].numel())
    flat = torch.zeros(n)
    for p, off in lay:
        p.grad = flat[off:off + p.numel()].view_as(p)
    return flat


def _device_slot(wave, lane, j, r):
    """frag_slot(dW, wave, lane, j) + r and the (row, col) the MFMA C register holds (8-wave mapping: row block
    wave & 3, adjacent column tiles 2 (wave >> 2) + j; lane (g, c) = rows 4g + r of column c)."""
    row = 16 * (wave & 3) + 4 * (lane >> 4) + r
    col = 16 * (2 * (wave >> 2) + j) + (lane & 15)
    return wave * 512 + lane * 8 + 4 * j + r, row, col


def test_fragment_dst_is_a_permutation_that_restores_row_major():
    torch.manual_seed(0)
    m = MultiAgentTransformer(34, 7, 2, 33, 2, 64, 2, action_type="Semi_Discrete", semi_index=-1)
    flat = _flat_grads(m)
    dst = mat_train._fragment_dst(m, flat).long()
    n = flat.numel()
    assert torch.equal(dst.sort().values, torch.arange(n)), "dst must be a permutation of the flat gradient"
    lins = mat_train.decoder_linears(m) + mat_train.encoder_linears(m)
    mats = [lin.weight for lin in lins if lin.weight.numel() == 4096]
    assert len(mats) == 34   # 2 x 10 decoder + 2 x 6 encoder block linears + the two heads' W_h1
    # a private copy written the way the kernels write it: each matrix's values at their fragment slots
    copy = torch.arange(n, dtype=torch.float32) * 1e-3   # non-matrix entries: identity
    want = copy.clone()
    g = torch.Generator().manual_seed(1)
    for w in mats:
        o = (w.grad.data_ptr() - flat.data_ptr()) // 4
        G = torch.randn(64, 64, generator=g)
        want[o:o + 4096] = G.reshape(-1)
        for wave in range(8):
            for lane in range(64):
                for j in range(2):
                    for r in range(4):
                        s, row, col = _device_slot(wave, lane, j, r)
                        copy[o + s] = G[row, col]
    # grad_reduce_priv: g[dst[s]] = sum over copies of ws[k][s]
    out = torch.empty(n)
    out[dst] = copy
    assert torch.equal(out, want)
