"""Section cycle breakdown of the fused decoder backward (workgroup 0, thread 0) at the bench minibatch shape.
Run with MAT_DCML_LIBNAME=libmatdcml_tprof.so (built with -DMDL_TRAIN_PROF)."""
import ctypes
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from test_gpu_train import make  # noqa: E402

from mat_dcml_amd.ops import kernels, mat_train  # noqa: E402

NAMES = {11: "head bwd", 8: "mlp bwd (block)", 9: "cross-attn bwd (block)", 10: "self-attn bwd (block)",
         0: " self: proj+LN bwd", 1: " self: wgrad proj", 2: " self: recompute qkv", 3: " self: attn bwd q",
         4: " self: attn bwd kv", 5: " self: wgrad qkv", 6: " self: dx GEMMs",
         7: " cross: proj+LN bwd", 12: " cross: wgrad proj", 13: " cross: recompute qkv", 14: " cross: attn bwd q",
         15: " cross: attn bwd kv", 17: " cross: rep + wgrad qkv"}
dev = torch.device("cuda")
L, B = 33, 3200
m = make(L, dev, seed=2)
g = torch.Generator(device=dev).manual_seed(3)
obs = torch.rand(B, L, 7, device=dev, generator=g)
ava = torch.ones(B, L, 2, device=dev)
actions = (torch.rand(B, L, 1, device=dev, generator=g) < 0.5).float()
actions[:, -1, 0] = torch.rand(B, device=dev, generator=g)
for _ in range(4):
    for p in m.parameters():
        p.grad = torch.zeros_like(p)
    v, lp, ent = mat_train.evaluate_actions(m, obs, actions, ava)
    (lp.sum() + v.sum() + ent.sum()).backward()
torch.cuda.synchronize()
out = (ctypes.c_ulonglong * 32)()
lib = kernels.lib()
lib.mdl_dec_prof_read.argtypes = [ctypes.c_void_p]
assert lib.mdl_dec_prof_read(ctypes.addressof(out)) == 0
tot = out[11] + out[8] + out[9] + out[10]
print(f"dec_bwd workgroup-0 cycles (4 launches): {tot}")
for k in (11, 8, 9, 7, 12, 13, 14, 15, 17, 10, 0, 1, 2, 3, 4, 5, 6):
    print(f"  {NAMES[k]:26s} {out[k]:12d} {100 * out[k] / tot:5.1f}%")

# encoder backward sections (value head, blocks (mlp + self-attention, marks 0-6 inside), embedding)
lib.mdl_enc_prof_read.argtypes = [ctypes.c_void_p]
eo = (ctypes.c_ulonglong * 32)()
assert lib.mdl_enc_prof_read(ctypes.addressof(eo)) == 0
etot = eo[20] + eo[21] + eo[22]
print(f"enc_bwd workgroup-0 cycles (4 launches): {etot}")
for k, n in ((20, "value head bwd"), (21, "blocks (mlp + self-attn)"), (22, "obs embedding bwd"), (0, " self: proj+LN bwd"),
             (1, " self: wgrad proj"), (2, " self: recompute qkv"), (3, " self: attn bwd q"), (4, " self: attn bwd kv"),
             (5, " self: wgrad qkv"), (6, " self: dx GEMMs")):
    print(f"  {n:26s} {eo[k]:12d} {100 * eo[k] / max(etot, 1):5.1f}%")
for k, n in ((23, "  emb: stage LN_obs"), (24, "  emb: pre GEMV"), (25, "  emb: LN/GELU bwd + dW_e acc"),
             (26, "  emb: LN_obs param grads"), (27, "  emb: flush LN0/b_e/W_e"), (29, "  emb: (loop glue)")):
    print(f"  {n:26s} {eo[k]:12d} {100 * eo[k] / max(etot, 1):5.1f}%")
