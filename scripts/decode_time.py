"""hipEvent time per env step of the default rollout decode path at the bench shapes (for A/B of library variants /
MAT_DCML_* settings):  python scripts/decode_time.py [L,nb,A,B ...]   (default: the DCML 32 / 100 / 128 and SMAC
rollout shapes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from test_gpu_decode import inputs, make  # noqa: E402

from mat_dcml_amd.ops import mat_fused  # noqa: E402


def main():
    shapes = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]] or \
        [(33, 2, 2, 256), (101, 2, 2, 256), (129, 2, 2, 256), (27, 2, 36, 32)]
    dev = torch.device("cuda:0")
    for L, nb, A, B in shapes:
        m = make(L, dev, nb=nb, A=A, atype="Discrete" if A > 2 else "Semi_Discrete")
        obs, ava, rep, _ = inputs(m, B, L, dev, A=A)
        for _ in range(3):
            mat_fused.decode(m, rep, ava, False, 1, None)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(30):
            mat_fused.decode(m, rep, ava, False, 1, None)
        e.record()
        torch.cuda.synchronize()
        print(f"[decode] {B}x{L} nb{nb} A{A} {m._mdl_decode_path:28s} {s.elapsed_time(e) / 30 * 1e3:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
