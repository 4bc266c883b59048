"""Micro-benchmark of the persistent decode kernel on the rollout shape (256 envs x 33 agents) over envs-per-WG caps."""
import os
import subprocess
import sys
import time

import torch

sys.path.insert(0, "/root/repo/tests")
sys.path.insert(0, "/root/repo")


def run(B=256, L=33, iters=20):
    from test_gpu_train import make
    from mat_dcml_amd.ops import mat_fused
    dev = torch.device("cuda")
    m = make(L, dev, seed=0, scale=0.05)
    obs = torch.rand(B, L, 7, device=dev)
    ava = torch.ones(B, L, 2, device=dev)
    with torch.no_grad():
        for _ in range(3):
            mat_fused.get_actions(m, obs, ava, False, 1, None)
        torch.cuda.synchronize()
        t = time.time()
        for _ in range(iters):
            mat_fused.get_actions(m, obs, ava, False, 1, None)
        torch.cuda.synchronize()
    return (time.time() - t) / iters * 1e6


if __name__ == "__main__":
    if len(sys.argv) > 1:
        print(f"{run(L=int(sys.argv[1])):.0f}")
        sys.exit(0)
    for L in (33, 101):
        for cap in (16, 8, 4, 2, 1):
            env = dict(os.environ, MAT_DCML_DECODE_EPW=str(cap))
            out = subprocess.run([sys.executable, __file__, str(L)], env=env, capture_output=True, text=True, timeout=120)
            print(f"L={L} epw_cap={cap}: get_actions {out.stdout.strip()} us {out.stderr.strip()[-200:]}", flush=True)
