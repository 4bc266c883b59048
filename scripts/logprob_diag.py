"""Where do the rollout's and the learner's log-probs part ways?  Rolls out with the production decode, then compares
per agent row: decode kernel vs fused training forward vs the fp32 torch teacher-forced log-probs of the SAME actions
(``models/act.parallel_act`` on the fp32 torch encoder's rep).

    python scripts/logprob_diag.py [--ckpt profiles/r5_train32/transformer_500_beta3.pt] [--n_workers 32]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ckpt", default="profiles/r5_train32/transformer_500_beta3.pt")
    ap.add_argument("--n_workers", type=int, default=32)
    ap.add_argument("--envs", type=int, default=256)
    ap.add_argument("--T", type=int, default=4)
    a = ap.parse_args()
    from test_gpu_logprob_consistency import _dcml_runner
    from mat_dcml_amd.models import act
    from mat_dcml_amd.ops import mat_train
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    r = _dcml_runner(dev, a.n_workers, a.envs, a.T)
    if a.ckpt:
        r.policy.restore(a.ckpt)
    m = r.policy.transformer
    print("log_std", m.decoder.log_std.detach().cpu().numpy() if hasattr(m.decoder, "log_std") else None,
          "std", m.action_std().detach().cpu().numpy() if m.action_type != "Discrete" else None)
    r.warmup()
    r.rollout()
    torch.cuda.synchronize()
    b = r.buffer
    obs, act_, ava, old = b.flat("obs"), b.flat("actions"), b.flat("available_actions"), b.flat("action_log_probs")
    enc, dec, _ = mat_train._state(m, dev)
    with torch.no_grad():
        _, rep = enc.forward(obs, save=True)
        new, _ = dec.forward(rep, act_, ava, save=True)
        _, rep32 = m.encoder(None, obs)
        ref, _ = act.parallel_act(m, rep32.float(), obs, act_, ava)
        print("rep: learner vs fp32 max", (rep - rep32).abs().max().item())
    new, ref, old = new.reshape(old.shape), ref.reshape(old.shape).float(), old.float()
    L = old.shape[1]
    print("row | mean|dec-lrn| max | mean|dec-fp32| max | mean|lrn-fp32| max | mean logp")
    for i in list(range(min(L, 4))) + list(range(max(4, L - 4), L)):
        f = lambda x: (x[:, i].abs().mean().item(), x[:, i].abs().max().item())  # noqa: E731
        d1, d2, d3 = f(old - new), f(old - ref), f(new - ref)
        print(f"{i:3d} | {d1[0]:.3e} {d1[1]:.3e} | {d2[0]:.3e} {d2[1]:.3e} | {d3[0]:.3e} {d3[1]:.3e} | "
              f"{old[:, i].mean().item():.3f}")
    disc = slice(0, L - 1)
    for name, x in (("dec-lrn", old - new), ("dec-fp32", old - ref), ("lrn-fp32", new - ref)):
        print(f"{name}: discrete rows mean {x[:, disc].abs().mean().item():.3e} max {x[:, disc].abs().max().item():.3e}; "
              f"last row mean {x[:, -1].abs().mean().item():.3e} max {x[:, -1].abs().max().item():.3e}")
    # the worst discrete entries: logp values of both paths
    x = (old - new)[:, disc].abs().flatten()
    idx = x.topk(5).indices
    print("worst discrete: dec", old[:, disc].flatten()[idx].tolist(), "lrn", new[:, disc].flatten()[idx].tolist(),
          "fp32", ref[:, disc].flatten()[idx].tolist())


if __name__ == "__main__":
    main()
