"""Localise a SMAC env kernel vs torch mismatch: replay the parity test's action stream and, at the first step whose
state differs, print the pre-step state of the differing env with every enemy's nearest-ally candidates."""
import torch

from mat_dcml_amd.envs.smac.synthetic import SyntheticSMACEnv

dev = torch.device("cuda")
NAMES = ("apos", "ahp", "epos", "ehp", "perm", "last", "t", "ep_ctr")
for map_name, rao in (("27m_vs_30m", False),):
    E = 24
    hip = SyntheticSMACEnv(E, map_name, device=dev, seed=11, random_agent_order=rao, env_id_offset=5, backend="hip")
    ref = SyntheticSMACEnv(E, map_name, device=dev, seed=11, random_agent_order=rao, env_id_offset=5, backend="torch")
    o1, o2 = hip.reset(), ref.reset()
    g = torch.Generator(device=dev).manual_seed(0)
    ava = o2[2]
    A, N, nA = hip.A, hip.N, hip.n_actions
    for t in range(120):
        pre = {n: getattr(ref, n).clone() for n in NAMES}
        w = ava * torch.where(torch.arange(nA, device=dev) >= 6, 4.0, 1.0)
        act = torch.multinomial(w.reshape(-1, nA), 1, generator=g).view(E, A).float()
        r1, r2 = hip.step(act), ref.step(act)
        ava = r2[5]
        bad = [n for n in NAMES if not torch.equal(getattr(hip, n), getattr(ref, n))]
        if not bad:
            continue
        print("step", t, "differs:", bad)
        d = (hip.ahp != ref.ahp).nonzero().tolist()
        print("ahp mismatches (env, ally, hip, ref):", [(e, i, float(hip.ahp[e, i]), float(ref.ahp[e, i])) for e, i in d[:10]])
        e = d[0][0]
        ap, ep, ah, eh = pre["apos"][e], pre["epos"][e], pre["ahp"][e], pre["ehp"][e]
        a = act[e].long()
        alive = ah > 0
        a = torch.where(alive, a, torch.zeros_like(a))
        dirs = torch.tensor([[0.0, 1.0], [0.0, -1.0], [1.0, 0.0], [-1.0, 0.0]], device=dev)
        mv = (a >= 2) & (a < 6)
        ap2 = (ap + dirs[(a - 2).clamp(0, 3)] * mv.unsqueeze(-1)).clamp(0.0, 32.0)
        print("ally pos hip==ref-moved:", torch.equal(ap2, ref.apos[e]), torch.equal(hip.apos[e], ref.apos[e]))
        for j in range(N):
            dx = ep[j, 0] - ap2[:, 0]
            dy = ep[j, 1] - ap2[:, 1]
            d2 = (dx * dx + dy * dy).masked_fill(~alive, float("inf"))
            m = d2.min()
            ties = (d2 == m).nonzero().flatten().tolist()
            print(f" enemy {j} hp {float(eh[j]):.4f} min d2 {float(m):.6f} ties {ties} "
                  f"dhip {float(hip.ahp[e].sum()):.6f} dref {float(ref.ahp[e].sum()):.6f}")
        print("actions", a.tolist())
        print("ehp hip", hip.ehp[e].tolist())
        print("ehp ref", ref.ehp[e].tolist())
        break
