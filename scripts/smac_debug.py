"""Localise a SMAC env kernel vs torch mismatch: first differing (env, row, feature) of obs / state / ava."""
import torch

from mat_dcml_amd.envs.smac.synthetic import SyntheticSMACEnv

dev = torch.device("cuda")
for map_name, rao in (("27m_vs_30m", False), ("3m", False)):
    hip = SyntheticSMACEnv(4, map_name, device=dev, seed=11, random_agent_order=rao, env_id_offset=5, backend="hip")
    ref = SyntheticSMACEnv(4, map_name, device=dev, seed=11, random_agent_order=rao, env_id_offset=5, backend="torch")
    o1, o2 = hip.reset(), ref.reset()
    print(map_name, "state equal:", {n: bool(torch.equal(getattr(hip, n), getattr(ref, n))) for n in
                                     ("apos", "ahp", "epos", "ehp", "perm", "last", "t", "ep_ctr")})
    for nm in ("apos", "epos"):
        a, b = getattr(hip, nm), getattr(ref, nm)
        d = (a != b).nonzero()
        print(f" {nm}: {len(d)} mismatches", [(tuple(i), float(a[tuple(i)]), float(b[tuple(i)])) for i in d[:6].tolist()])
    for name, a, b in zip(("obs", "state", "ava"), o1, o2):
        d = (a != b).nonzero()
        print(f" {name}: {len(d)} mismatches of {a.numel()}")
        for idx in d[:8].tolist():
            print("   ", idx, float(a[tuple(idx)]), float(b[tuple(idx)]))
