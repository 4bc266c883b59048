"""Multi-agent MuJoCo partition graphs: which joints each agent controls and what it observes (k-hop).

Behaviour of the reference's ``obsk.py`` (``mat_src/mat/envs/ma_mujoco/multiagent_mujoco/obsk.py``):

* a robot is a hyper-graph over its actuated joints (``Node`` ``:5-21``, ``HyperEdge`` ``:24-35``);
* ``parts_and_edges(scenario, conf)`` gives the agent partition, the edges and the global joints / bodies
  (``get_parts_and_edges`` ``:250-657``: HalfCheetah 2x3 / 6x1, Ant 2x4 / 2x4d / 4x2 / 8x1, Hopper 3x1,
  Humanoid(Standup) 9|8 / 17x1, Reacher 2x1, Swimmer 2x1, Walker2d 2x3 / 6x1, coupled_half_cheetah 1p1,
  manyagent_swimmer NxM, manyagent_ant NxM);
* ``joints_at_kdist`` = BFS over hyper-edges from an agent's joints (``:38-71``);
* ``build_obs`` concatenates, per hop k, the categories of ``k_categories[k]`` of every joint at that hop, then the
  global categories of the global joints / bodies, zero-padded to ``vec_len`` (``:138-242``).

Here the scenario tables are data (``_SPECS``) and ``build_obs`` works on BATCHED simulator data — ``data.qpos``
(E, nq), ``data.qvel`` (E, nv), ``data.qfrc_actuator`` (E, nv), ``data.cfrc_ext`` / ``cvel`` / ``cinert``
(E, nbody, ·) — returning one (E, n) tensor for all envs at once.  Reference behaviours kept on purpose (checked
by ``tests/test_mujoco.py`` against the reference module):

* body categories (``cvel``, ``cinert``, ``cfrc_ext``) of LOCAL joints are visited but never appended (the append
  is commented out, ``:190``), and ``cfrc_ext`` extra-obs of GLOBAL joints is skipped (``:203``);
* manyagent_ant's qpos ids wrap into the free joint for all but the last segment (the table is marked
  ``TODO: FIX!`` upstream, ``:588``) — reproduced, since it defines the observation layout;
* global BODIES of a non-body category (Reacher's ``qpos`` over bodies 0 and 4) make the reference raise
  (``float.tolist()`` is not iterable); here they contribute nothing.
"""
from __future__ import annotations

import torch

BODY_CATS = ("cvel", "cinert", "cfrc_ext")


class Node:
    """One actuated (or global) joint: qpos / qvel index, actuator index, bodies, per-category overrides."""

    def __init__(self, label, qpos_ids, qvel_ids, act_ids, bodies=None, clip_bodies=False, extra_obs=None,
                 tendons=None):
        self.label = label
        self.qpos_ids, self.qvel_ids, self.act_ids = qpos_ids, qvel_ids, act_ids
        self.bodies = bodies
        self.clip_bodies = clip_bodies
        self.extra_obs = extra_obs or {}
        self.tendons = tendons

    def __repr__(self):
        return self.label


class HyperEdge:
    def __init__(self, *nodes):
        self.edges = set(nodes)

    def __contains__(self, n):
        return n in self.edges

    def __repr__(self):
        return f"HyperEdge({sorted(n.label for n in self.edges)})"


def joints_at_kdist(agent_id, parts, edges, k=0):
    """{hop: [joints at exactly that hop, sorted by label]} for hops 0..k."""
    seen, frontier, out = set(), set(parts[agent_id]), {}
    for hop in range(k + 1):
        if hop:
            nxt = set()
            for n in frontier:
                for e in edges:
                    if n in e:
                        nxt |= e.edges - {n}
            frontier = nxt - seen
        seen |= frontier
        out[hop] = sorted(frontier, key=lambda n: n.label)
    return out


# ------------------------------------------------------------------------------------------ scenario tables
def _clipv(i, lo=-10.0, hi=10.0):
    return lambda d: d.qvel[:, i:i + 1 if i != -1 else None].clamp(lo, hi)


def _chain(labels, first_q, edges_idx):
    nodes = [Node(lab, first_q + i, first_q + i, a) for i, (lab, a) in enumerate(labels)]
    return nodes, [HyperEdge(*(nodes[i] for i in e)) for e in edges_idx]


def _root3(extra_x=None, extra_z=None, extra_y=None):
    empty = lambda d: d.qpos[:, :0]
    return [Node("root_x", 0, 0, -1, extra_obs={"qpos": empty, **(extra_x or {})}),
            Node("root_y", 2, 2, -1, extra_obs=extra_y), Node("root_z", 1, 1, -1, extra_obs=extra_z)]


def _free_joint():
    return Node("free", 0, 0, -1, extra_obs={"qpos": lambda d: d.qpos[:, :7], "qvel": lambda d: d.qvel[:, :6],
                                             "cfrc_ext": lambda d: d.cfrc_ext[:, 0:1].reshape(d.E, -1).clamp(-1, 1)})


def _half_cheetah(conf):
    # (label, actuator) for qpos -6..-1
    n, e = _chain([("bthigh", 0), ("bshin", 1), ("bfoot", 2), ("fthigh", 3), ("fshin", 4), ("ffoot", 5)], -6,
                  [(2, 1), (1, 0), (0, 3), (3, 4), (4, 5)])
    bt, bs, bf, ft, fs, ff = n
    parts = {"2x3": [(bf, bs, bt), (ff, fs, ft)], "6x1": [(bf,), (bs,), (bt,), (ff,), (fs,), (ft,)]}[conf]
    return parts, e, {"joints": _root3()}


def _ant(conf):
    legs = [("hip1", 2, [1, 2]), ("ankle1", 3, [2, 3, 4]), ("hip2", 4, [1, 5]), ("ankle2", 5, [5, 6, 7]),
            ("hip3", 6, [1, 8]), ("ankle3", 7, [8, 9, 10]), ("hip4", 0, [1, 11]), ("ankle4", 1, [11, 12, 13])]
    n = [Node(lab, -8 + i, -8 + i, a, bodies=b, clip_bodies=True) for i, (lab, a, b) in enumerate(legs)]
    h1, a1, h2, a2, h3, a3, h4, a4 = n
    e = [HyperEdge(a4, h4), HyperEdge(a1, h1), HyperEdge(a2, h2), HyperEdge(a3, h3), HyperEdge(h4, h1, h2, h3)]
    parts = {"2x4": [(h1, a1, h2, a2), (h3, a3, h4, a4)], "2x4d": [(h1, a1, h3, a3), (h2, a2, h4, a4)],
             "4x2": [(h1, a1), (h2, a2), (h3, a3), (h4, a4)],
             "8x1": [(h1,), (a1,), (h2,), (a2,), (h3,), (a3,), (h4,), (a4,)]}[conf]
    return parts, e, {"joints": [_free_joint()]}


def _hopper(conf):
    n = [Node(lab, -3 + i, -3 + i, i, extra_obs={"qvel": _clipv(-3 + i)})
         for i, lab in enumerate(("thigh_joint", "leg_joint", "foot_joint"))]
    th, lg, ft = n
    e = [HyperEdge(ft, lg), HyperEdge(lg, th)]
    if conf != "3x1":
        raise ValueError(f"UNKNOWN partitioning config: {conf}")
    g = _root3(extra_x={"qvel": _clipv(1)}, extra_z={"qvel": _clipv(1)}, extra_y={"qvel": _clipv(2)})
    return [(th,), (lg,), (ft,)], e, {"joints": g}


_HUMANOID = [("abdomen_y", -16), ("abdomen_z", -17), ("abdomen_x", -15), ("right_hip_x", -14),
             ("right_hip_z", -13), ("right_hip_y", -12), ("right_knee", -11), ("left_hip_x", -10),
             ("left_hip_z", -9), ("left_hip_y", -8), ("left_knee", -7), ("right_shoulder1", -6),
             ("right_shoulder2", -5), ("right_elbow", -4), ("left_shoulder1", -3), ("left_shoulder2", -2),
             ("left_elbow", -1)]


def _humanoid(conf):
    J = {lab: Node(lab, q, q, a) for a, (lab, q) in enumerate(_HUMANOID)}
    ab = [J["abdomen_x"], J["abdomen_y"], J["abdomen_z"]]
    rh = [J["right_hip_x"], J["right_hip_y"], J["right_hip_z"]]
    lh = [J["left_hip_x"], J["left_hip_y"], J["left_hip_z"]]
    ls, rs = [J["left_shoulder1"], J["left_shoulder2"]], [J["right_shoulder1"], J["right_shoulder2"]]
    e = [HyperEdge(*ab), HyperEdge(*rh), HyperEdge(*lh), HyperEdge(J["left_elbow"], *ls),
         HyperEdge(J["right_elbow"], *rs), HyperEdge(J["left_knee"], *lh), HyperEdge(J["right_knee"], *rh),
         HyperEdge(*ls, *ab), HyperEdge(*rs, *ab), HyperEdge(*ab, *lh), HyperEdge(*ab, *rh)]
    upper = ("left_shoulder1", "left_shoulder2", "abdomen_x", "abdomen_y", "abdomen_z", "right_shoulder1",
             "right_shoulder2", "right_elbow", "left_elbow")
    lower = ("left_hip_x", "left_hip_y", "left_hip_z", "right_hip_x", "right_hip_y", "right_hip_z", "right_knee",
             "left_knee")
    if conf == "9|8":
        parts = [tuple(J[x] for x in upper), tuple(J[x] for x in lower)]
    elif conf == "17x1":
        parts = [(J[x],) for x in upper + lower]
    else:
        raise ValueError(f"UNKNOWN partitioning config: {conf}")
    return parts, e, {}


def _reacher(conf):
    sincos = lambda i: (lambda d: torch.stack([torch.sin(d.qpos[:, i]), torch.cos(d.qpos[:, i])], -1))
    j0 = Node("joint0", -4, -4, 0, bodies=[1, 2], extra_obs={"qpos": sincos(-4)})
    j1 = Node("joint1", -3, -3, 1, bodies=[2, 3], extra_obs={"fingertip_dist": lambda d: d.fingertip_dist(),
                                                             "qpos": sincos(-3)})
    none = lambda d: d.qvel[:, :0]
    g = {"bodies": [0, 4], "joints": [Node("target_x", -2, -2, -1, extra_obs={"qvel": none}),
                                      Node("target_y", -1, -1, -1, extra_obs={"qvel": none})]}
    if conf != "2x1":
        raise ValueError(f"UNKNOWN partitioning config: {conf}")
    return [(j0,), (j1,)], [HyperEdge(j0, j1)], g


def _swimmer(conf):
    j0, j1 = Node("rot2", -2, -2, 0), Node("rot3", -1, -1, 1)
    if conf != "2x1":
        raise ValueError(f"UNKNOWN partitioning config: {conf}")
    return [(j0,), (j1,)], [HyperEdge(j0, j1)], {}


def _walker(conf):
    n, e = _chain([("thigh_joint", 0), ("leg_joint", 1), ("foot_joint", 2), ("thigh_left_joint", 3),
                   ("leg_left_joint", 4), ("foot_left_joint", 5)], -6, [(2, 1), (1, 0), (5, 4), (4, 3), (0, 3)])
    th, lg, ft, thl, lgl, ftl = n
    parts = {"2x3": [(ft, lg, th), (ftl, lgl, thl)], "6x1": [(ft,), (lg,), (th,), (ftl,), (lgl,), (thl,)]}[conf]
    return parts, e, {}


def _coupled_half_cheetah(conf):
    ten = {"ten_J": lambda d: d.ten_J[:, 0], "ten_length": lambda d: d.ten_length,
           "ten_velocity": lambda d: d.ten_velocity}
    names = ("bthigh", "bshin", "bfoot", "fthigh", "fshin", "ffoot")
    a = [Node(lab, -6 + i, -6 + i, i, tendons=[0] if i == 0 else None, extra_obs=ten if i == 0 else None)
         for i, lab in enumerate(names)]
    b = [Node(lab + "2", -6 + i, -6 + i, i, tendons=[0] if i == 0 else None, extra_obs=ten if i == 0 else None)
         for i, lab in enumerate(names)]
    ch = [(2, 1), (1, 0), (0, 3), (3, 4), (4, 5)]
    e = [HyperEdge(a[i], a[j]) for i, j in ch] + [HyperEdge(b[i], b[j]) for i, j in ch]
    if conf != "1p1":
        raise ValueError(f"UNKNOWN partitioning config: {conf}")
    order = (2, 1, 0, 5, 4, 3)
    return [tuple(a[i] for i in order), tuple(b[i] for i in order)], e, {"joints": _root3()}


def _nxm(conf):
    try:
        na, per = (int(x) for x in conf.split("x"))
    except Exception:   # noqa: BLE001
        raise ValueError(f"UNKNOWN partitioning config: {conf}")
    return na, per, na * per


def _manyagent_swimmer(conf):
    na, per, ns = _nxm(conf)
    j = [Node(f"rot{i:d}", -ns + i, -ns + i, i) for i in range(ns)]
    return ([tuple(j[i * per:(i + 1) * per]) for i in range(na)], [HyperEdge(j[i], j[i + 1]) for i in range(ns - 1)],
            {})


def _manyagent_ant(conf):
    na, per, ns = _nxm(conf)
    edges, segs, prev = [], [], None
    for s in range(ns):
        off = -4 * (ns - 1 - s)
        b = 7 * s
        h1 = Node(f"hip1_{s:d}", -4 - off, -4 - off, 2 + 4 * s, bodies=[1 + b, 2 + b], clip_bodies=True)
        a1 = Node(f"ankle1_{s:d}", -3 - off, -3 - off, 3 + 4 * s, bodies=[2 + b, 3 + b, 4 + b], clip_bodies=True)
        h2 = Node(f"hip2_{s:d}", -2 - off, -2 - off, 0 + 4 * s, bodies=[1 + b, 5 + b], clip_bodies=True)
        a2 = Node(f"ankle2_{s:d}", -1 - off, -1 - off, 1 + 4 * s, bodies=[5 + b, 6 + b, 7 + b], clip_bodies=True)
        edges += [HyperEdge(a1, h1), HyperEdge(a2, h2), HyperEdge(h1, h2)]
        if prev is not None:
            # the reference links deep copies of the previous segment's hips (distinct objects), so the
            # inter-segment edge never matches a real joint during the BFS; mirrored with fresh nodes
            edges.append(HyperEdge(Node(prev[0].label, prev[0].qpos_ids, prev[0].qvel_ids, prev[0].act_ids),
                                   Node(prev[1].label, prev[1].qpos_ids, prev[1].qvel_ids, prev[1].act_ids), h1, h2))
        prev = (h1, h2)
        segs.append([h1, a1, h2, a2])
    parts = [[x for seg in segs[i * per:(i + 1) * per] for x in seg] for i in range(na)]
    return parts, edges, {"joints": [_free_joint()]}


_SPECS = {
    "half_cheetah": _half_cheetah, "HalfCheetah-v2": _half_cheetah, "Ant-v2": _ant, "Hopper-v2": _hopper,
    "Humanoid-v2": _humanoid, "HumanoidStandup-v2": _humanoid, "Reacher-v2": _reacher, "Swimmer-v2": _swimmer,
    "Walker2d-v2": _walker, "coupled_half_cheetah": _coupled_half_cheetah, "manyagent_swimmer": _manyagent_swimmer,
    "manyagent_ant": _manyagent_ant,
}

DEFAULT_K_CATEGORIES = {   # mujoco_multi.py:60-70
    "Ant-v2": "qpos,qvel,cfrc_ext|qpos", "manyagent_ant": "qpos,qvel,cfrc_ext|qpos",
    "Humanoid-v2": "qpos,qvel,cfrc_ext,cvel,cinert,qfrc_actuator|qpos",
    "HumanoidStandup-v2": "qpos,qvel,cfrc_ext,cvel,cinert,qfrc_actuator|qpos",
    "Reacher-v2": "qpos,qvel,fingertip_dist|qpos", "coupled_half_cheetah": "qpos,qvel,ten_J,ten_length,ten_velocity|",
}


def parts_and_edges(scenario, conf):
    if scenario not in _SPECS:
        raise ValueError(f"unknown MuJoCo scenario {scenario!r}; have {sorted(_SPECS)}")
    try:
        return _SPECS[scenario](conf)
    except KeyError:
        raise ValueError(f"UNKNOWN partitioning config: {conf}") from None


def k_categories(scenario, k, label=None):
    label = label or DEFAULT_K_CATEGORIES.get(scenario, "qpos,qvel|qpos")
    split = label.split("|")
    return [split[h if h < len(split) else -1].split(",") for h in range(k + 1)]


# ------------------------------------------------------------------------------------------ observation
def _joint_items(data, node, c, is_global):
    """(E, n) tensor for category ``c`` of joint ``node`` (None when the category contributes nothing)."""
    if c in node.extra_obs:
        if is_global and c == "cfrc_ext":
            return None
        v = node.extra_obs[c](data)
        return v.reshape(data.E, -1)
    if c in ("qvel", "qpos"):
        idx = getattr(node, f"{c}_ids")
        return getattr(data, c)[:, idx].reshape(data.E, -1)
    if c == "qfrc_actuator":
        return data.qfrc_actuator[:, node.qvel_ids].reshape(data.E, -1)
    return None    # body categories of joints are never appended (obsk.py:180-191, 213-224)


def build_obs(data, k_dict, k_cats, global_dict, global_cats, vec_len=None):
    out = []
    for hop in sorted(k_dict):
        for n in k_dict[hop]:
            for c in k_cats[hop]:
                v = _joint_items(data, n, c, False)
                if v is not None:
                    out.append(v)
    for c in global_cats:
        for j in global_dict.get("joints", []):
            v = _joint_items(data, j, c, True)
            if v is not None:
                out.append(v)
        if c in BODY_CATS:
            for b in dict.fromkeys(global_dict.get("bodies", [])):
                out.append(getattr(data, c)[:, b].reshape(data.E, -1))
    x = torch.cat(out, -1) if out else data.qpos[:, :0]
    if vec_len is not None and x.shape[1] < vec_len:
        x = torch.nn.functional.pad(x, (0, vec_len - x.shape[1]))
    return x


def n_actions(parts):
    return max(len(p) for p in parts)
