"""Batched planar articulated-body simulator: a MuJoCo-shaped surrogate for the multi-agent MuJoCo tasks.

mujoco-py and the MuJoCo binaries are not installable here, so the reference's MA-MuJoCo robots
(``mat_src/mat/envs/ma_mujoco/multiagent_mujoco/``: gym HalfCheetah / Hopper / Walker2d / Swimmer / Ant / Reacher /
Humanoid(Standup),
``coupled_half_cheetah.py``, ``manyagent_swimmer.py``, ``manyagent_ant.py``) are re-modelled as planar link trees
simulated for E envs at once on the device.  What is kept EXACTLY is the interface the multi-agent layer and the
policy see: the gym ``qpos`` / ``qvel`` layouts (so ``graph.py``'s joint ids index the right entries), the
``_get_obs`` vectors, the action layout (including Ant's actuator order hip4, ankle4, hip1, …), the reward terms
(forward velocity, control cost, healthy / survive bonus) and the termination rules.  The dynamics are a
surrogate — documented, not MuJoCo:

* a floating root (x, z, pitch) — or (x, y, yaw) in a viscous fluid for the swimmers, or a fixed base for the
  Reacher arm — carries the whole mass; every actuated hinge drives one link of a tree hanging off the root;
* forward kinematics for all links at once: absolute angle = root angle + Σ over the link's ancestors of
  (rest + q) — one matmul with the (J, J) ancestor matrix — and link ends likewise;
* ground contact at every link end / torso end: penalty spring-damper normal force + regularised Coulomb
  friction; swimmers feel anisotropic viscous drag on every segment instead;
* external forces act on the root (force + moment about its centre) and on every joint upstream of the contact
  (moment about the joint) — so a foot pushed back against the ground moves the body forward; motor torques of
  root-attached joints react on the root;
* semi-implicit Euler at ``h`` with ``frame_skip`` × (dt / h) sub-steps per env step, velocities clamped.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import torch

PI = math.pi


@dataclass
class Link:
    parent: int            # -1 = root body
    length: float
    rest: float            # rest angle relative to the parent's direction (root: its body x axis)
    attach: tuple = (0.0, 0.0)   # attachment point in the root frame (parent == -1 only)
    mass: float = 1.0
    rng: tuple | None = None     # joint range (radians)
    damping: float = 1.0
    body: int = -1         # body id whose cfrc_ext row receives this link end's contact force
    stiffness: float = 0.0  # spring towards q = 0 (HalfCheetah's joints have them in its XML)


@dataclass
class Model:
    name: str
    kind: str                       # "ground" | "fluid" | "arm"
    layout: str                     # qpos layout: "slide3" | "free" | "swim" | "fixed"
    links: list
    gear: list                      # per actuator
    act_joint: list                 # actuator -> joint (-1: torque on the root angle)
    mass: float
    root_ends: tuple = ((0.0, 0.0), (0.0, 0.0))   # torso segment end points in the root frame
    dt: float = 0.01
    frame_skip: int = 5
    h: float = 0.0025
    z_offset: float = 0.0           # reported root z = z - z_offset (HalfCheetah's rootz is relative)
    init_z: float | None = None     # None: rest pose resting on the ground
    reset_pos: float = 0.1
    reset_vel: float = 0.1
    reset_vel_normal: bool = True
    nbody: int = 0
    armature: float = 0.15
    extra: dict = field(default_factory=dict)


def _cheetah(name="HalfCheetah-v2"):
    L = [Link(-1, 0.29, -PI / 2 - 0.6, (-0.5, 0.0), 1.5, (-0.52, 1.05), 6.0, stiffness=240),
         Link(0, 0.30, 0.9, mass=1.5, rng=(-0.785, 0.785), damping=4.5, stiffness=180),
         Link(1, 0.19, -0.6, mass=1.0, rng=(-0.4, 0.785), damping=3.0, stiffness=120),
         Link(-1, 0.27, -PI / 2 + 0.5, (0.5, 0.0), 1.4, (-1.0, 0.7), 4.5, stiffness=180),
         Link(3, 0.21, -0.7, mass=1.2, rng=(-1.2, 0.87), damping=3.0, stiffness=120),
         Link(4, 0.14, 0.5, mass=0.9, rng=(-0.5, 0.5), damping=1.5, stiffness=60)]
    return Model(name, "ground", "slide3", L, [120, 90, 60, 120, 60, 30], list(range(6)), 14.0,
                 root_ends=((-0.5, 0.0), (0.6, 0.1)), z_offset=0.7, nbody=8)


def _leg(parent_attach, base, mass=(3.9, 2.7, 2.9), damp=1.0):
    return [Link(-1, 0.45, -PI / 2, parent_attach, mass[0], (-2.6, 0.0), damp),
            Link(base, 0.50, 0.0, mass=mass[1], rng=(-2.6, 0.0), damping=damp),
            Link(base + 1, 0.26, PI / 2, mass=mass[2], rng=(-0.785, 0.785), damping=damp)]


def _hopper():
    return Model("Hopper-v2", "ground", "slide3", _leg((0.0, -0.2), 0, (3.9, 2.7, 5.1)), [200, 200, 200],
                 [0, 1, 2], 15.3, root_ends=((0.0, 0.2), (0.0, -0.2)), dt=0.002, frame_skip=4, h=0.002,
                 init_z=1.25, reset_pos=0.005, reset_vel=0.005, reset_vel_normal=False, nbody=5)


def _walker():
    return Model("Walker2d-v2", "ground", "slide3", _leg((0.0, -0.2), 0) + _leg((0.0, -0.2), 3), [100] * 6,
                 list(range(6)), 22.7, root_ends=((0.0, 0.2), (0.0, -0.2)), dt=0.002, frame_skip=4, h=0.002,
                 init_z=1.25, reset_pos=0.005, reset_vel=0.005, reset_vel_normal=False, nbody=8)


def _swimmer(n_segs=3, name="Swimmer-v2", root_actuated=False):
    links = [Link(-1 if i == 0 else i - 1, 1.0, PI if i == 0 else 0.0, (-1.0, 0.0) if i == 0 else (0.0, 0.0),
                  35.0, (-1.745, 1.745) if not root_actuated else None, 0.0) for i in range(n_segs - 1)]
    acts = ([-1] if root_actuated else []) + list(range(n_segs - 1))
    return Model(name, "fluid", "swim", links, [150.0] * len(acts), acts, 35.0 * n_segs,
                 root_ends=((0.0, 0.0), (-1.0, 0.0)), dt=0.01, frame_skip=4, h=0.005, reset_vel_normal=False,
                 armature=12.0, extra={"cn": 40.0, "ct": 2.0})


def _ant_legs(x_front, x_back, s=0, mass=1.0):
    # per segment: front leg (hip, ankle), back leg (hip, ankle); bodies as in the gym XML numbering
    b = 7 * s
    # planar legs need joint springs to carry the body (the 3-D ant stands on splayed legs)
    k = 80.0
    return [Link(-1, 0.28, -PI / 4, (x_front, 0.0), mass, (-0.52, 0.52), 1.0, 2 + b, k),
            Link(4 * s + 0, 0.57, -PI / 3, mass=mass, rng=(-0.35, 0.35), damping=1.0, body=4 + b, stiffness=k),
            Link(-1, 0.28, -3 * PI / 4, (x_back, 0.0), mass, (-0.52, 0.52), 1.0, 5 + b, k),
            Link(4 * s + 2, 0.57, PI / 3, mass=mass, rng=(-0.35, 0.35), damping=1.0, body=7 + b, stiffness=k)]


def _ant():
    # joints in qpos order hip1, ankle1, hip2, ankle2, hip3, ankle3, hip4, ankle4 (front legs 1-2, back 3-4);
    # actuators in the gym XML order hip4, ankle4, hip1, ankle1, hip2, ankle2, hip3, ankle3
    legs = _ant_legs(0.25, 0.25, 0) + _ant_legs(-0.25, -0.25, 0)
    legs[5].parent, legs[7].parent = 4, 6
    legs[1].body, legs[3].body, legs[5].body, legs[7].body = 4, 7, 10, 13
    legs[0].body, legs[2].body, legs[4].body, legs[6].body = 2, 5, 8, 11
    legs[2].rest, legs[3].rest = -PI / 4, -PI / 3
    legs[4].rest, legs[5].rest = -3 * PI / 4, PI / 3
    return Model("Ant-v2", "ground", "free", legs, [40.0] * 8, [6, 7, 0, 1, 2, 3, 4, 5], 8.0,
                 root_ends=((-0.25, 0.0), (0.25, 0.0)), h=0.0025, nbody=14)


def _manyagent_ant(n_segs):
    links, acts = [], []
    for s in range(n_segs):
        x = 0.5 * (n_segs - 1) / 2 - 0.5 * s
        seg = _ant_legs(x + 0.2, x - 0.2, s)
        seg[1].parent, seg[3].parent = 4 * s, 4 * s + 2
        links += seg
        acts += [4 * s + 2, 4 * s + 3, 4 * s + 0, 4 * s + 1]
    half = 0.25 * n_segs
    return Model("manyagent_ant", "ground", "free", links, [40.0] * (4 * n_segs), acts, 6.0 * n_segs,
                 root_ends=((-half, 0.0), (half, 0.0)), h=0.0025, nbody=1 + 7 * n_segs)


def _humanoid(name="Humanoid-v2"):
    # planar biped with the XML's 17 hinge joints in qpos order: abdomen z, y, x (a 3-link waist chain down to
    # the pelvis), right hip x, z, y + knee, left hip x, z, y + knee (legs hang off the waist), right shoulder1,
    # shoulder2 + elbow, left likewise (arms hang off the chest).  Actuators in the XML order abdomen_y,
    # abdomen_z, abdomen_x, … (gear 100, knees 200, arms 25).
    P2 = PI / 2
    L = [Link(-1, 0.12, -P2, (0.0, -0.10), 2.0, (-0.78, 0.78), 5.0, stiffness=20),      # 0 abdomen_z
         Link(0, 0.10, 0.0, mass=2.0, rng=(-1.31, 0.52), damping=5.0, stiffness=10),     # 1 abdomen_y
         Link(1, 0.08, 0.0, mass=2.5, rng=(-0.61, 0.61), damping=5.0, stiffness=10),     # 2 abdomen_x
         Link(2, 0.04, 0.0, mass=1.0, rng=(-0.44, 0.09), damping=5.0),                   # 3 right_hip_x
         Link(3, 0.04, 0.0, mass=1.0, rng=(-1.05, 0.61), damping=5.0),                   # 4 right_hip_z
         Link(4, 0.34, 0.0, mass=4.5, rng=(-1.92, 0.35), damping=5.0),                   # 5 right_hip_y (thigh)
         Link(5, 0.38, 0.0, mass=2.6, rng=(-2.79, 0.03), damping=1.0),                   # 6 right_knee (shin)
         Link(2, 0.04, 0.0, mass=1.0, rng=(-0.44, 0.09), damping=5.0),                   # 7 left_hip_x
         Link(7, 0.04, 0.0, mass=1.0, rng=(-1.05, 0.61), damping=5.0),                   # 8 left_hip_z
         Link(8, 0.34, 0.0, mass=4.5, rng=(-1.92, 0.35), damping=5.0),                   # 9 left_hip_y
         Link(9, 0.38, 0.0, mass=2.6, rng=(-2.79, 0.03), damping=1.0),                   # 10 left_knee
         Link(-1, 0.06, -P2, (0.0, 0.15), 0.5, (-1.48, 1.05), 1.0),                      # 11 right_shoulder1
         Link(11, 0.22, 0.0, mass=1.5, rng=(-1.48, 1.05), damping=1.0),                  # 12 right_shoulder2
         Link(12, 0.25, 0.0, mass=1.2, rng=(-1.57, 0.87), damping=1.0),                  # 13 right_elbow
         Link(-1, 0.06, -P2, (0.0, 0.15), 0.5, (-1.05, 1.48), 1.0),                      # 14 left_shoulder1
         Link(14, 0.22, 0.0, mass=1.5, rng=(-1.05, 1.48), damping=1.0),                  # 15 left_shoulder2
         Link(15, 0.25, 0.0, mass=1.2, rng=(-1.57, 0.87), damping=1.0)]                  # 16 left_elbow
    gear = [100, 100, 100, 100, 100, 300, 200, 100, 100, 300, 200, 25, 25, 25, 25, 25, 25]
    acts = [1, 0] + list(range(2, 17))
    m = Model(name, "ground", "free", L, gear, acts, 40.0, root_ends=((0.0, 0.19), (0.0, -0.10)), dt=0.003,
              frame_skip=5, h=0.0025, init_z=1.4, reset_pos=0.01, reset_vel=0.01, reset_vel_normal=False, nbody=14,
              armature=0.2)
    m.extra["standup"] = name == "HumanoidStandup-v2"
    return m


def _reacher():
    L = [Link(-1, 0.1, 0.0, (0.0, 0.0), 0.05, None, 1.0), Link(0, 0.11, 0.0, mass=0.05, rng=(-3.0, 3.0), damping=1.0)]
    return Model("Reacher-v2", "arm", "fixed", L, [200.0, 200.0], [0, 1], 1.0, dt=0.01, frame_skip=2, h=0.005,
                 armature=1.0, nbody=5)


def make_model(scenario, agent_conf=""):
    if scenario in ("HalfCheetah-v2", "half_cheetah"):
        return _cheetah()
    if scenario == "coupled_half_cheetah":
        m = _cheetah("coupled_half_cheetah")
        m.extra["coupled"] = True
        return m
    if scenario == "Hopper-v2":
        return _hopper()
    if scenario == "Walker2d-v2":
        return _walker()
    if scenario == "Swimmer-v2":
        return _swimmer()
    if scenario == "manyagent_swimmer":
        na, per = (int(x) for x in agent_conf.split("x"))
        return _swimmer(na * per, "manyagent_swimmer", root_actuated=True)
    if scenario == "Ant-v2":
        return _ant()
    if scenario == "manyagent_ant":
        na, per = (int(x) for x in agent_conf.split("x"))
        return _manyagent_ant(na * per)
    if scenario == "Reacher-v2":
        return _reacher()
    if scenario in ("Humanoid-v2", "HumanoidStandup-v2"):
        return _humanoid(scenario)
    raise NotImplementedError(f"no surrogate dynamics for {scenario!r}")


def _cross(a, b):          # planar cross product (…, 2) × (…, 2) -> (…)
    return a[..., 0] * b[..., 1] - a[..., 1] * b[..., 0]


def _rot(th, xy):          # rotate body-frame points xy (P, 2) by th (B,) -> (B, P, 2)
    c, s = torch.cos(th)[:, None], torch.sin(th)[:, None]
    return torch.stack([c * xy[None, :, 0] - s * xy[None, :, 1], s * xy[None, :, 0] + c * xy[None, :, 1]], -1)


class PlanarSim:
    """E independent copies of ``model`` (plus a tendon-coupled twin for coupled_half_cheetah)."""

    def __init__(self, model: Model, n_envs: int, device="cpu", generator=None):
        self.m, self.E, self.dev = model, int(n_envs), torch.device(device)
        self.twins = 2 if model.extra.get("coupled") else 1
        self.B = self.E * self.twins
        self.gen = generator
        J = len(model.links)
        self.J = J
        f = dict(device=self.dev, dtype=torch.float32)
        anc = torch.zeros(J, J, **f)          # anc[l, a] = 1 if a is l or an ancestor of l
        for l in range(J):
            a = l
            while a >= 0:
                anc[l, a] = 1.0
                a = model.links[a].parent
        self.anc = anc
        top = [l if model.links[l].parent < 0 else None for l in range(J)]
        for l in range(J):
            a = l
            while model.links[a].parent >= 0:
                a = model.links[a].parent
            top[l] = a
        self.attach = torch.tensor([model.links[t].attach for t in top], **f).reshape(J, 2)
        self.length = torch.tensor([lk.length for lk in model.links], **f)
        self.rest = torch.tensor([lk.rest for lk in model.links], **f)
        self.damp = torch.tensor([lk.damping for lk in model.links], **f)
        self.stiff = torch.tensor([lk.stiffness for lk in model.links], **f)
        lo = [lk.rng[0] if lk.rng else -1e9 for lk in model.links]
        hi = [lk.rng[1] if lk.rng else 1e9 for lk in model.links]
        self.lo, self.hi = torch.tensor(lo, **f), torch.tensor(hi, **f)
        # subtree mass -> joint inertia; contact points: torso ends (2) then link ends (J)
        msub = anc.t() @ torch.tensor([lk.mass for lk in model.links], **f)
        self.inertia = model.armature + msub * self.length ** 2 / 3.0
        self.root_attached = torch.tensor([lk.parent < 0 for lk in model.links], device=self.dev)
        self.gear = torch.tensor(model.gear, **f)
        nu = len(model.act_joint)
        act_map = torch.zeros(nu, J + 1, **f)   # last column: root-angle torque
        for a, j in enumerate(model.act_joint):
            act_map[a, j if j >= 0 else J] = 1.0
        self.act_map = act_map
        self.root_ends = torch.tensor(model.root_ends, **f)
        ext = max(abs(x) for p in model.root_ends for x in p) + 0.3
        self.root_I = model.mass * (2 * ext) ** 2 / 12.0 if model.kind != "arm" else 1.0
        # (J, P) downstream mask: point p (link end) is below joint j
        self.down = anc.t().contiguous()     # down[j, l] = 1 if j is l or an ancestor of l
        self.body_of_link = [lk.body for lk in model.links]
        self.nsub = max(1, int(round(model.frame_skip * model.dt / model.h)))
        self.dt_env = model.frame_skip * model.dt
        # per-point spring-damper sized for ~half the contact points carrying the body, critically damped
        npts = max(2, (J + 2) // 2)
        w = 40.0
        self.k_contact = model.mass * w * w / npts
        self.c_contact = 2.0 * model.mass * w / npts
        self.mu = 0.9
        self.gravity = torch.tensor([0.0, -9.81 * model.mass], **f)
        # launch-bound inner loop (nsub sub-steps x ~50 small kernels): captured once into a hipGraph on GPU
        self.use_graph = self.dev.type == "cuda" and os.environ.get("MAT_DCML_ENV_GRAPHS", "1") != "0"
        self._graph = None
        # one-launch fused step (csrc/planar_sim.hip) on GPU; the tendon-coupled twin model keeps the torch path
        self.use_fused = (self.dev.type == "cuda" and self.twins == 1 and J <= 64
                          and os.environ.get("MAT_DCML_ENV_FUSED", "1") != "0")
        self.target = torch.zeros(self.B, 2, **f)
        self.p = torch.zeros(self.B, 2, **f)
        self.th = torch.zeros(self.B, **f)
        self.v = torch.zeros(self.B, 2, **f)
        self.w = torch.zeros(self.B, **f)
        self.q = torch.zeros(self.B, J, **f)
        self.qd = torch.zeros(self.B, J, **f)
        self.tau = torch.zeros(self.B, J, **f)
        self.f_end = torch.zeros(self.B, J, 2, **f)
        self.f_root = torch.zeros(self.B, 2, **f)
        if model.init_z is None and model.kind == "ground":
            zs = self._fk(torch.zeros(1, 2, **f), torch.zeros(1, **f), torch.zeros(1, J, **f))[0][..., 1]
            rz = _rot(torch.zeros(1, **f), self.root_ends)[..., 1]
            self.z0 = float(-torch.cat([zs, rz], 1).min()) + 0.005
        else:
            self.z0 = float(model.init_z or 0.0)

    # -------------------------------------------------------------------------------- kinematics
    def _fk(self, p, th, q):
        ang = th[:, None] + (self.rest[None] + q) @ self.anc.t()                    # (B, J)
        d = self.length[None, :, None] * torch.stack([torch.cos(ang), torch.sin(ang)], -1)
        base = p[:, None, :] + _rot(th, self.attach)                                 # (B, J, 2)
        end = base + torch.einsum("la,bad->bld", self.anc, d)
        start = end - d
        return end, start, ang, d

    def _point_vel(self, pts, v, w, ang_w, d):
        """velocity of link ends: root velocity + root rotation + Σ ancestors ω_a × d_a"""
        rel = pts - self.p[:, None, :]
        vroot = v[:, None, :] + w[:, None, None] * torch.stack([-rel[..., 1], rel[..., 0]], -1)
        perp = torch.stack([-d[..., 1], d[..., 0]], -1) * ang_w[..., None]          # ω_a × d_a
        return vroot + torch.einsum("la,bad->bld", self.anc, perp)

    # -------------------------------------------------------------------------------- dynamics
    def _forces(self, end, start, ang, d, v_end, ang_w):
        """external forces F (B, P, 2) at points pts (B, P, 2): the root's points first (2 torso ends on the
        ground, 1 torso midpoint in the fluid), then one per link"""
        m = self.m
        B, J = self.B, self.J
        if m.kind == "ground":
            rpts = self.p[:, None, :] + _rot(self.th, self.root_ends)
            rrel = rpts - self.p[:, None, :]
            rvel = self.v[:, None, :] + self.w[:, None, None] * torch.stack([-rrel[..., 1], rrel[..., 0]], -1)
            pts = torch.cat([rpts, end], 1)
            vel = torch.cat([rvel, v_end], 1)
            pen = (-pts[..., 1]).clamp_min(0.0)
            fn = (self.k_contact * pen - self.c_contact * vel[..., 1]).clamp_min(0.0) * (pen > 0)
            ft = -self.mu * fn * torch.tanh(vel[..., 0] / 0.05)
            F = torch.stack([ft, fn], -1)
        elif m.kind == "fluid":
            cn, ct = m.extra["cn"], m.extra["ct"]
            # torso segment (root_ends) + every link segment; force at the midpoint
            r0 = _rot(self.th, self.root_ends)
            tseg = r0[:, 1] - r0[:, 0]
            tmid = self.p + 0.5 * (r0[:, 0] + r0[:, 1])
            rel = tmid - self.p
            tvel = self.v + self.w[:, None] * torch.stack([-rel[:, 1], rel[:, 0]], -1)
            mid = 0.5 * (start + end)
            mvel = v_end - 0.5 * torch.stack([-d[..., 1], d[..., 0]], -1) * ang_w[..., None]
            segs = torch.cat([tseg[:, None], d], 1)
            pts = torch.cat([tmid[:, None], mid], 1)
            vel = torch.cat([tvel[:, None], mvel], 1)
            ln = segs.norm(dim=-1, keepdim=True).clamp_min(1e-6)
            t = segs / ln
            n = torch.stack([-t[..., 1], t[..., 0]], -1)
            vt = (vel * t).sum(-1, keepdim=True)
            vn = (vel * n).sum(-1, keepdim=True)
            F = -(ct * vt * t + cn * vn * n) * ln
        else:
            return None, None
        return pts, F

    def substep(self, tau_motor, tau_root_motor):
        m = self.m
        h = m.h
        end, start, ang, d = self._fk(self.p, self.th, self.q)
        ang_w = self.w[:, None] + self.qd @ self.anc.t()
        v_end = self._point_vel(end, self.v, self.w, ang_w, d)
        tau = tau_motor - self.damp * self.qd - self.stiff * self.q
        tau = tau - 200.0 * ((self.q - self.hi).clamp_min(0) + (self.q - self.lo).clamp_max(0)) * (1 + 0.1 * self.qd.abs())
        if m.kind == "arm":
            self.f_end.zero_()
            qdd = tau / self.inertia
            self.qd = (self.qd + h * qdd).clamp(-50, 50)
            self.q = self.q + h * self.qd
            return
        pts, F = self._forces(end, start, ang, d, v_end, ang_w)
        nr = pts.shape[1] - self.J                                      # root points (2 ground / 1 fluid)
        Fl = F[:, nr:]                                                  # forces at link points (B, J, 2)
        Pl = pts[:, nr:]
        # joint j: moment about its position (start of link j) of every force downstream of it
        cpf = _cross(Pl, Fl)                                            # (B, J)
        Fd = torch.einsum("jl,bld->bjd", self.down, Fl)                 # Σ downstream forces (B, J, 2)
        tau = tau + cpf @ self.down.t() - _cross(start, Fd)
        Ftot = F.sum(1)
        if m.kind == "ground":
            Ftot = Ftot + self.gravity
        rel = pts - self.p[:, None, :]
        tau_root = _cross(rel, F).sum(1) - (tau_motor * self.root_attached).sum(1) + tau_root_motor
        self.f_end = Fl
        self.f_root = F[:, :nr].sum(1)
        self.v = (self.v + h * Ftot / m.mass).clamp(-30, 30)
        self.w = (self.w + h * tau_root / self.root_I).clamp(-40, 40)
        self.qd = (self.qd + h * tau / self.inertia).clamp(-60, 60)
        self.p = self.p + h * self.v
        self.th = self.th + h * self.w
        self.q = self.q + h * self.qd
        self.tau = tau_motor

    _STATE = ("p", "th", "v", "w", "q", "qd", "tau", "f_end", "f_root")

    def step(self, a):
        """a: (E, nu) in [-1, 1] (coupled twin: (E, 2·nu))."""
        a = a.reshape(self.B, -1).float()
        if self.use_fused:
            return self._step_fused(a)
        if not self.use_graph:
            return self._step(a)
        if self._graph is None:
            self._capture(a)
        self._a_in.copy_(a)
        self._graph.replay()

    def _fused_consts(self):
        m = self.m
        parts = [self.anc, self.attach, self.length, self.rest, self.damp, self.stiff, self.lo, self.hi,
                 self.inertia, self.root_attached.float(), self.root_ends, self.gear, self.act_map]
        consts = torch.cat([t.reshape(-1).float() for t in parts]).contiguous()
        kind = {"ground": 0, "fluid": 1, "arm": 2}[m.kind]
        cn, ct = (m.extra["cn"], m.extra["ct"]) if m.kind == "fluid" else (0.0, 0.0)
        return consts, (self.B, self.J, self.root_ends.shape[0], self.act_map.shape[0], self.nsub, kind, m.h, m.mass,
                        self.root_I, self.k_contact, self.c_contact, self.mu, float(self.gravity[1]), cn, ct)

    def _step_fused(self, a):
        from ...ops import kernels
        if getattr(self, "_fconsts", None) is None:
            self._fconsts = self._fused_consts()
        consts, scal = self._fconsts
        for k in self._STATE:                  # state stays in place: the kernel updates it
            t = getattr(self, k)
            if not t.is_contiguous():
                setattr(self, k, t.contiguous())
        kernels.planar_step(consts, scal, a.contiguous(), self.p, self.th, self.v, self.w, self.q, self.qd,
                            self.tau, self.f_end, self.f_root)

    def _capture(self, a):
        """Record one env step (all sub-steps) as a hipGraph whose inputs / outputs are the state buffers."""
        self._a_in = a.clone()
        saved = {k: getattr(self, k).clone() for k in self._STATE}
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):          # warm-up outside capture (allocator / library init)
            self._step(self._a_in)
        torch.cuda.current_stream().wait_stream(side)
        bufs = {k: v.clone() for k, v in saved.items()}
        for k, v in bufs.items():
            setattr(self, k, v)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._step(self._a_in)
            for k in self._STATE:
                bufs[k].copy_(getattr(self, k))
        for k, v in bufs.items():              # the state lives in the graph's input buffers
            setattr(self, k, v)
        self._graph = g

    def _step(self, a):
        a = a.clamp(-1.0, 1.0)
        full = (a * self.gear) @ self.act_map                           # (B, J + 1)
        tau_m, tau_root = full[:, :self.J], full[:, self.J]
        for _ in range(self.nsub):
            t = tau_m
            if self.twins == 2:     # tendon coupling the two back thighs (coupled_half_cheetah.xml)
                k = 50.0
                ql = self.q.view(self.E, 2, self.J)[:, :, 0]
                ten = (ql[:, 0] - ql[:, 1])
                t = tau_m.clone().view(self.E, 2, self.J)
                t[:, 0, 0] -= k * ten
                t[:, 1, 0] += k * ten
                t = t.view(self.B, self.J)
            self.substep(t, tau_root)

    # -------------------------------------------------------------------------------- reset / state
    def _u(self, shape, scale):
        return (torch.rand(shape, generator=self.gen, device=self.dev) * 2 - 1) * scale

    def reset(self, mask=None):
        m = self.m
        B, J = self.B, self.J
        mask = torch.ones(self.E, dtype=torch.bool, device=self.dev) if mask is None else mask
        mk = mask.repeat_interleave(self.twins)
        sel = lambda new, old: old.copy_(torch.where(mk.view(-1, *([1] * (old.dim() - 1))), new, old))
        rp, rv = m.reset_pos, m.reset_vel
        vel = (lambda s: torch.randn(s, generator=self.gen, device=self.dev) * rv) if m.reset_vel_normal else \
            (lambda s: self._u(s, rv))
        p = torch.stack([self._u(B, rp), self.z0 + self._u(B, rp)], -1) if m.kind == "ground" else \
            self._u((B, 2), rp) * (m.kind == "fluid")
        self.p = sel(p, self.p)
        self.th = sel(self._u(B, rp) if m.kind != "arm" else torch.zeros(B, device=self.dev), self.th)
        self.q = sel(self._u((B, J), rp), self.q)
        self.v = sel(vel((B, 2)) if m.kind != "arm" else torch.zeros(B, 2, device=self.dev), self.v)
        self.w = sel(vel(B) if m.kind != "arm" else torch.zeros(B, device=self.dev), self.w)
        self.qd = sel(vel((B, J)), self.qd)
        if m.kind == "ground" and m.init_z is None:
            # lift freshly reset bodies out of the ground (noise on q can push a foot below z = 0)
            zs = self._fk(self.p, self.th, self.q)[0][..., 1]
            rz = (self.p[:, None, :] + _rot(self.th, self.root_ends))[..., 1]
            lift = (0.002 - torch.cat([zs, rz], 1).min(1).values).clamp_min(0.0)
            self.p += torch.stack([torch.zeros_like(lift), lift * mk], -1)
        if m.kind == "arm":
            tgt = self._u((B, 2), 0.2)
            for _ in range(8):     # rejection: ‖goal‖ < 0.2 (reacher.py reset_model)
                bad = tgt.norm(dim=-1) >= 0.2
                tgt = torch.where(bad[:, None], self._u((B, 2), 0.2), tgt)
            self.target = sel(tgt, self.target)
        self.f_end.copy_(torch.where(mk[:, None, None], torch.zeros_like(self.f_end), self.f_end))

    def fingertip(self):
        end = self._fk(self.p, self.th, self.q)[0]
        return end[:, -1]

    def root_x(self):
        return self.p[:, 0].view(self.E, self.twins)
