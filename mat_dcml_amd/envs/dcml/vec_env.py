"""Device-vectorised bid-first DCML environment: E independent envs x W workers as tensors.

Semantics follow the reference single-process env exactly where they define the MDP:

* ``reset`` — ``DCML_BID_FIRST_MA_ENV_SingleProcess.py:157-274``: sample the task (R, C, Pr) (``DCML_Master.py:46-56``),
  the disabled subset (``:199``), per-worker loss probabilities (``:197``), the arrival slot (``:159-161``) and the
  noisy background-load profile each worker bids (``DCML_Worker_TIMESLOT_MultiProcess.py:37-39,114-135``); build
  obs (A,7), share_obs (A,W+2) and availability (A,2) with the reference layout, including the
  "previous worker's 7th feature" carry for disabled workers (``:210-213``).
* ``step`` — ``:57-144`` + ``Worker.process`` (``DCML_Worker_TIMESLOT_MultiProcess.py:46-112``): K = ceil(N*ratio)
  clamped to [1, N]; each worker's job is (ceil(R/K), C); geometric download retries; the timeslot loop with upload
  retries accumulated inside it; delay = K-th order statistic of the selected workers' delays; payment = sum of
  the selected workers' per-slot cumulative price at ceil(delay); the N == 0 standalone branch with the 1.5x
  penalty; done ~ Bernoulli(0.8); every step starts a new task.

Randomness: every draw is Philox keyed by (seed, task counter, global env id, worker, purpose) — see
``utils/philox.py``.  ``while U < Pr: n += 1`` loops become one inverse-CDF geometric draw each (exact in
distribution).  This torch implementation is the CPU path and the oracle for the HIP kernels in
``csrc/dcml_env.hip``, which reproduce it draw-for-draw.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ...utils import philox as px
from .config import DCMLConfig
from .data import load_preset, load_profiles


class DeviceDCMLEnv:
    """Batched DCML env.  All state lives on ``device``; outputs are device tensors."""

    def __init__(self, n_envs: int, cfg: DCMLConfig | None = None, device="cpu", seed: int = 1,
                 env_id_offset: int = 0, fixed: bool = False, preset: bool = False,
                 backend: str = "auto"):
        self.cfg = cfg or DCMLConfig()
        self.E = int(n_envs)
        self.W = self.cfg.n_workers
        self.A = self.cfg.n_agents
        self.P = self.cfg.period
        self.device = torch.device(device)
        self.seed = int(seed)
        self.k0, self.k1 = px.seed_key(seed)
        self.fixed = fixed
        self.preset = preset
        dev = self.device
        self.gid = torch.arange(self.E, device=dev, dtype=torch.int64) + int(env_id_offset)
        self.profiles = torch.tensor(load_profiles(self.cfg), dtype=torch.float32, device=dev)  # (W,P)
        E, W, A, P = self.E, self.W, self.A, self.P
        f32, f64, i64 = torch.float32, torch.float64, torch.int64
        self.counter = torch.zeros(E, dtype=i64, device=dev)      # next task counter
        self.task_ctr = torch.zeros(E, dtype=i64, device=dev)     # counter of the current task
        self.R = torch.zeros(E, dtype=f64, device=dev)
        self.C = torch.zeros(E, dtype=f64, device=dev)
        self.master_pr = torch.zeros(E, dtype=f64, device=dev)
        self.worker_pr = torch.zeros(E, W, dtype=f64, device=dev)
        self.avail = torch.zeros(E, W, dtype=torch.bool, device=dev)
        self.n_disable = torch.zeros(E, dtype=i64, device=dev)
        self.arrive = torch.zeros(E, dtype=i64, device=dev)
        self.lw = torch.zeros(E, W, P, dtype=f32, device=dev)
        self.rate = torch.full((E, W), self.cfg.data_rate, dtype=f64, device=dev)   # download rate per link
        self.up_rate = torch.full((E, W), self.cfg.data_rate, dtype=f64, device=dev)
        self.obs = torch.zeros(E, A, self.cfg.obs_dim, dtype=f32, device=dev)
        self.share = torch.zeros(E, self.cfg.share_dim, dtype=f32, device=dev)
        self.ava = torch.zeros(E, A, 2, dtype=f32, device=dev)
        # preset replay tables (Sample_1 by default)
        self.preset_idx = torch.zeros(E, dtype=i64, device=dev)
        self.preset_start = torch.zeros(E, dtype=i64, device=dev)   # first preset row per env (benchmark sharding)
        if preset:
            m, prs, dis = load_preset(self.cfg)
            self.preset_master = torch.tensor(m, dtype=f64, device=dev)
            self.preset_prs = torch.tensor(prs, dtype=f64, device=dev)
            self.preset_disable = torch.tensor(dis, dtype=i64, device=dev)
        self.backend = backend
        self._kern = None
        if backend in ("auto", "hip") and self.device.type == "cuda":
            from ...ops import kernels
            if kernels.available() or backend == "hip":
                self._kern = kernels.lib()

    # ------------------------------------------------------------------ spaces (reference API shape)
    @property
    def n_agents(self):
        return self.A

    @property
    def observation_space(self):
        return [[self.cfg.obs_dim]] * self.A

    @property
    def share_observation_space(self):
        return [[self.cfg.share_dim]] * self.A

    def modify_preset(self, R=None, C=None, Pr=None, disable_rate=None):
        """``DCML_BID_FIRST_MA_ENV_SingleProcess.py:344-353``."""
        assert self.preset, "modify_preset needs preset=True"
        if R is not None:
            self.preset_master[:, 0] = float(R)
        if C is not None:
            self.preset_master[:, 1] = float(C)
        if disable_rate is not None:
            self.preset_disable[:] = int(disable_rate)
        if Pr is not None:
            self.preset_prs[:] = float(Pr)

    def set_preset_tables(self, master, worker_prs, disable, start):
        """Install stacked preset tables (G sweep points x rows) and each env's first row.

        Used by the benchmark to run every sweep point (and several shards of each point's episode sequence) as
        independent envs of ONE batched env, instead of the reference's one-env-per-point Python loop.
        """
        assert self.preset
        dev = self.device
        self.preset_master = torch.as_tensor(master, dtype=torch.float64, device=dev).contiguous()
        self.preset_prs = torch.as_tensor(worker_prs, dtype=torch.float64, device=dev).contiguous()
        self.preset_disable = torch.as_tensor(disable, dtype=torch.int64, device=dev).contiguous()
        self.preset_start = torch.as_tensor(start, dtype=torch.int64, device=dev).contiguous()

    # ------------------------------------------------------------------ public API
    def reset(self):
        self.counter.zero_()
        self.preset_idx.copy_(self.preset_start)
        self._reset(torch.ones(self.E, dtype=torch.bool, device=self.device))
        return self.obs, self.share_view(), self.ava

    def share_view(self):
        return self.share.unsqueeze(1).expand(self.E, self.A, self.cfg.share_dim)

    def step(self, actions: torch.Tensor):
        """actions: (E, A) or (E, A, 1) float.  Returns obs, share, reward (E,), done (E,), delay (E,), payment (E,), ava."""
        actions = actions.reshape(self.E, self.A).to(torch.float32)
        if self._kern is not None:
            out = self._step_hip(actions)
        else:
            out = self._step_torch(actions)
        self._sync_parent()
        return out

    # ------------------------------------------------------------------ env-range views (pipelined rollouts)
    # per-env state: dim 0 = env.  The step reads / writes only these (plus the shared, read-only tables).
    _PER_ENV = ("gid", "counter", "task_ctr", "R", "C", "master_pr", "worker_pr", "avail", "n_disable", "arrive", "lw",
                "rate", "up_rate", "obs", "share", "ava", "preset_idx", "preset_start")

    def group_views(self, G: int):
        """G envs-range views [g E/G, (g+1) E/G) sharing this env's state, each stepped on its own (the runner's
        two-group pipelined rollout, SURVEY §2.4: one group's env step overlaps the other group's decode).  Every
        draw is keyed by the global env id (``gid``), so stepping the views reproduces stepping the whole env.  The
        HIP step updates the shared storage in place; the torch step rebinds its state tensors, so a view copies
        them back into the parent's rows after each step (``_sync_parent``)."""
        import copy
        assert self.E % G == 0, (self.E, G)
        n = self.E // G
        views = []
        for g in range(G):
            v = copy.copy(self)
            for k in ("_out", "last_debug", "last_near_int"):
                v.__dict__.pop(k, None)
            v._rows = {k: getattr(self, k)[g * n:(g + 1) * n] for k in self._PER_ENV}
            for k, t in v._rows.items():
                setattr(v, k, t)
            v.E = n
            views.append(v)
        return views

    def _sync_parent(self):
        rows = self.__dict__.get("_rows")
        if rows is None:
            return
        for k, t in rows.items():
            cur = getattr(self, k)
            if cur is not t:   # rebound by the torch path: write the new values into the parent's rows
                t.copy_(cur)
                setattr(self, k, t)

    # ------------------------------------------------------------------ reset
    def _reset(self, mask: torch.Tensor):
        """Start a new task for envs where mask is True (torch path)."""
        if self._kern is not None:
            self._reset_hip(mask)
            return
        cfg, E, W, P = self.cfg, self.E, self.W, self.P
        dev = self.device
        ctr = self.counter.clone()
        u = px.philox4x32(ctr, self.gid, 0, px.P_MASTER, self.k0, self.k1)
        R = cfg.r_min + torch.floor(px.u01_open(u[0]) * (cfg.r_hi - cfg.r_min + 1))
        C = cfg.c_min + torch.floor(px.u01_open(u[1]) * (cfg.c_hi - cfg.c_min + 1))
        mpr = cfg.pr_min + px.u01_open(u[2]) * (cfg.pr_max - cfg.pr_min)
        dis = 1 + torch.floor(px.u01_open(u[3]) * cfg.max_disable).to(torch.int64)
        ua = px.philox4x32(ctr, self.gid, 0, px.P_ARRIVE, self.k0, self.k1)
        arrive = torch.floor(px.u01_open(ua[0]) * P).to(torch.int64)
        wi = torch.arange(W, device=dev, dtype=torch.int64).view(1, W)
        uw = px.philox4x32(ctr.view(E, 1), self.gid.view(E, 1), wi, px.P_WORKER_PR, self.k0, self.k1)
        wpr = cfg.pr_min + px.u01_open(uw[0]) * (cfg.pr_max - cfg.pr_min)
        key = uw[1]
        if self.preset:
            idx = self.preset_idx.clamp(max=self.preset_master.shape[0] - 1)
            R = self.preset_master[idx, 0].clone()
            C = self.preset_master[idx, 1].clone()
            mpr = self.preset_master[idx, 2].clone()
            wpr = self.preset_prs[idx].clone()
            dis = self.preset_disable[idx].clone()
        if cfg.shannon:
            rate_dn, rate_up = self._shannon_rates(ctr, wi)
            mpr = torch.zeros_like(mpr)                        # DCML_Master.reset: Pr = 0 under Shannon
        dis = dis.clamp(0, W - 1)
        # disabled subset = the `dis` workers with the smallest random keys (ties by index)
        kk = key.view(E, W, 1)
        kv = key.view(E, 1, W)
        vi = wi.view(1, 1, W)
        wv = wi.view(1, W, 1)
        rank = ((kv < kk) | ((kv == kk) & (vi < wv))).sum(-1)
        avail = rank >= dis.view(E, 1)
        # noisy bid profile: clip(profile * U(0.8, 1.2), 0, 1) in float32
        noise = []
        for k in range((P + 3) // 4):
            un = px.philox4x32(ctr.view(E, 1), self.gid.view(E, 1), wi + (k << 16), px.P_NOISE, self.k0, self.k1)
            noise.extend(un)
        noise = torch.stack(noise[:P], -1)  # (E, W, P) uint32
        nf = ((noise >> 8).to(torch.float32) + 0.5) * (1.0 / 16777216.0)
        nf = nf * 0.4 + 0.8
        lw = torch.clamp(self.profiles.view(1, W, P) * nf, 0.0, 1.0)
        m = mask
        self.task_ctr = torch.where(m, ctr, self.task_ctr)
        self.counter = torch.where(m, ctr + 1, self.counter)
        self.preset_idx = torch.where(m, self.preset_idx + 1, self.preset_idx)
        self.R = torch.where(m, R, self.R)
        self.C = torch.where(m, C, self.C)
        self.master_pr = torch.where(m, mpr, self.master_pr)
        self.n_disable = torch.where(m, dis, self.n_disable)
        self.arrive = torch.where(m, arrive, self.arrive)
        m2 = m.view(E, 1)
        self.worker_pr = torch.where(m2, wpr, self.worker_pr)
        self.avail = torch.where(m2, avail, self.avail)
        self.lw = torch.where(m.view(E, 1, 1), lw, self.lw)
        if cfg.shannon:
            self.rate = torch.where(m2, rate_dn, self.rate)
            self.up_rate = torch.where(m2, rate_up, self.up_rate)
        self._build_obs()

    def _shannon_rates(self, ctr, wi):
        """Shannon-capacity links (``Shannon.py:14-21``, ``DCML_Master.get_transmission_rate`` ``:41-45``):
        rate = B log2(1 + P d^-4 / noise) with B = B_total / W, master power ~ U(50,60) per task, worker power
        ~ U(10,20) and distance ~ U(10,100) per worker.  Returns (download, upload) in bytes/s."""
        cfg, E = self.cfg, self.E
        us = px.philox4x32(ctr.view(E, 1), self.gid.view(E, 1), wi, px.P_SHANNON, self.k0, self.k1)
        dist = cfg.distance[0] + px.u01_open(us[0]) * (cfg.distance[1] - cfg.distance[0])
        wpow = cfg.worker_power[0] + px.u01_open(us[1]) * (cfg.worker_power[1] - cfg.worker_power[0])
        um = px.philox4x32(ctr, self.gid, 0xFFFF, px.P_SHANNON, self.k0, self.k1)
        mpow = (cfg.master_power[0] + px.u01_open(um[0]) * (cfg.master_power[1] - cfg.master_power[0])).view(E, 1)
        band = cfg.bandwidth_total / self.W
        noise = 10.0 ** (cfg.noise_dbm / 10.0)
        gain = torch.pow(dist, cfg.path_loss_exp) / noise
        return band * torch.log2(1.0 + mpow * gain), band * torch.log2(1.0 + wpow * gain)

    def _build_obs(self):
        cfg, E, W, P = self.cfg, self.E, self.W, self.P
        dev = self.device
        Rn = ((self.R - cfg.r_min) / (cfg.r_max - cfg.r_min)).to(torch.float32)
        Cn = ((self.C - cfg.c_min) / (cfg.c_max - cfg.c_min)).to(torch.float32)
        t = self.arrive.view(E, 1)
        lw0 = torch.gather(self.lw, 2, t.view(E, 1, 1).expand(E, W, 1)).squeeze(-1)
        lw1 = torch.gather(self.lw, 2, ((t + 1) % P).view(E, 1, 1).expand(E, W, 1)).squeeze(-1)
        lw2 = torch.gather(self.lw, 2, ((t + 2) % P).view(E, 1, 1).expand(E, W, 1)).squeeze(-1)
        av = self.avail
        # rank feature (i - disabled_before_i) / (W - d): number of available workers before i
        avf = av.to(torch.float32)
        before = torch.cumsum(avf, 1) - avf
        denom = (W - self.n_disable).to(torch.float32).view(E, 1)
        rankf = before / denom
        carry = torch.where(before >= 1, (before - 1) / denom, torch.zeros_like(before))
        one = torch.ones_like(lw0)
        obs_w = torch.stack([
            Rn.view(E, 1).expand(E, W), Cn.view(E, 1).expand(E, W),
            torch.where(av, lw0, one), torch.where(av, lw1, one), torch.where(av, lw2, one),
            torch.where(av, self.worker_pr.to(torch.float32), one), torch.where(av, rankf, carry)], -1)
        navail = avf.sum(1).clamp(min=1)
        mu0 = (lw0 * avf).sum(1) / navail
        mu1 = (lw1 * avf).sum(1) / navail
        mu2 = (lw2 * avf).sum(1) / navail
        mpr = (self.worker_pr * av.to(torch.float64)).sum(1) / navail.to(torch.float64)
        master = torch.stack([Rn, Cn, mu0, mu1, mu2, mpr.to(torch.float32),
                              torch.full_like(Rn, cfg.master_feature)], -1)
        self.obs = torch.cat([obs_w, master.view(E, 1, -1)], 1).contiguous()
        if cfg.shannon:   # ENV_SingleProcess.py:253-255
            self.share = torch.cat([Rn.view(E, 1), Cn.view(E, 1), (self.up_rate / 1e7).to(torch.float32),
                                    (self.rate / 1e7).to(torch.float32)], 1).contiguous()
        else:
            self.share = torch.cat([Rn.view(E, 1), Cn.view(E, 1), self.worker_pr.to(torch.float32)], 1).contiguous()
        ava = torch.ones(E, self.A, 2, dtype=torch.float32, device=dev)
        ava[:, :W, 1] = avf
        self.ava = ava

    # ------------------------------------------------------------------ step (torch path)
    def _geom(self, u, pr):
        """Number of extra tries of ``while U < pr: n += 1``: floor(log U / log pr)."""
        U = px.u01_open(u)
        safe = pr.clamp(min=1e-300, max=1 - 1e-12)
        k = torch.floor(torch.log(U) / torch.log(safe))
        return torch.where(pr > 0, k, torch.zeros_like(k))

    def _near_int(self, u, pr, tol=1e-6):
        """Geometric draws whose log U / log pr lies within ``tol`` of an integer: there the floor may legitimately
        differ between two correct implementations (libm vs device log)."""
        U = px.u01_open(u)
        safe = pr.clamp(min=1e-300, max=1 - 1e-12)
        x = torch.log(U) / torch.log(safe)
        return (pr > 0) & ((x - torch.round(x)).abs() < tol)

    def _step_torch(self, actions):
        cfg, E, W, P = self.cfg, self.E, self.W, self.P
        dev = self.device
        f64 = torch.float64
        if self.fixed:
            strategy = self.avail.to(f64)
            N = strategy.sum(1)
            K = torch.floor(N * cfg.fixed_k_ratio)
        else:
            strategy = actions[:, :W].to(f64)
            ratio = actions[:, W].to(f64)
            N = strategy.sum(1)
            K = torch.ceil(N * ratio)
        standalone = N == 0
        N = N.clamp(1, W)
        K = torch.minimum(torch.maximum(K, torch.ones_like(K)), N)
        K = torch.where(standalone, torch.ones_like(K), K)
        r = torch.ceil(self.R / K)                             # DCML_Master.get_workload: (ceil(R/K), C)
        c = self.C
        ctr = self.task_ctr
        wi = torch.arange(W, device=dev, dtype=torch.int64).view(1, W)
        pr = self.worker_pr
        rr, cc = r.view(E, 1), c.view(E, 1)
        need = torch.ceil((9 * rr - 3) * cc) / cfg.frequency                   # SECOND_TO_CENTSEC * ceil(.)/freq
        ud = px.philox4x32(ctr.view(E, 1), self.gid.view(E, 1), wi, px.P_DOWNLOAD, self.k0, self.k1)
        n = 1 + self._geom(ud[0], pr)
        rec = getattr(self, "record_debug", False)
        near = self._near_int(ud[0], pr) if rec else None
        rate = self.rate                                       # Worker.process uses the download rate for both legs
        transmit = ((torch.ceil((rr + 1) * cc) * cfg.bit_to_byte) / rate + 0.001) * n
        price0 = torch.floor(transmit) * 0.1
        arrive = self.arrive.view(E, 1).to(f64)
        arrive_slot = torch.floor(transmit + arrive)
        tp = torch.remainder(arrive_slot, P).to(torch.int64)
        frac = transmit - torch.floor(transmit)
        lw = self.lw.to(f64)
        lw_tp = torch.gather(lw, 2, tp.unsqueeze(-1)).squeeze(-1)
        need = torch.where(frac > lw_tp, need + frac - lw_tp, need)
        availability = torch.zeros_like(need)
        nslots = torch.zeros_like(need)
        up_unit = (rr * cfg.bit_to_byte) / rate + 0.001
        active = availability < need
        it = 0
        while bool(active.any()) and it < cfg.max_slot_iters:
            a = 1.0 - torch.gather(lw, 2, tp.unsqueeze(-1)).squeeze(-1)
            uu = px.philox4x32(ctr.view(E, 1), self.gid.view(E, 1), wi + (it << 16), px.P_UPLOAD, self.k0, self.k1)
            g = self._geom(uu[0], pr)
            if rec:
                near = near | (active & self._near_int(uu[0], pr))
            availability = torch.where(active, availability + a, availability)
            nslots = torch.where(active, nslots + 1, nslots)
            n = torch.where(active, n + g, n)
            tp = torch.where(active, (tp + 1) % P, tp)
            active = active & (availability < need)
            it += 1
        upload = up_unit * n + 0.02
        delay = arrive_slot + nslots - arrive - (availability - need) + upload        # (E, W)
        tp0 = torch.remainder(arrive_slot, P).to(torch.int64)
        sel = strategy > 0.5
        # K-th order statistic of the selected delays; standalone: worker 0 alone
        big = torch.where(sel, delay, torch.full_like(delay, float("inf")))
        srt, _ = torch.sort(big, 1)
        kidx = (K.to(torch.int64) - 1).clamp(0, W - 1)
        final = torch.gather(srt, 1, kidx.view(E, 1)).squeeze(1)
        final = torch.where(standalone, delay[:, 0], final)
        end = torch.ceil(final)
        # price at index min(end, nslots) - 1 = price0 + sum of the first min(end, nslots) slot availabilities
        cnt = torch.minimum(end.view(E, 1), nslots)
        lw_cyc = 1.0 - lw
        cum = torch.cumsum(torch.cat([lw_cyc, lw_cyc], 2), 2)  # (E, W, 2P)
        period_sum = cum[:, :, P - 1]
        price = price0 + torch.floor(cnt / P) * period_sum + self._partial(cum, tp0, cnt)
        last_price = price0 + torch.floor(nslots / P) * period_sum + self._partial(cum, tp0, nslots)
        payment = (strategy * price).sum(1)
        payment = torch.where(standalone, last_price[:, 0], payment)
        reward = torch.tensor(0.0, dtype=f64, device=dev) + cfg.reward(final, payment)
        reward = torch.where(standalone, reward * cfg.standalone_penalty, reward)
        udn = px.philox4x32(ctr, self.gid, 0, px.P_DONE, self.k0, self.k1)
        done = px.u01_open(udn[0]) < cfg.continue_prob
        if rec:   # the kernel's parity record (csrc/dcml_env.hip StepOut.dbg) + which envs had a borderline draw
            self.last_debug = torch.cat([torch.stack([N, K, standalone.to(f64), final, payment, reward], 1),
                                         n, nslots, delay], 1)
            self.last_near_int = near.any(1)
        self._reset(torch.ones(E, dtype=torch.bool, device=dev))
        return (self.obs, self.share_view(), reward.to(torch.float32), done, final.to(torch.float32),
                payment.to(torch.float32), self.ava)

    def _partial(self, cum, start, cnt):
        P = self.P
        rem = (cnt - torch.floor(cnt / P) * P).to(torch.int64)
        endi = start + rem
        s_end = torch.gather(cum, 2, (endi - 1).clamp(min=0).unsqueeze(-1)).squeeze(-1)
        s_start = torch.gather(cum, 2, (start - 1).clamp(min=0).unsqueeze(-1)).squeeze(-1)
        s_start = torch.where(start > 0, s_start, torch.zeros_like(s_start))
        return torch.where(rem > 0, s_end - s_start, torch.zeros_like(s_end))

    # ------------------------------------------------------------------ HIP path
    def _state_ptrs(self):
        return dict(R=self.R, C=self.C, master_pr=self.master_pr, worker_pr=self.worker_pr,
                    n_disable=self.n_disable, arrive=self.arrive, lw=self.lw, obs=self.obs,
                    share=self.share, ava=self.ava, counter=self.counter, task_ctr=self.task_ctr, rate=self.rate,
                    up_rate=self.up_rate)

    def _reset_hip(self, mask):
        from ...ops import kernels
        kernels.dcml_env_reset(self, mask)

    def _step_hip(self, actions):
        from ...ops import kernels
        return kernels.dcml_env_step(self, actions)
