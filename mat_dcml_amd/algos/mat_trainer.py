"""MAT-PPO trainer on device tensors, data-parallel aware.

Algorithm contract = reference ``mat_src/mat/algorithms/mat/mat_trainer.py:11-223``:

* every PPO epoch recomputes next values, GAE returns and the normalised advantages (``:178-198``);
* advantage normalisation over active entries with population std, ``(A - mean) / (std + 1e-5)`` (``:193-197``);
* policy loss = −Σ min(r·Â, clip(r, 1±ε)·Â)·active / Σ active (``:129-139``);
* value loss: ValueNorm.update(returns) then clipped + Huber(δ) on normalised returns, max, active-masked mean
  (``:54-94``); total = policy − c_e·entropy + c_v·value (``:144``); clip_grad_norm(10) + Adam (``:146-154``).

MI355X-specific:
* statistics that the reference computes over the whole buffer (advantage mean/std, ValueNorm batch moments)
  are all-reduced across ranks, and gradients are averaged with one flat all-reduce per minibatch
  (``parallel/comm.py``), so N ranks ≡ one process with the N-times-larger buffer;
* the per-minibatch loss/backward/clip/Adam runs either in eager PyTorch or through the fused HIP path
  (``ops/mat_fused.py`` teacher-forced encoder/decoder kernels + ``ops/rl_ops``) with no host sync inside an
  epoch, so the host launches run ahead and the GPU never waits on Python (the rocprof kernel sum equals the
  wall time per iteration, ``profiles/r1_kernel_stats_v9.csv``); hipGraph capture is used where launches do bound
  the time (the MuJoCo surrogate's sub-step loop, ``envs/mujoco/physics.py``).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from ..ops import kernels, mat_fused, rl_ops
from .valuenorm import ValueNorm


def huber_loss(e, d):
    a = (e.abs() <= d).float()
    b = (e.abs() > d).float()
    return a * e ** 2 / 2 + b * d * (e.abs() - d / 2)


def mse_loss(e):
    return e ** 2 / 2


class _GatherAhead:
    """``kernels.gather_rows`` of the next minibatch on a side stream: started after the current minibatch's backward
    kernels are queued (it waits for them, so it never competes with the persistent training kernels for CUs) and
    overlapped with that minibatch's workspace reduction + Adam / repack launches; ``take()`` makes the main stream
    wait for it.  Same rows, same arithmetic as the in-line gather: the training step is unchanged bit for bit."""
    _side = {}

    def __init__(self, src, idx, sums):
        main = torch.cuda.current_stream()
        side = _GatherAhead._side.get(main.device)
        if side is None:
            side = _GatherAhead._side[main.device] = torch.cuda.Stream(main.device)
        ready = torch.cuda.Event()
        ready.record(main)
        side.wait_event(ready)
        with torch.cuda.stream(side):
            self.mb = kernels.gather_rows(src, idx, sums, ("adv",))
        self.done = torch.cuda.Event()
        self.done.record(side)
        for t in self.mb.values():   # allocated on the side stream, consumed on the main one
            t.record_stream(main)

    def take(self):
        torch.cuda.current_stream().wait_event(self.done)
        return self.mb


class MATTrainer:
    def __init__(self, args, policy, num_agents, device=torch.device("cpu"), comm=None):
        self.device = torch.device(device)
        self.policy = policy
        self.num_agents = num_agents
        self.comm = comm
        from ..utils.timers import PhaseTimers
        self.timers = PhaseTimers(device, enabled=False)   # the runner shares its own (bench.py phase breakdown)
        self.clip_param = args.clip_param
        self.ppo_epoch = args.ppo_epoch
        self.num_mini_batch = args.num_mini_batch
        self.value_loss_coef = args.value_loss_coef
        self.entropy_coef = args.entropy_coef
        self.max_grad_norm = args.max_grad_norm
        self.huber_delta = args.huber_delta
        self._use_max_grad_norm = args.use_max_grad_norm
        self._use_clipped_value_loss = args.use_clipped_value_loss
        self._use_huber_loss = args.use_huber_loss
        self._use_valuenorm = args.use_valuenorm
        self._use_value_active_masks = args.use_value_active_masks
        self._use_policy_active_masks = args.use_policy_active_masks
        self.recompute_gae_every_epoch = getattr(args, "recompute_gae_every_epoch", True)
        # data parallelism: the decoder's gradient slice all-reduced asynchronously, overlapped with the encoder
        # backward (--grad_overlap, off by default: one blocking all-reduce of the flat buffer per minibatch)
        self.grad_overlap = bool(getattr(args, "grad_overlap", False)) and comm is not None and comm.world_size > 1
        self.value_normalizer = ValueNorm(getattr(args, "n_objective", 1), device=self.device, comm=comm) \
            if self._use_valuenorm else None
        self.generator = None
        self.params = [p for p in policy.transformer.parameters() if p.requires_grad]
        self.poison = False          # fault injection: non-finite gradients this iteration
        self.skipped = torch.zeros((), device=self.device)
        self._vn_pre = None          # (Σ, Σ², n) of the current minibatch's returns when precomputed per epoch
        self.collectives = 0         # statistics / gradient collectives issued (DP accounting, tests)
        self.fused = self._setup_fused(args)

    def _setup_fused(self, args):
        """Fused minibatch step on GPU: fused fwd kernels → fused PPO loss/grad kernel → fused bwd kernels →
        fused clip+Adam over the flat parameter buffer (no autograd graph, ~15 launches per minibatch).
        ``self.fused_reason`` records why the eager path was taken instead."""
        pol = self.policy
        flat = self.comm._flat if self.comm is not None else None
        self.fused_reason = None
        if flat is None:
            self.fused_reason = "no flat gradient buffer"
        elif not pol._fused():
            if pol.device.type != "cuda":
                self.fused_reason = "cpu device"
            elif pol.kernels == "torch" or not pol._is_mat():
                self.fused_reason = f"kernels={pol.kernels}, model {type(pol.transformer).__name__}"
            else:
                self.fused_reason = "; ".join(mat_fused.unsupported_reasons(pol.transformer))
        if self.fused_reason:
            return False
        from ..ops import mat_train, paths, ppo_fused
        m = pol.transformer
        why = paths.train_unsupported_reasons(m)
        if why:
            self.fused_reason = "; ".join(why)
            return False
        fp = ppo_fused.flat_params_of(m)
        if fp is None or fp.numel() != flat.buf.numel():
            self.fused_reason = "parameters are not one flat buffer"
            return False
        for p in self.params:   # grads and params must share one layout
            if p.grad is None or (p.grad.data_ptr() - flat.buf.data_ptr()) != (p.data_ptr() - fp.data_ptr()):
                self.fused_reason = "gradient / parameter layouts differ"
                return False
        self.loss_fused = ppo_fused.PPOLossFused(self, self.device)
        if self.comm.world_size > 1:
            self.grad_allreduce = self.comm.maybe_enable_oneshot(flat.buf.numel())
        copies = int(os.environ.get("MAT_DCML_GRAD_COPIES", "32"))
        # private per-workgroup copies (deterministic, no atomics; round 6) unless MAT_DCML_GRAD_MODE=atomic
        mode = os.environ.get("MAT_DCML_GRAD_MODE", "private")
        if copies > 0:
            mat_train.attach_grad_workspace(m, flat.buf, copies=copies, mode=mode)
        # kernels that add into .grad directly, outside the workspace (the wide-observation embedding backward): the
        # flat buffer is then zeroed per minibatch and the reduction adds to it; otherwise the reduction overwrites
        self._direct_grads = m.encoder.obs_dim > mat_train.MAX_FUSED_OBS or mode != "private" or copies <= 0
        self.deterministic = mode == "private" and copies > 0 and not self._direct_grads
        self._upd_fused = (mode == "private" and copies > 0 and self.comm.world_size == 1
                           and os.environ.get("MAT_DCML_FUSED_UPDATE", "1") != "0")
        # opt-in (MAT_DCML_GATHER_AHEAD=1): the next minibatch's gather on a side stream, overlapped with this
        # minibatch's reduction + Adam launches.  Measured a LOSS at the bench shape (165.1k / 165.3k vs 171.6k /
        # 170.9k env-steps/s, profiles/r6_ab/README.md): the gather contends with the bandwidth-bound workspace
        # reduction (20 us instead of 11) and the cross-stream event waits add latency to every minibatch
        self.gather_ahead = self.device.type == "cuda" and os.environ.get("MAT_DCML_GATHER_AHEAD", "0") == "1"
        # the next minibatch's gather inside the fused update's adam_pack launch (extra workgroups next to the Adam
        # ones, which leave most CUs idle): one launch fewer per minibatch after an epoch's first
        self.fused_gather = self.device.type == "cuda" and os.environ.get("MAT_DCML_FUSED_GATHER", "1") != "0"
        # the reference's cuda_deterministic (store_false: ON unless --cuda_deterministic is passed,
        # DCML_MAT_Train.py:108-110): the fused trainer's PPO update is bit-reproducible with the private gradient
        # workspace (tests/test_gpu_determinism.py); wide observations keep fp32 atomics in their embedding backward
        if getattr(args, "cuda_deterministic", False) and not self.deterministic and self.device.type == "cuda":
            import warnings
            warnings.warn("cuda_deterministic: this configuration's fused update is not bit-reproducible "
                          f"(gradient mode {mode}, direct gradient writers {self._direct_grads})")
        pol.optimizer = ppo_fused.FlatAdam(fp, flat.buf, lr=pol.optimizer.param_groups[0]["lr"], eps=args.opti_eps,
                                           weight_decay=args.weight_decay,
                                           max_grad_norm=args.max_grad_norm if self._use_max_grad_norm else None,
                                           layout=ppo_fused.param_offsets(m))
        return True

    # ------------------------------------------------------------------------------------------------
    def cal_value_loss(self, values, value_preds_batch, return_batch, active_masks_batch):
        clipped = value_preds_batch + (values - value_preds_batch).clamp(-self.clip_param, self.clip_param)
        if self.value_normalizer is not None:
            self.value_normalizer.update(return_batch, presummed=self._vn_pre)
            target = self.value_normalizer.normalize(return_batch)
        else:
            target = return_batch
        e_clip, e_orig = target - clipped, target - values
        if self._use_huber_loss:
            l_clip, l_orig = huber_loss(e_clip, self.huber_delta), huber_loss(e_orig, self.huber_delta)
        else:
            l_clip, l_orig = mse_loss(e_clip), mse_loss(e_orig)
        vl = torch.max(l_orig, l_clip) if self._use_clipped_value_loss else l_orig
        if self._use_value_active_masks:
            am = active_masks_batch.expand_as(vl)
            return (vl * am).sum() / am.sum()
        return vl.mean()

    def ppo_update(self, mb):
        """One minibatch step.  ``mb`` is a dict of device tensors shaped (B, A, ·)."""
        pol = self.policy
        with self.timers("train_fwd"):
            values, logp, entropy = pol.evaluate_actions(None, mb["obs"], mb["actions"], mb["ava"], mb["active"])
        imp = torch.exp(logp - mb["old_logp"])
        surr1 = imp * mb["adv"]
        surr2 = torch.clamp(imp, 1.0 - self.clip_param, 1.0 + self.clip_param) * mb["adv"]
        act = mb["active"]
        if self._use_policy_active_masks:
            policy_loss = -(torch.min(surr1, surr2).sum(-1, keepdim=True) * act).sum() / act.sum()
        else:
            policy_loss = -torch.min(surr1, surr2).sum(-1, keepdim=True).mean()
        value_loss = self.cal_value_loss(values, mb["value_preds"], mb["returns"], act)
        loss = policy_loss - entropy * self.entropy_coef + value_loss * self.value_loss_coef
        flat = self.comm._flat if self.comm is not None else None
        if flat is not None:
            flat.ensure_views()
            flat.buf.zero_()
        else:
            pol.optimizer.zero_grad(set_to_none=False)
        split = self._overlap_split() if self.grad_overlap and flat is not None and not self.poison else None
        with self.timers("train_bwd"):
            if split is None:
                loss.backward()
            else:   # decoder slice first, its all-reduce in flight while the encoder's gradients are computed
                dec_params, enc_params, (lo, hi), rest = split
                loss.backward(inputs=dec_params, retain_graph=True)
                work = self.comm.all_reduce_sum_async(flat.buf[lo:hi], grad=True)
                loss.backward(inputs=enc_params)
        if self.poison:
            for p in self.params:
                p.grad.fill_(float("nan"))
        if split is not None:
            self._finish_overlap(flat.buf, work, rest)
        elif self.comm is not None and self.comm.world_size > 1:
            self.comm.all_reduce_grads_(self.params)
            self.collectives += 1
        if flat is not None:
            grad_norm = flat.buf.norm()
            if self._use_max_grad_norm:   # clip_grad_norm_ semantics: scale = max / (norm + 1e-6), capped at 1
                flat.buf.mul_(torch.clamp(self.max_grad_norm / (grad_norm + 1e-6), max=1.0))
        elif self._use_max_grad_norm:
            grad_norm = nn.utils.clip_grad_norm_(self.params, self.max_grad_norm, foreach=True)
        else:
            grad_norm = torch.norm(torch.stack([p.grad.norm() for p in self.params if p.grad is not None]))
        if bool(torch.isfinite(grad_norm)):     # non-finite guard (torch path: one host sync per step)
            pol.optimizer.step()
        else:
            self.skipped += 1
        mat_fused.bump_version(pol.transformer)
        return value_loss.detach(), grad_norm.detach(), policy_loss.detach(), entropy.detach(), imp.detach().mean()

    def ppo_update_fused(self, mb, pre_stats=None, ahead=None):
        """One fused PPO minibatch step.  ``ahead`` = (sources, row index, advantage sums) of the NEXT minibatch: its
        gather is issued with this minibatch's update — inside the fused update's adam_pack launch (default), on a
        side stream (``gather_ahead``, opt-in), or as its own launch after the update — and returned (a dict, or a
        ``_GatherAhead`` to ``take()``)."""
        from ..ops import mat_train
        pol = self.policy
        m = pol.transformer
        enc, dec, _ = mat_train._state(m, mb["obs"].device)
        tm = self.timers
        with tm("train_fwd"):
            v, rep = enc.forward(mb["obs"], save=True, idx=mb.get("idx"))
            logp, ent = dec.forward(rep, mb["actions"], mb["ava"], save=True, idx=mb.get("idx"))
        buf = self.comm._flat.buf
        if self._direct_grads:
            buf.zero_()
        dv, dlp, dent = self.loss_fused.run(v, logp, ent, mb, self.comm, pre_stats=pre_stats)
        m._mdl_gws_active = hasattr(m, "_mdl_gws")   # weight gradients into the workspace copies
        split = self._overlap_split() if self.grad_overlap and not self.poison else None
        work = None
        with tm("train_bwd"):
            drep = dec.backward(dlp, dent)
            if split is not None:   # the decoder slice is final: reduce its copies, all-reduce it under enc_bwd
                lo, hi = split[2]
                mat_train.reduce_grad_workspace(m, lo, hi, accumulate=self._direct_grads, last=False)
                work = self.comm.all_reduce_sum_async(buf[lo:hi], grad=True)
            enc.backward(drep, dv)
        m._mdl_gws_active = False
        nxt = _GatherAhead(*ahead) if ahead is not None and self.gather_ahead else None
        if split is not None:
            for lo, hi in split[3]:
                mat_train.reduce_grad_workspace(m, lo, hi, accumulate=self._direct_grads, last=(lo, hi) == split[3][-1])
            dec.ctx = None
            enc.ctx = None
            self._finish_overlap(buf, work, split[3])
            pol.optimizer.step(norm_ready=False)
            mat_fused.bump_version(m)
            return self._next_minibatch(ahead, nxt)
        # one process: the workspace reduction also leaves the optimizer's Σ g² partials of the final gradient (no
        # norm launch); under data parallelism the norm is the all-reduced gradient's, so the Adam step computes it
        fuse_norm = self.comm.world_size == 1 and not self.poison
        if fuse_norm and self._upd_fused:
            # round 6: workspace reduction, then clip + Adam + weight repack: two launches (csrc/ppo.hip)
            ga = None
            if ahead is not None and nxt is None and self.fused_gather and \
                    all(t[0].numel() <= 1024 for t in ahead[0].values()):
                ga, nxt = kernels.gather_args(*ahead, ("adv",))   # rows gathered by the adam_pack launch
            mat_train.update_fused(m, pol.optimizer, accumulate=self._direct_grads, gather=ga)
            dec.ctx = None
            enc.ctx = None
            mat_fused.bump_version(m)
            mat_train.mark_packs_current(m)
            return self._next_minibatch(ahead, nxt)
        norm_ready = mat_train.reduce_grad_workspace(m, norm_into=pol.optimizer.scratch if fuse_norm else None,
                                                     accumulate=self._direct_grads)
        dec.ctx = None
        enc.ctx = None
        if self.poison:
            buf[:1].fill_(float("nan"))   # the fused Adam kernel skips non-finite steps
        if self.comm.world_size > 1:
            # ONE blocking all-reduce of the whole 0.6 MB flat gradient per minibatch (the default; --grad_overlap
            # all-reduces the decoder slice asynchronously under enc_bwd instead, the branch above)
            self.comm.grad_mean_(buf)
            self.collectives += 1
        pol.optimizer.step(norm_ready=norm_ready)
        mat_fused.bump_version(m)
        return self._next_minibatch(ahead, nxt)

    @staticmethod
    def _next_minibatch(ahead, nxt):
        """The next minibatch: the one already gathered (``nxt``), else gathered now (its own launch), else None."""
        if nxt is not None or ahead is None:
            return nxt
        return kernels.gather_rows(*ahead, ("adv",))

    # ------------------------------------------------------------------------------------------------
    def _overlap_split(self):
        """(decoder params, encoder params, decoder flat range, other flat ranges) of the overlapped gradient
        all-reduce, or None when the decoder's gradients are not one contiguous range of the flat buffer."""
        cached = getattr(self, "_split", False)
        if cached is not False:
            return cached
        from ..ops import mat_train
        m = self.policy.transformer
        flat = self.comm._flat
        dec = [p for p in m.decoder.parameters() if p.requires_grad]
        ids = {id(p) for p in dec}
        enc = [p for p in self.params if id(p) not in ids]
        flat.ensure_views()
        r = mat_train.flat_range(dec, flat.buf) if dec and enc else None
        if r is None:
            self._split = None
            return None
        lo, hi = r
        hi = min(flat.buf.numel(), (hi + 15) // 16 * 16)   # the per-parameter padding belongs to the slice
        rest = [x for x in ((0, lo), (hi, flat.buf.numel())) if x[1] > x[0]]
        self._split = (dec, enc, (lo, hi), rest)
        return self._split

    def _finish_overlap(self, buf, work, rest):
        """All-reduce the remaining ranges (blocking), wait for the decoder slice, average."""
        for lo, hi in rest:
            self.comm.grad_sum_(buf[lo:hi])
        if work is not None:
            with self.comm._timed("grad_allreduce"):
                work.wait()
        buf.mul_(1.0 / self.comm.world_size)
        self.collectives += 1 + len(rest)

    def _epoch_stats(self, buffer, idx_list, native):
        """Advantage moments (masked Σ, Σ², n) and, under data parallelism with a value normaliser, every
        minibatch's return moments of this epoch — ONE all-reduce per epoch (the reference's per-minibatch
        ValueNorm update order is kept: minibatch m updates with its own, now global, moments).
        Returns (adv_sums fp64[3], per-minibatch stats fp32 [n_mb, 2·n_obj + 2] or None)."""
        act = buffer.active_masks[:-1]
        adv_sums = kernels.masked_sums(buffer.advantages, act) if native else rl_ops.masked_sums(buffer.advantages, act)
        dp = self.comm is not None and self.comm.world_size > 1
        if not dp:
            if native and self.value_normalizer is not None:
                # single process: the same one-launch per-epoch moments replace a memset + reduction launch per
                # minibatch inside the fused loss (fixed-order sums instead of fp32 atomics)
                mbs = kernels.mb_stats(buffer.flat("returns"), buffer.flat("active_masks"), torch.cat(idx_list),
                                       len(idx_list))
                return adv_sums, mbs.float().contiguous()
            return adv_sums, None
        mbs = None
        if self.value_normalizer is not None:
            ret_f, am_f = buffer.flat("returns"), buffer.flat("active_masks")
            if native:
                mbs = kernels.mb_stats(ret_f, am_f, torch.cat(idx_list), len(idx_list))
            else:
                rows = []
                for idx in idx_list:
                    r = ret_f[idx].double().reshape(-1, ret_f.shape[-1])
                    rows.append(torch.cat([r.sum(0), (r * r).sum(0),
                                           torch.tensor([float(r.shape[0])], dtype=torch.float64, device=r.device),
                                           am_f[idx].double().sum().reshape(1)]))
                mbs = torch.stack(rows)
            K = mbs.shape[1]
            packed = torch.cat([adv_sums, mbs[:, :K - 1].reshape(-1)])
        else:
            packed = adv_sums
        self.comm.all_reduce_sum_(packed)
        self.collectives += 1
        adv_sums = packed[:3]
        if mbs is None:
            return adv_sums, None
        # global (Σ ret, Σ ret², n); the active count stays local (losses are local means, gradients are averaged)
        pre = torch.cat([packed[3:].view(len(idx_list), K - 1), mbs[:, K - 1:]], 1).float().contiguous()
        return adv_sums, pre

    def train(self, buffer):
        pol = self.policy
        keys = ["value_loss", "policy_loss", "dist_entropy", "actor_grad_norm", "critic_grad_norm", "ratio"]
        acc = torch.zeros(len(keys), device=self.device)
        if self.fused:
            self.loss_fused.out.zero_()
            pol.optimizer.clear_grad_norm_sum()
        T, E = buffer.T, buffer.E
        obs_f = buffer.flat("obs")
        act_f = buffer.flat("actions")
        ava_f = buffer.flat("available_actions")
        lp_f = buffer.flat("action_log_probs")
        vp_f = buffer.flat("value_preds")
        am_f = buffer.flat("active_masks")
        n_obj = buffer.returns.shape[-1]
        # HIP path: advantage statistics by a fixed-order fp64 reduction kernel, and each minibatch gathered by ONE
        # launch that also standardises the advantages of the rows it reads (no full normalised copy)
        native = self.fused and kernels.use_hip(obs_f)
        from ..ops import mat_train
        if native and mat_train.WIDE_OBS_BF16 and obs_f.shape[-1] > mat_train.MAX_FUSED_OBS and \
                self.num_mini_batch == 1:
            # wide observations (SMAC) as bf16 ONCE per update, not per epoch: the obs-embedding kernels read half
            # the bytes (the encoder would round them itself, identically, on every call)
            obs_f = obs_f.to(torch.bfloat16)
        for epoch in range(self.ppo_epoch):
            if epoch == 0 or self.recompute_gae_every_epoch:
                next_values = pol.get_values(None, buffer.obs[-1], buffer.available_actions[-1])
                buffer.compute_returns(next_values, self.value_normalizer)
            ret_f = buffer.flat("returns")
            idx_list = buffer.minibatch_indices(self.num_mini_batch, self.generator)
            sums, pre = self._epoch_stats(buffer, idx_list, native)
            if native:
                adv_f = buffer.flat("advantages")
            else:
                adv = rl_ops.normalize_from_sums(buffer.advantages, sums)
                adv_f = adv.reshape(T * E, *adv.shape[2:])
            src = {"obs": obs_f, "actions": act_f, "ava": ava_f, "old_logp": lp_f, "value_preds": vp_f,
                   "returns": ret_f, "active": am_f, "adv": adv_f}
            ahead = None   # the next minibatch, gathered during this one's update (fused launch or side stream)
            for m, idx in enumerate(idx_list):
                if ahead is not None:
                    mb = ahead.take() if isinstance(ahead, _GatherAhead) else ahead
                    ahead = None
                elif native and len(idx_list) == 1 and getattr(self, "inplace_single_minibatch", True):
                    # one minibatch = the whole batch: the permutation only reorders the rows the loss averages
                    # over, so the buffer's rows are used in place (SMAC: no 2 x 445 MB gather copy per epoch);
                    # the loss kernel standardises the advantages itself (adv_sums)
                    mb = dict(src, idx=None, adv_sums=sums)
                elif native and self.fused and os.environ.get("MAT_DCML_MB_INDEX", "gather") == "kernel":
                    # opt-in (round 6): no gather — the training kernels and the loss read the buffer's rows through
                    # the epoch permutation (sequence index) and standardise the advantages in-kernel.  Measured at
                    # the bench shape it is ~0.5 % slower than the gather (the indexed reads cost the four training
                    # kernels more than the 2-launch gather costs), so the gather stays the default
                    mb = dict(src, idx=idx, adv_sums=sums)
                elif native:
                    mb = kernels.gather_rows(src, idx, sums, ("adv",))
                else:
                    mb = {k: v[idx] for k, v in src.items()}
                if self.fused:
                    nxt = None
                    if native and m + 1 < len(idx_list) and "idx" not in mb and (self.gather_ahead or self.fused_gather):
                        nxt = (src, idx_list[m + 1], sums)
                    ahead = self.ppo_update_fused(mb, None if pre is None else pre[m], ahead=nxt)
                    continue
                self._vn_pre = None if pre is None else (pre[m, :n_obj], pre[m, n_obj:2 * n_obj], pre[m, 2 * n_obj])
                vl, gn, pl, ent, ratio = self.ppo_update(mb)
                self._vn_pre = None
                acc += torch.stack([vl, pl, ent, gn, gn, ratio]).float()
        if self.fused:   # loss scalars accumulated on device by the loss kernel: [policy, value, entropy, ratio]
            o = self.loss_fused.out
            acc[0], acc[1], acc[2], acc[5] = o[1], o[0], o[2], o[3]
            acc[3] = acc[4] = pol.optimizer.grad_norm_sum
        acc /= self.ppo_epoch * self.num_mini_batch
        if self.comm is not None and self.comm.world_size > 1:
            self.comm.poll_errors()
        return dict(zip(keys, acc))

    def prep_training(self):
        self.policy.train()

    def prep_rollout(self):
        self.policy.eval()
