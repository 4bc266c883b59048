"""MAT policy wrapper: action-type dispatch, Adam, save/restore — on device tensors only.

Mirrors ``TransformerPolicy`` (reference ``mat_src/mat/algorithms/mat/algorithm/transformer_policy.py:20-255``):
same action-type selection from the action-space object (``:27-39``), same model variants (``:66-79``),
same Adam (``:104-106``), same ``get_actions / get_values / evaluate_actions / act / save / restore /
lr_decay`` surface.  Differences: inputs/outputs are device tensors shaped (B, A, ·) (no numpy reshapes),
and the fused HIP paths (``ops/mat_fused.py``) are used for the rollout decode and the training forward on GPU.
Checkpoints are the reference file (``transformer_{episode}.pt``, plain fp32 state_dict, ``:243-244``).
"""
from __future__ import annotations

import os

import torch

from ..models import act as act_mod
from ..models.mat import MultiAgentTransformer
from ..models.variants import build_variant
from ..ops import kernels, mat_fused


def action_type_of(act_space):
    cls = act_space.__class__.__name__
    if cls == "Box":
        return "Continuous", None
    if cls in ("Action_Space", "ActionSpec"):
        si = getattr(act_space, "semi_index", 0)
        if si != 0:
            return "Semi_Discrete", si
        if getattr(act_space, "continuous", False) and not getattr(act_space, "mixed", True):
            return "Continuous", None
        return "Discrete", None
    if cls in ("Available_Continous_Space", "Available_Continuous_Space"):
        return "Available_Continous", None
    return "Discrete", None


class TransformerPolicy:
    def __init__(self, args, obs_space, cent_obs_space, act_space, num_agents, device=torch.device("cpu")):
        self.args = args
        self.device = torch.device(device)
        self.algorithm_name = getattr(args, "algorithm_name", "mat")
        self.lr = args.lr
        self.opti_eps = args.opti_eps
        self.weight_decay = args.weight_decay
        self._use_policy_active_masks = args.use_policy_active_masks
        self.action_type, semi_index = action_type_of(act_space)
        self.obs_dim = _dim(obs_space)
        self.share_obs_dim = _dim(cent_obs_space)
        if self.action_type in ("Discrete", "Semi_Discrete"):
            self.act_dim = act_space.n
            self.act_output_num = 1
            self.act_prob_dim = 1
        elif self.action_type == "Available_Continous":
            self.act_dim = act_space.shape if isinstance(act_space.shape, int) else act_space.shape[0]
            self.act_output_num = self.act_dim
            self.act_prob_dim = 2
        else:
            self.act_dim = act_space.shape[0]
            self.act_output_num = self.act_dim
            self.act_prob_dim = self.act_dim
        self.num_agents = num_agents
        self.n_objective = getattr(args, "n_objective", 1)
        if self.algorithm_name in ("mat", "mat_dec", "momat", "dmomat"):
            self.transformer = MultiAgentTransformer(
                self.share_obs_dim, self.obs_dim, self.act_dim, num_agents, n_block=args.n_block, n_embd=args.n_embd,
                n_head=args.n_head, encode_state=args.encode_state, device=self.device, action_type=self.action_type,
                dec_actor=args.dec_actor, share_actor=args.share_actor, semi_index=semi_index,
                n_objective=self.n_objective)
        else:
            self.transformer = build_variant(self.algorithm_name, self.share_obs_dim, self.obs_dim, self.act_dim,
                                             num_agents, args, self.device, self.action_type, semi_index)
        if getattr(args, "env_name", "") == "hands":
            self.transformer.zero_std()
        # all parameters in one flat fp32 buffer (fused Adam / flat grads / one all-reduce)
        from ..ops.ppo_fused import flatten_params
        flatten_params(self.transformer)
        self.optimizer = torch.optim.Adam(self.transformer.parameters(), lr=self.lr, eps=self.opti_eps,
                                          weight_decay=self.weight_decay)
        self.kernels = getattr(args, "kernels", "auto")
        self.amp_dtype = torch.bfloat16 if (self.device.type == "cuda" and getattr(args, "dtype", "bf16") == "bf16") else None

    # --------------------------------------------------------------------------------------------
    def lr_decay(self, episode, episodes):
        lr = self.lr - self.lr * (episode / float(episodes))   # utils/util.py:17-21
        for g in self.optimizer.param_groups:
            g["lr"] = lr

    def _fused(self):
        return (self.kernels != "torch" and self.device.type == "cuda" and self._is_mat()
                and mat_fused.supports(self.transformer))

    def _enc_fused(self):
        """Hybrid path for MAT configs the fused decode rejects (``dec_actor`` / mat_dec, ...): the encoder still
        runs on the fused HIP kernels (inference and, under autograd, training); only the decoder runs eager."""
        if self.kernels == "torch" or self.device.type != "cuda" or not self._is_mat() or not kernels.available():
            return False
        from ..ops import mat_train
        m = self.transformer
        return not m.encoder.encode_state and mat_train.encoder_supported(m)

    def _is_mat(self):
        return isinstance(self.transformer, MultiAgentTransformer)

    def _autocast(self):
        return torch.autocast("cuda", dtype=self.amp_dtype, enabled=self.amp_dtype is not None)

    @torch.no_grad()
    def get_actions(self, cent_obs, obs, available_actions=None, deterministic=False, stride=1, rand=None):
        """(B, A, ·) inputs → values (B,A,n_obj), actions (B,A,out), log-probs (B,A,out)."""
        m = self.transformer
        if self._fused():
            return mat_fused.get_actions(m, obs, available_actions, deterministic, stride, rand)
        if rand is None and not deterministic and getattr(m, "_mdl_env0", None) is not None:
            # globally keyed noise (mat_fused.set_sampling_key): the same draws as the decode kernel's
            B, L = obs.shape[0], obs.shape[1]
            k0, k1, c = mat_fused.next_draw_key(m)
            rand = act_mod.philox_rand(B, L, m.action_dim, k0, k1, c, m._mdl_env0, obs.device,
                                       normal=m.action_type != "Discrete")
        if not self._is_mat():   # variants (models/variants.py): model-level API
            with self._autocast():
                a, lp, v = m.get_actions(cent_obs, obs, available_actions, deterministic, stride, rand)
            return v.float(), a, lp
        if self._enc_fused():
            v, rep = mat_fused.get_values_rep(m, obs)
            with torch.autocast("cuda", dtype=self.amp_dtype, enabled=self.amp_dtype is not None):
                a, lp = act_mod.autoregressive_act(m, rep, obs, available_actions, deterministic, stride, rand)
            return v, a, lp
        with torch.autocast("cuda", dtype=self.amp_dtype, enabled=self.amp_dtype is not None):
            v, rep = m.encoder(cent_obs, obs)
            a, lp = act_mod.autoregressive_act(m, rep, obs, available_actions, deterministic, stride, rand)
        return v.float(), a, lp

    @torch.no_grad()
    def get_values(self, cent_obs, obs, available_actions=None):
        m = self.transformer
        if self._fused() or self._enc_fused():
            return mat_fused.get_values(m, obs)
        if not self._is_mat():
            with self._autocast():
                return m.get_values(cent_obs, obs, available_actions).float()
        with torch.autocast("cuda", dtype=self.amp_dtype, enabled=self.amp_dtype is not None):
            v, _ = m.encoder(cent_obs, obs)
        return v.float()

    def evaluate_actions(self, cent_obs, obs, actions, available_actions=None, active_masks=None):
        """Returns values (B,A,n_obj), log-probs (B,A,p), scalar entropy (active-masked mean)."""
        m = self.transformer
        if self._fused() or self._enc_fused():   # fully fused, or hybrid (fused encoder + eager decoder)
            values, logp, ent = mat_fused.evaluate_actions(m, obs, actions, available_actions)
        elif not self._is_mat():
            with self._autocast():
                logp, values, ent = m(cent_obs, obs, actions, available_actions)
            values = values.float()
        else:
            with torch.autocast("cuda", dtype=self.amp_dtype, enabled=self.amp_dtype is not None):
                v, rep = m.encoder(cent_obs, obs)
                logp, ent = act_mod.parallel_act(m, rep, obs, actions, available_actions)
            values = v.float()
        if self._use_policy_active_masks and active_masks is not None:
            # (N, A) entropies times (N, 1) masks (transformer_policy.py:212-213): summed over the action dims,
            # divided by the active-token count
            am = active_masks.reshape(ent.shape[:-1] + (1,)) if active_masks.numel() * ent.shape[-1] == ent.numel() \
                else active_masks.expand_as(ent)
            entropy = (ent * am).sum() / am.sum()
        else:
            entropy = ent.mean()
        return values, logp, entropy

    def act(self, cent_obs, obs, available_actions=None, deterministic=True, stride=2):
        _, a, _ = self.get_actions(cent_obs, obs, available_actions, deterministic, stride)
        return a

    def save(self, save_dir, episode):
        from ..utils.checkpoint import save_transformer
        return save_transformer(self.transformer, save_dir, episode)

    def restore(self, model_dir):
        from ..utils.checkpoint import load_transformer
        load_transformer(self.transformer, model_dir)
        mat_fused.bump_version(self.transformer)

    def train(self):
        self.transformer.train()

    def eval(self):
        self.transformer.eval()


def _dim(space):
    if isinstance(space, (list, tuple)):
        x = space[0]
        return x[0] if isinstance(x, (list, tuple)) else x
    if hasattr(space, "shape"):
        return space.shape[0]
    return int(space)
