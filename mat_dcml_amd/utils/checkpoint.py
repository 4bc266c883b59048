"""Checkpoint I/O compatible with the reference layout.

* ``transformer_{episode}.pt`` = a plain fp32 ``state_dict`` saved with ``torch.save`` into
  ``results/<env>/<scenario>/<algo>/<exp>/run{n}/models/`` (reference ``transformer_policy.py:243-248``,
  ``base_runner.py:64,437-470``).  Written atomically (tmp + rename) by rank 0 only.
* ``trainer_state_{episode}.pt`` (new) = Adam moments, ValueNorm statistics, episode counter, env counters and
  config — a true resume instead of the reference's weights-only warm start.
Loads always use ``weights_only=True``.
"""
from __future__ import annotations

import os

import torch


def _atomic_save(obj, path):
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def save_transformer(model, save_dir, episode):
    os.makedirs(str(save_dir), exist_ok=True)
    sd = {k: v.detach().float().cpu() for k, v in model.state_dict().items()}
    path = os.path.join(str(save_dir), f"transformer_{episode}.pt")
    _atomic_save(sd, path)
    return path


def load_transformer(model, path):
    sd = torch.load(path, map_location="cpu", weights_only=True)
    model.load_state_dict(sd)
    return model


def save_trainer_state(path, policy, trainer, episode, extra=None):
    state = {"episode": int(episode), "optimizer": policy.optimizer.state_dict()}
    if trainer.value_normalizer is not None:
        state["value_normalizer"] = trainer.value_normalizer.state_dict()
    if extra:
        state.update(extra)
    _atomic_save(state, path)


def load_trainer_state(path, policy, trainer):
    state = torch.load(path, map_location="cpu", weights_only=True)
    policy.optimizer.load_state_dict(state["optimizer"])
    if trainer.value_normalizer is not None and "value_normalizer" in state:
        trainer.value_normalizer.load_state_dict(state["value_normalizer"])
    return state
