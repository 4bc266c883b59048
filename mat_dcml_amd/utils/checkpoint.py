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
from pathlib import Path

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
    state = {"episode": int(episode), "optimizer": policy.optimizer.state_dict(),
             "lr": policy.optimizer.param_groups[0]["lr"]}
    if trainer.value_normalizer is not None:
        state["value_normalizer"] = trainer.value_normalizer.state_dict()
    if extra:
        state.update(extra)
    _atomic_save(state, path)


def latest_checkpoint(models_dir):
    """Highest episode with both ``transformer_{ep}.pt`` and ``trainer_state_{ep}.pt`` present."""
    import re
    if not models_dir or not os.path.isdir(models_dir):
        return None
    eps = []
    for f in os.listdir(models_dir):
        m = re.fullmatch(r"trainer_state_(\d+)\.pt", f)
        if m and os.path.exists(os.path.join(models_dir, f"transformer_{m.group(1)}.pt")):
            eps.append(int(m.group(1)))
    return max(eps) if eps else None


def save_env_state(models_dir, episode, rank, env):
    """Per-rank env counters.  Philox streams are counter-based, so (task counter, preset index) regenerate the
    current task exactly on restore."""
    os.makedirs(str(models_dir), exist_ok=True)
    st = {"task_ctr": env.task_ctr.cpu(), "preset_idx": env.preset_idx.cpu()}
    _atomic_save(st, os.path.join(str(models_dir), f"env_state_{episode}_rank{rank}.pt"))


def load_env_state(models_dir, episode, rank, env):
    path = os.path.join(str(models_dir), f"env_state_{episode}_rank{rank}.pt")
    if not os.path.exists(path):
        return False
    st = torch.load(path, map_location="cpu", weights_only=True)
    dev = env.counter.device
    env.counter.copy_(st["task_ctr"].to(dev))
    env.preset_idx.copy_((st["preset_idx"] - 1).clamp(min=0).to(dev))
    env._reset(torch.ones(env.E, dtype=torch.bool, device=dev))
    return True


def load_trainer_state(path, policy, trainer):
    state = torch.load(path, map_location="cpu", weights_only=True)
    policy.optimizer.load_state_dict(state["optimizer"])
    if trainer.value_normalizer is not None and "value_normalizer" in state:
        trainer.value_normalizer.load_state_dict(state["value_normalizer"])
    return state


def make_run_dir(all_args, comm):
    """``results/<env>/<scenario>/<algo>/<exp>/run{n}`` (reference ``DCML_MAT_Train.py:116-147``); rank 0 picks
    the run number, every rank gets the same path."""
    root = Path(all_args.results_dir or os.path.join(os.getcwd(), "results"))
    run_dir = root / all_args.env_name / all_args.scenario / all_args.algorithm_name / all_args.experiment_name
    name = None
    if comm.is_main:
        run_dir.mkdir(parents=True, exist_ok=True)
        nums = [int(p.name[3:]) for p in run_dir.iterdir() if p.name.startswith("run") and p.name[3:].isdigit()]
        name = f"run{max(nums) + 1}" if nums and not all_args.resume else (f"run{max(nums)}" if nums else "run1")
    name = comm.all_gather_object(name)[0]
    run_dir = run_dir / name
    if comm.is_main:
        run_dir.mkdir(parents=True, exist_ok=True)
    return run_dir
