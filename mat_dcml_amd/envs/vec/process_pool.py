"""CPU process pool for external, CPU-bound simulators (SC2, MPE, …) — ``ShareSubprocVecEnv`` semantics.

Reference: ``mat_src/mat/envs/env_wrappers.py:300-403`` — one worker process per env connected by a
``multiprocessing.Pipe``; ``step`` = send every action then receive every result (a lock-step barrier),
``auto_reset`` of finished episodes inside the worker, ``reset`` / ``close`` / ``get_spaces`` RPCs, the env factory
shipped once with cloudpickle.

MI355X-side differences: results are stacked into pinned host tensors and copied to the GPU with ONE
non-blocking H2D copy per field (instead of the reference's per-call ``torch.from_numpy(...).to(device)`` in the
policy), and ``n_workers`` may be smaller than the env count (each worker steps ``envs_per_worker`` envs
sequentially), so a 32-env SMAC pool need not fork 32 processes on a small CPU share.  DCML never uses this
path — its env lives on the GPU.
"""
from __future__ import annotations

import multiprocessing as mp

import cloudpickle
import numpy as np
import torch


def _worker(remote, parent_remote, fn_blob, auto_reset):
    parent_remote.close()
    fns = cloudpickle.loads(fn_blob)
    envs = [f() for f in fns]
    try:
        while True:
            cmd, data = remote.recv()
            if cmd == "step":
                out = []
                for env, a in zip(envs, data):
                    ob, s_ob, rew, done, info, ava = env.step(a)
                    if auto_reset and np.all(done):
                        ob, s_ob, ava = env.reset()
                    out.append((ob, s_ob, rew, done, info, ava))
                remote.send(out)
            elif cmd == "reset":
                remote.send([env.reset() for env in envs])
            elif cmd == "get_spaces":
                e = envs[0]
                remote.send((e.observation_space, e.share_observation_space, e.action_space,
                             getattr(e, "n_agents", len(e.observation_space))))
            elif cmd == "close":
                for env in envs:
                    getattr(env, "close", lambda: None)()
                remote.close()
                break
            else:
                raise NotImplementedError(cmd)
    except KeyboardInterrupt:
        pass


class ProcessPoolVecEnv:
    def __init__(self, env_fns, device="cpu", n_workers=None, auto_reset=True, context="spawn"):
        self.n_envs = len(env_fns)
        n_workers = min(n_workers or self.n_envs, self.n_envs)
        per = [env_fns[i::n_workers] for i in range(n_workers)]
        self._order = [i for w in range(n_workers) for i in range(w, self.n_envs, n_workers)]
        ctx = mp.get_context(context)
        self.remotes, work_remotes = zip(*[ctx.Pipe() for _ in range(n_workers)])
        self.procs = []
        for wr, r, fns in zip(work_remotes, self.remotes, per):
            p = ctx.Process(target=_worker, args=(wr, r, cloudpickle.dumps(fns), auto_reset), daemon=True)
            p.start()
            self.procs.append(p)
            wr.close()
        self.device = torch.device(device)
        self.remotes[0].send(("get_spaces", None))
        self.observation_space, self.share_observation_space, self.action_space, self.n_agents = self.remotes[0].recv()
        self.closed = False

    def _gather(self):
        res = [None] * self.n_envs
        k = 0
        for r in self.remotes:
            for item in r.recv():
                res[self._order[k]] = item
                k += 1
        return res

    def _to_dev(self, arrs, dtype=torch.float32):
        t = torch.from_numpy(np.stack(arrs).astype(np.float32 if dtype == torch.float32 else np.bool_))
        if self.device.type == "cuda":
            return t.pin_memory().to(self.device, non_blocking=True)
        return t

    def reset(self):
        for r in self.remotes:
            r.send(("reset", None))
        res = self._gather()
        obs, share, ava = zip(*res)
        return self._to_dev(obs), self._to_dev(share), self._to_dev(ava)

    def step(self, actions):
        a = actions.detach().cpu().numpy() if isinstance(actions, torch.Tensor) else np.asarray(actions)
        # worker w owns envs w, w + n_workers, …  (same striding as construction)
        nw = len(self.remotes)
        for w, r in enumerate(self.remotes):
            r.send(("step", [a[i] for i in range(w, self.n_envs, nw)]))
        res = self._gather()
        obs, share, rew, done, info, ava = zip(*res)
        return (self._to_dev(obs), self._to_dev(share), self._to_dev(rew), self._to_dev(done, torch.bool),
                list(info), self._to_dev(ava))

    def close(self):
        if self.closed:
            return
        for r in self.remotes:
            r.send(("close", None))
        for p in self.procs:
            p.join(timeout=5)
        self.closed = True
