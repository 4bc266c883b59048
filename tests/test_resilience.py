"""Fault injection, non-finite guard, checkpoint/resume and the restart launcher."""
import os
import subprocess
import sys

import torch

import DCML_MAT_Train
from mat_dcml_amd.parallel.resilience import FaultInjector, launch_with_restarts

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--n_workers", "4", "--n_rollout_threads", "2", "--episode_length", "4", "--ppo_epoch", "2",
         "--num_mini_batch", "2", "--n_embd", "32", "--cuda", "--log_interval", "100", "--save_interval", "1"]


def test_fault_spec_parsing():
    f = FaultInjector("nan@3,kill@1:5,disable@0.5", rank=1)
    assert f.poison_grads(3) and not f.poison_grads(2)
    assert f.kill_at == 5 and f.disable_frac == 0.5
    assert FaultInjector("kill@0:5", rank=1).kill_at is None


def test_nan_injection_skips_the_step(tmp_path):
    argv = DCML_MAT_Train.DEFAULT_ARGV + SMALL + ["--num_env_steps", "8", "--results_dir", str(tmp_path),
                                                 "--fault_inject", "nan@0"]
    runner = DCML_MAT_Train.main(argv)
    assert float(runner.trainer.skipped) == 2 * 2          # every minibatch step of iteration 0 was skipped
    for p in runner.policy.transformer.parameters():
        assert torch.isfinite(p).all()


def test_resume_restores_weights_optimizer_and_counters(tmp_path):
    argv = DCML_MAT_Train.DEFAULT_ARGV + SMALL + ["--results_dir", str(tmp_path)]
    r1 = DCML_MAT_Train.main(argv + ["--num_env_steps", "16"])          # 2 episodes: 0, 1
    w1 = torch.cat([p.detach().reshape(-1) for p in r1.policy.transformer.parameters()])
    ctr1 = r1.envs.task_ctr.clone()
    r2 = DCML_MAT_Train.Runner.__new__(DCML_MAT_Train.Runner)
    from mat_dcml_amd.config import get_config, parse_args
    from mat_dcml_amd.parallel.comm import Comm
    a = parse_args(argv + ["--num_env_steps", "16"], get_config(), warn=False)
    run_dir = max((tmp_path / "DCML" / "AS" / "mat" / "check").iterdir())
    r2.__init__({"all_args": a, "device": torch.device("cpu"), "run_dir": run_dir, "comm": Comm()})
    ep = r2.resume()
    assert ep == 1 and r2.start_episode == 2
    w2 = torch.cat([p.detach().reshape(-1) for p in r2.policy.transformer.parameters()])
    assert torch.equal(w1, w2)
    assert torch.equal(r2.envs.task_ctr, ctr1) and r2._resumed
    sd1, sd2 = r1.policy.optimizer.state_dict(), r2.policy.optimizer.state_dict()
    assert sd1["state"][0]["exp_avg"].equal(sd2["state"][0]["exp_avg"])
    assert torch.equal(r1.trainer.value_normalizer.running_mean, r2.trainer.value_normalizer.running_mean)


def test_killed_run_restarts_from_checkpoint(tmp_path):
    cmd = [sys.executable, os.path.join(REPO, "DCML_MAT_Train.py")] + SMALL + \
        ["--num_env_steps", "24", "--results_dir", str(tmp_path), "--fault_inject", "kill@0:2"]
    # first attempt dies at episode 2 (after checkpoints 0 and 1); the relaunch resumes at episode 2 and finishes —
    # the kill spec fires again only at episode 2, which the resumed run starts at, so strip it on restart
    rc = launch_with_restarts(cmd, max_restarts=0)
    assert rc == 17
    models = max((tmp_path / "DCML" / "AS" / "mat" / "check").iterdir()) / "models"
    assert (models / "trainer_state_1.pt").exists() and not (models / "transformer_2.pt").exists()
    cmd2 = [c for c in cmd if c not in ("--fault_inject", "kill@0:2")]
    rc = subprocess.call(cmd2 + ["--resume"], cwd=str(tmp_path))
    assert rc == 0
    assert (models / "transformer_2.pt").exists()


def test_kill_flushes_the_queued_log(tmp_path):
    """log() only queues its statistics (asynchronous all-reduce); an injected kill at episode 2 must still print the
    episode-1 log line that was queued before it."""
    small = [a if a != "100" else "1" for a in SMALL]   # --log_interval 1
    cmd = [sys.executable, os.path.join(REPO, "DCML_MAT_Train.py")] + small + \
        ["--num_env_steps", "24", "--results_dir", str(tmp_path), "--fault_inject", "kill@0:2"]
    r = subprocess.run(cmd, cwd=str(tmp_path), capture_output=True, text=True, timeout=600)
    assert r.returncode == 17, r.stderr[-2000:]
    assert "updates 1/3 episodes" in r.stdout, r.stdout[-2000:]


def test_heartbeat_detects_silent_rank(monkeypatch):
    import time
    import types
    from mat_dcml_amd.parallel import resilience

    class Store(dict):
        def set(self, k, v):
            self[k] = v.encode()

        def get(self, k):
            return self[k]
    hb = resilience.Heartbeat(types.SimpleNamespace(world_size=1, rank=0), 0.0)   # disabled (single rank)
    assert hb.store is None
    hb.comm = types.SimpleNamespace(world_size=3, rank=0)
    hb.store, hb.timeout = Store(), 5.0
    now = time.time()
    hb.store.set("mdl_hb/0", repr(now))
    hb.store.set("mdl_hb/1", repr(now - 1))
    hb.store.set("mdl_hb/2", repr(now - 60))
    exits = []
    monkeypatch.setattr(resilience.os, "_exit", lambda c: exits.append(c))
    assert hb.check() == [2] and exits == [resilience.KILL_EXIT_CODE + 1]
