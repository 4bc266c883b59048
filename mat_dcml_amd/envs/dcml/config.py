"""Typed DCML environment configuration.

The reference keeps these as module constants and hard-wires the worker count to 100
(``DCML_ENVs/DCML_utils/DCML_Config.py:1-25``, ``DCML_Master.py:6-16``,
``DCML_Worker_TIMESLOT_MultiProcess.py:5-12``).  Here the worker count is a runtime parameter
(4 / 32 / 100 / 128 in the BASELINE configs) and every quantity that scaled with 100 scales with it.
"""
from __future__ import annotations

import dataclasses
import math
import os

REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
DATA_DIR = os.path.join(REPO_ROOT, "data")


@dataclasses.dataclass
class DCMLConfig:
    n_workers: int = 100                 # WORKER_NUMBER_MAX (DCML_Config.py:7)
    extra_agents: int = 1                # EXTRA_AGENT: the master / ratio agent (DCML_Config.py:3)
    period: int = 20                     # LOCAL_WORKLOAD_PERIOD (DCML_Config.py:2)
    data_rate: float = 150.0 * 2 ** 20   # NON_SHANNON_DATA_RATE (DCML_Config.py:5)
    frequency: float = 2e9               # worker CPU frequency (DCML_Worker_TIMESLOT_MultiProcess.py:16)
    bit_to_byte: float = 4.0             # BIT_TO_BYTE (DCML_Worker_TIMESLOT_MultiProcess.py:11)
    r_min: int = 2 ** 10                 # DCML_Master.py:6-9
    r_max: int = 2 ** 20
    c_min: int = 2 ** 5
    c_max: int = 2 ** 10
    inflate: float = 1.1                 # R, C sampled up to round(max * 1.1) (DCML_Master.py:47-48)
    pr_min: float = 0.0                  # PR_MIN/PR_MAX (DCML_Config.py:22-23)
    pr_max: float = 0.95
    continue_prob: float = 0.8           # CONTINUE_PROBABILITY (DCML_Config.py:25)
    disable_frac: float = 0.8            # disable_rate ~ U{1..80} of 100 (ENV_SingleProcess.py:158)
    alpha: float = 99.0                  # reward = -(alpha*delay + beta*payment) (DCML_ENV_Functions.py:15-17)
    beta: float = 1.0
    standalone_penalty: float = 1.5      # N == 0 branch (ENV_SingleProcess.py:81-92)
    master_feature: float = 1.1          # last feature of the master row (ENV_SingleProcess.py:236)
    fixed_k_ratio: float = 0.7           # fixed heuristic K = floor(0.7 N) (ENV_SingleProcess.py:58-62)
    max_slot_iters: int = 512            # bound on the timeslot loop (measured max 15)
    shannon: bool = False                # shannon_enable: per-worker Shannon-capacity links (Shannon.py:6-21)
    bandwidth_total: float = 100e9       # B_total, split evenly over the workers (DCML_Master.py:27-28)
    noise_dbm: float = -50.0             # Shannon(noise=-50) (Shannon.py:7-9)
    master_power: tuple = (50.0, 60.0)   # TRANSMISSION_POWER_{LOWER,UPPER}_BOUND (DCML_Master.py:11-12)
    worker_power: tuple = (10.0, 20.0)   # MIN/MAX_WORKER_POWER (DCML_Config.py:10-11)
    distance: tuple = (10.0, 100.0)      # DISTANCE_{LOWER,UPPER}_BOUND (DCML_Master.py:13-14)
    path_loss_exp: float = -4.0          # PATH_LOSS_EXPONENT (Shannon.py:4)
    obs_dim: int = 7                     # LOCAL_OBS_DIM
    action_dim: int = 2                  # ACTION_DIM
    workload_file: str = os.path.join(DATA_DIR, "workloads.txt")
    preset_dir: str = os.path.join(DATA_DIR, "dcml_benchmark")
    preset_sample: int = 1

    @property
    def n_agents(self) -> int:
        return self.n_workers + self.extra_agents

    @property
    def share_dim(self) -> int:          # SOB_DIM = 2 + W (DCML_Config.py:12); Shannon: R, C, up/1e7, down/1e7
        return 2 + self.n_workers * (2 if self.shannon else 1)

    @property
    def max_disable(self) -> int:
        """Upper bound of the disabled-worker count (80 for W=100, 26 for W=32)."""
        return max(1, min(self.n_workers - 1, int(round(self.disable_frac * self.n_workers))))

    @property
    def r_hi(self) -> int:
        return int(round(self.r_max * self.inflate))

    @property
    def c_hi(self) -> int:
        return int(round(self.c_max * self.inflate))

    def reward(self, delay, payment):
        return -(self.alpha * delay + self.beta * payment)


def ceil_div(a: int, b: int) -> int:
    return -(-a // b)


def pad_to(x: int, m: int) -> int:
    return int(math.ceil(x / m) * m)
