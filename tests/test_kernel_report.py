"""Kernel-path visibility: which fused HIP gates a config passes, with the reason when not.

The gates are device-independent (``ops/paths.gate_reasons``); ``kernel_report`` adds the device and is what
``bench.py`` prints under ``"kernels"`` and the runners log at start-up.
"""
import os

import pytest
import torch

from mat_dcml_amd.ops import kernels


def _need_lib():
    if not os.path.exists(kernels.LIB_PATH):
        pytest.skip("HIP library not built")


def _mat(obs_dim, act_dim, n_agent, action_type, semi_index=None, n_objective=1):
    from mat_dcml_amd.models.mat import MultiAgentTransformer
    return MultiAgentTransformer(obs_dim, obs_dim, act_dim, n_agent, 2, 64, 2, action_type=action_type,
                                 semi_index=semi_index, n_objective=n_objective)


def test_dcml_config_takes_every_hip_path():
    _need_lib()
    from mat_dcml_amd.ops.paths import gate_reasons
    g = gate_reasons(_mat(7, 2, 33, "Semi_Discrete", -1))
    assert g == {"encoder": [], "decode": [], "train": []}, g


def test_smac_config_gates():
    _need_lib()
    from mat_dcml_amd.envs.smac.synthetic import SyntheticSMACEnv
    from mat_dcml_amd.ops.paths import gate_reasons
    env = SyntheticSMACEnv(2, "27m_vs_30m")
    obs_dim = env.observation_space[0][0]
    g = gate_reasons(_mat(obs_dim, 36, env.n_agents, "Discrete"))
    assert g["decode"] == []
    assert g["encoder"] == [], g
    assert g["train"] == [], g


def test_momat_config_gates():
    _need_lib()
    from mat_dcml_amd.ops.paths import gate_reasons
    g = gate_reasons(_mat(7, 2, 33, "Semi_Discrete", -1, n_objective=2))
    assert g["encoder"] == [] and g["decode"] == []
    assert g["train"] == [], g


def test_runner_report_on_cpu_names_the_reason():
    from mat_dcml_amd.config import get_config, parse_args
    from mat_dcml_amd.ops.paths import kernel_report
    from mat_dcml_amd.runner.dcml_runner import DCMLRunner
    args = parse_args(["--env_name", "DCML", "--n_workers", "4", "--n_rollout_threads", "2", "--episode_length", "2"],
                      get_config(), warn=False)
    r = DCMLRunner({"all_args": args, "device": torch.device("cpu"), "run_dir": None})
    rep = kernel_report(r)
    assert rep["train"] == "torch (cpu device)" and rep["decode"].startswith("torch (")


def test_available_continuous_takes_the_hybrid_gates():
    """Available_Continuous: the fused encoder and decode kernels run; the fused decoder training kernels do not
    (so ops/mat_fused.evaluate_actions trains with the fused encoder under autograd and an eager decoder)."""
    _need_lib()
    from mat_dcml_amd.ops.paths import gate_reasons
    g = gate_reasons(_mat(7, 4, 9, "Available_Continuous"))
    assert g["encoder"] == [] and g["decode"] == [], g
    assert any("Available_Continuous" in r for r in g["train"]), g
