"""Baseline algorithms (HAPPO / R-MAPPO / IPPO / HATRPO / PPO / random) on the DCML env, and their building blocks."""
import pytest
import torch

from mat_dcml_amd.algos.stacked_adam import StackedAdam
from mat_dcml_amd.config import get_config, parse_args
from mat_dcml_amd.models.ac import MLPBase, SGRU, SLinear


def test_slinear_matches_per_agent_linears():
    torch.manual_seed(0)
    lin = SLinear(3, 5, 4)
    x = torch.randn(7, 3, 5)
    y = lin(x)
    for m in range(3):
        assert torch.allclose(y[:, m], x[:, m] @ lin.weight[m].t() + lin.bias[m], atol=1e-6)
        assert torch.allclose(lin(x[:, m], idx=m), y[:, m], atol=1e-6)


def test_sgru_matches_torch_gru():
    torch.manual_seed(0)
    g = SGRU(2, 6, 8, recurrent_N=1)
    ref = torch.nn.GRU(6, 8)
    m = 1
    with torch.no_grad():
        ref.weight_ih_l0.copy_(g.w_ih[0].weight[m]); ref.bias_ih_l0.copy_(g.w_ih[0].bias[m])
        ref.weight_hh_l0.copy_(g.w_hh[0].weight[m]); ref.bias_hh_l0.copy_(g.w_hh[0].bias[m])
    x = torch.randn(5, 3, 2, 6)
    h0 = torch.randn(3, 2, 1, 8)
    masks = torch.ones(5, 3, 2, 1)
    y, h = g(x, h0, masks)
    yr, hr = ref(x[:, :, m], h0[:, m, 0][None].contiguous())
    assert torch.allclose(h[:, m, 0], hr[0], atol=1e-5)
    # output is LayerNorm(GRU output) (RNNLayer)
    assert torch.allclose(y[:, :, m], g.norm(yr, idx=m), atol=1e-5)


def test_stacked_adam_touches_only_the_selected_agent():
    torch.manual_seed(0)
    net = MLPBase(3, 4, 8, 1)
    opt = StackedAdam(net.parameters(), 3, lr=1e-2)
    before = [p.detach().clone() for p in net.parameters()]
    for _ in range(2):
        opt.zero_grad()
        net(torch.randn(10, 3, 4)).pow(2).sum().backward()
        opt.step(idx=1)
    for p, b in zip(net.parameters(), before):
        assert torch.equal(p[0], b[0]) and torch.equal(p[2], b[2])
    assert any(not torch.equal(p[1], b[1]) for p, b in zip(net.parameters(), before))
    assert float(opt.t[1]) == 2 and float(opt.t[0]) == 0


@pytest.mark.parametrize("algo,extra", [("happo", []), ("rmappo", []), ("ippo", []), ("hatrpo", []), ("ppo", []),
                                        ("random", []), ("happo", ["--use_popart", "--use_cent_local_observe"]),
                                        ("ippo", ["--use_naive_recurrent_policy"])])
def test_baseline_trains_on_dcml(algo, extra, tmp_path):
    import DCML_MAT_Train
    argv = DCML_MAT_Train.DEFAULT_ARGV + ["--algorithm_name", algo, "--n_workers", "4", "--n_rollout_threads", "3",
                                          "--episode_length", "10", "--num_env_steps", "60", "--ppo_epoch", "2",
                                          "--num_mini_batch", "2", "--hidden_size", "16", "--results_dir",
                                          str(tmp_path), "--cuda", "--log_interval", "1", "--data_chunk_length", "5",
                                          "--use_eval", "--eval_interval", "1", "--eval_episodes", "2"] + extra
    if algo != "ppo":
        argv = [a for a in argv if a != "--use_popart"] if "--use_popart" not in extra else argv
    runner = DCML_MAT_Train.main(argv)
    assert runner.buffer.rewards.abs().sum() > 0
    if algo != "random":
        files = list((tmp_path / "DCML").rglob("baseline_*.pt"))
        assert files
        sd = torch.load(files[0], weights_only=True)
        assert "actors" in sd and "critic" in sd
        for p in runner.ac.actors.parameters():
            assert torch.isfinite(p).all()
