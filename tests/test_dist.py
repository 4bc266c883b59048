"""Data-parallel semantics without a cluster: gloo, world_size 2, CPU processes."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(rank, world, port, fn, q, gpu=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    if gpu:   # ranks share the box's GPU(s); gloo carries the collectives (RCCL wants one GPU per rank)
        os.environ["MAT_DCML_DIST_BACKEND"] = "gloo"
        os.environ["MAT_DCML_SHARE_DEVICES"] = "1"
    torch.set_num_threads(1)
    try:
        from mat_dcml_amd.parallel.comm import init_from_env
        comm = init_from_env(prefer_gpu=gpu)
        q.put((rank, fn(comm)))
        comm.destroy()
    except Exception as e:  # pragma: no cover - surfaced by the assert below
        import traceback
        q.put((rank, "ERR " + traceback.format_exc()))


def spawn(fn, world=2, gpu=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run, args=(r, world, port, fn, q, gpu)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(60)
    for r, v in out.items():
        assert not (isinstance(v, str) and v.startswith("ERR")), v
    return out


def _grad_case(comm):
    from mat_dcml_amd.models.mat import MultiAgentTransformer
    torch.manual_seed(0)
    m = MultiAgentTransformer(9, 7, 2, 8, 2, 64, 2, action_type="Semi_Discrete", semi_index=-1)
    g = torch.Generator().manual_seed(1)
    obs = torch.rand(8, 8, 7, generator=g)
    act = torch.randint(0, 2, (8, 8, 1), generator=g).float()
    params = [p for p in m.parameters()]
    comm.attach_flat_grads(params)

    def loss_on(o, a):
        lp, v, ent = m(None, o, a, None)
        return lp.mean() + v.pow(2).mean() - 0.01 * ent.mean()
    # full-batch reference gradient (identical on every rank)
    m.zero_grad(set_to_none=False)
    loss_on(obs, act).backward()
    full = torch.cat([p.grad.reshape(-1) for p in params]).clone()
    # data-parallel: each rank its half, averaged by ONE flat all-reduce
    m.zero_grad(set_to_none=False)
    h = slice(4 * comm.rank, 4 * comm.rank + 4)
    loss_on(obs[h], act[h]).backward()
    comm.all_reduce_grads_(params)
    dp = torch.cat([p.grad.reshape(-1) for p in params])
    return float((dp - full).abs().max()), float(full.abs().max())


def _valuenorm_case(comm):
    from mat_dcml_amd.algos.valuenorm import ValueNorm
    x = torch.arange(20, dtype=torch.float32).view(20, 1) * (comm.rank + 1)
    vn = ValueNorm(1, comm=comm)
    vn.update(x[:10] if comm.rank == 0 else x[10:])
    ref = ValueNorm(1)
    full = torch.cat([torch.arange(10.0), torch.arange(10.0, 20.0) * 2]).view(-1, 1)
    ref.update(full)
    return [float(t) for t in vn.running_mean_var()] + [float(t) for t in ref.running_mean_var()]


def _runner_case(comm):
    from mat_dcml_amd.config import get_config, parse_args
    from mat_dcml_amd.runner.dcml_runner import DCMLRunner
    args = parse_args(["--n_workers", "4", "--n_rollout_threads", "2", "--episode_length", "4", "--ppo_epoch", "2",
                       "--num_mini_batch", "2", "--use_valuenorm", "--env_name", "DCML"], get_config(), warn=False)
    r = DCMLRunner({"all_args": args, "device": comm.device, "run_dir": None, "comm": comm})
    r.warmup()
    r.train_iteration()
    flat = torch.cat([p.detach().reshape(-1) for p in r.policy.transformer.parameters()])
    obs0 = r.buffer.obs[0].clone()
    return float(flat.double().sum()), float(flat.double().pow(2).sum()), obs0.sum().item(), \
        [float(t) for t in r.trainer.value_normalizer.running_mean_var()]


def test_dp_gradient_average_equals_full_batch():
    out = spawn(_grad_case)
    for err, scale in out.values():
        assert err < 1e-5 * max(1.0, scale), (err, scale)


def test_dp_valuenorm_statistics_are_global():
    out = spawn(_valuenorm_case)
    for v in out.values():
        assert abs(v[0] - v[2]) < 1e-4 and abs(v[1] - v[3]) < 1e-3
    assert out[0] == out[1]


def test_dp_runner_keeps_ranks_in_sync():
    out = spawn(_runner_case)
    assert out[0][0] == out[1][0] and out[0][1] == out[1][1]  # identical parameters after the update
    assert out[0][2] != out[1][2]                              # but different env partitions
    assert out[0][3] == out[1][3]                              # identical ValueNorm statistics


def _runner_case_w32(comm):
    from mat_dcml_amd.config import get_config, parse_args
    from mat_dcml_amd.runner.dcml_runner import DCMLRunner
    args = parse_args(["--n_workers", "32", "--n_rollout_threads", "16", "--episode_length", "8", "--ppo_epoch", "2",
                       "--num_mini_batch", "2", "--use_valuenorm", "--env_name", "DCML"], get_config(), warn=False)
    r = DCMLRunner({"all_args": args, "device": comm.device, "run_dir": None, "comm": comm})
    r.warmup()
    for _ in range(2):
        r.train_iteration()
    flat = torch.cat([p.detach().reshape(-1) for p in r.policy.transformer.parameters()]).double().cpu()
    return float(flat.sum()), float(flat.pow(2).sum()), bool(r.trainer.fused), \
        [float(t) for t in r.trainer.value_normalizer.running_mean_var()]


@pytest.mark.gpu
def test_dp_fused_gpu_path_keeps_ranks_in_sync(gpu):
    """2 ranks on the GPU box through the fused HIP trainer (flat grads, 8-copy dW workspace, fused loss with the
    ValueNorm sums all-reduced between its kernels, fused Adam): parameters identical across ranks."""
    out = spawn(_runner_case_w32, world=2, gpu=True)
    assert out[0][2] and out[1][2]
    assert out[0][0] == out[1][0] and out[0][1] == out[1][1]
    assert out[0][3] == out[1][3]


def _rng_case(comm):
    from mat_dcml_amd.config import get_config, parse_args
    from mat_dcml_amd.runner.dcml_runner import DCMLRunner
    args = parse_args(["--n_workers", "4", "--n_rollout_threads", "2", "--episode_length", "2", "--env_name", "DCML"],
                      get_config(), warn=False)
    r = DCMLRunner({"all_args": args, "device": comm.device, "run_dir": None, "comm": comm})
    flat = torch.cat([p.detach().reshape(-1) for p in r.policy.transformer.parameters()]).double()
    return float(flat.sum()), torch.rand(8).tolist()


def test_dp_ranks_share_weights_but_not_exploration_noise():
    """identical init on every rank, independent sampling streams (else every replica repeats rank 0's
    exploration noise and the N-rank gradient average has less independent data than one N-times-larger batch)."""
    out = spawn(_rng_case)
    assert out[0][0] == out[1][0]
    assert out[0][1] != out[1][1]


# ------------------------------------------------------------------------------------------ DP at 2 / 4 / 8 ranks
E_TOT, T_SYN, W_SYN = 8, 4, 4


def _synthetic_trainer(comm, E, env_off):
    """A MAT trainer + buffer over envs [env_off, env_off + E) of a fixed synthetic rollout (same data whatever the
    rank count)."""
    from mat_dcml_amd.algos.buffer import RolloutBuffer
    from mat_dcml_amd.algos.mat_trainer import MATTrainer
    from mat_dcml_amd.algos.policy import TransformerPolicy
    from mat_dcml_amd.config import get_config, parse_args
    from mat_dcml_amd.envs.dcml.spaces import dcml_action_spaces
    args = parse_args(["--env_name", "DCML", "--n_workers", str(W_SYN), "--ppo_epoch", "3", "--num_mini_batch", "1",
                       "--use_valuenorm", "--lr", "1e-3"], get_config(), warn=False)
    A = W_SYN + 1
    torch.manual_seed(0)
    pol = TransformerPolicy(args, [7], [W_SYN + 2], dcml_action_spaces(W_SYN)[0], A)
    comm.attach_flat_grads(pol.transformer.parameters())
    tr = MATTrainer(args, pol, A, comm=comm)
    buf = RolloutBuffer(T_SYN, E, A, 7, W_SYN + 2, 2)
    g = torch.Generator().manual_seed(123)
    full = {"obs": torch.rand(T_SYN + 1, E_TOT, A, 7, generator=g),
            "actions": (torch.rand(T_SYN, E_TOT, A, 1, generator=g) < 0.5).float(),
            "action_log_probs": -torch.rand(T_SYN, E_TOT, A, 1, generator=g),
            "value_preds": torch.randn(T_SYN + 1, E_TOT, A, 1, generator=g),
            "rewards": torch.randn(T_SYN, E_TOT, A, 1, generator=g) * 5}
    for k, v in full.items():
        getattr(buf, k).copy_(v[:, env_off:env_off + E])
    return tr, buf, pol


def _dp_equiv_case(comm):
    E = E_TOT // comm.world_size
    tr, buf, pol = _synthetic_trainer(comm, E, comm.rank * E)
    tr.prep_training()
    tr.train(buf)
    flat = torch.cat([p.detach().reshape(-1) for p in pol.transformer.parameters()])
    vn = [t.clone() for t in tr.value_normalizer.running_mean_var()]
    return flat.numpy(), [t.numpy() for t in vn], tr.collectives   # numpy: tensors would travel by shared fd


def _single_reference():
    from mat_dcml_amd.parallel.comm import Comm
    tr, buf, pol = _synthetic_trainer(Comm(), E_TOT, 0)
    tr.prep_training()
    tr.train(buf)
    return torch.cat([p.detach().reshape(-1) for p in pol.transformer.parameters()]), \
        [t.clone() for t in tr.value_normalizer.running_mean_var()]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_dp_equals_single_process_large_batch(world):
    """N ranks with 1/N of the envs each == one process with all of them: parameters identical across ranks and
    within 1e-5 of the single-process update (full-batch minibatches, so the partition does not matter); one
    statistics all-reduce per epoch + one gradient all-reduce per minibatch."""
    torch.set_num_threads(1)
    ref, ref_vn = _single_reference()
    out = spawn(_dp_equiv_case, world=world)
    for r in range(1, world):
        assert (out[r][0] == out[0][0]).all()
    err = (torch.from_numpy(out[0][0]) - ref).abs().max().item()
    assert err < 1e-5, err
    for a, b in zip(out[0][1], ref_vn):
        assert torch.allclose(torch.from_numpy(a), b, rtol=1e-5, atol=1e-6)
    ppo_epoch, n_mb = 3, 1
    assert all(o[2] == ppo_epoch * (n_mb + 1) for o in out.values()), [o[2] for o in out.values()]


def _runner_case_world(comm):
    from mat_dcml_amd.config import get_config, parse_args
    from mat_dcml_amd.runner.dcml_runner import DCMLRunner
    args = parse_args(["--n_workers", "4", "--n_rollout_threads", "2", "--episode_length", "3", "--ppo_epoch", "2",
                       "--num_mini_batch", "2", "--use_valuenorm", "--env_name", "DCML"], get_config(), warn=False)
    r = DCMLRunner({"all_args": args, "device": comm.device, "run_dir": None, "comm": comm})
    r.warmup()
    r.train_iteration()
    flat = torch.cat([p.detach().reshape(-1) for p in r.policy.transformer.parameters()])
    return float(flat.double().sum()), float(flat.double().pow(2).sum()), r.trainer.collectives, \
        [float(t) for t in r.trainer.value_normalizer.running_mean_var()]


@pytest.mark.parametrize("world", [4, 8])
def test_dp_runner_ranks_stay_in_sync_at_4_and_8(world):
    out = spawn(_runner_case_world, world=world)
    for r in range(1, world):
        assert out[r][0] == out[0][0] and out[r][1] == out[0][1] and out[r][3] == out[0][3]
    assert out[0][2] == 2 * (2 + 1)   # 2 epochs x (1 statistics + 2 gradient all-reduces)


def _allreduce_mode_case(comm):
    os.environ["MAT_DCML_ALLREDUCE"] = "auto"
    path = comm.maybe_enable_oneshot(1024)
    buf = torch.full((1024,), float(comm.rank + 1))
    comm.grad_mean_(buf)
    return path, comm.oneshot is None, float(buf[0])


def test_gradient_allreduce_mode_falls_back_to_the_backend_on_cpu():
    """One-shot needs a GPU per rank: on CPU ranks every mode resolves to the process-group backend, and grad_mean_
    averages over ranks."""
    out = spawn(_allreduce_mode_case)
    for r in (0, 1):
        path, none, v = out[r]
        assert path == "gloo" and none and v == 1.5


# ------------------------------------------------------------------------------------------ rank-count invariance
def _rollout_case(comm, E, gpu_fused=False):
    """One rollout (T steps, no update) of E envs per rank; the buffer as CPU tensors."""
    from mat_dcml_amd.config import get_config, parse_args
    from mat_dcml_amd.runner.dcml_runner import DCMLRunner
    args = parse_args(["--n_workers", "32" if gpu_fused else "4", "--n_rollout_threads", str(E), "--episode_length",
                       "6", "--env_name", "DCML", "--use_valuenorm"], get_config(), warn=False)
    r = DCMLRunner({"all_args": args, "device": comm.device, "run_dir": None, "comm": comm})
    r.warmup()
    for _ in range(2):   # two rollouts: the noise counter and the env task counters advance identically
        r.rollout()
    b = r.buffer
    out = {k: getattr(b, k).detach().cpu().numpy().copy() for k in ("obs", "actions", "action_log_probs", "value_preds",
                                                                "rewards", "masks", "available_actions")}
    out["fused"] = bool(r.policy._fused()) if hasattr(r.policy, "_fused") else False
    return out


def _rollout_e2(comm):
    return _rollout_case(comm, 2)


def _rollout_e4(comm):
    return _rollout_case(comm, 4)


def _assert_rank_split_equal(single, parts, exact_model_outputs=True):
    import numpy as np
    for k, v in single.items():
        if k == "fused":
            continue
        joined = np.concatenate([parts[r][k] for r in sorted(parts)], axis=1)
        if k in ("action_log_probs", "value_preds") and not exact_model_outputs:
            # CPU BLAS picks its GEMM kernel by batch size: model outputs may differ in the last bit
            assert np.allclose(joined, v, rtol=1e-6, atol=1e-6), (k, np.abs(joined - v).max())
        else:
            assert np.array_equal(joined, v), (k, np.abs(joined - v).max())


def test_rollout_is_identical_at_one_and_two_ranks():
    """the same global env set (4 envs) split over 2 ranks (gloo, CPU) or run by 1 rank produces
    identical rollouts — env draws AND policy sampling noise are keyed by the global env id: observations, actions,
    rewards, masks bit-identical (model outputs to the last bit of CPU BLAS)."""
    one = spawn(_rollout_e4, world=1)[0]
    two = spawn(_rollout_e2, world=2)
    _assert_rank_split_equal(one, two, exact_model_outputs=False)


def _rollout_gpu_e8(comm):
    return _rollout_case(comm, 8, gpu_fused=True)


def _rollout_gpu_e16(comm):
    return _rollout_case(comm, 16, gpu_fused=True)


@pytest.mark.gpu
def test_rollout_is_identical_at_one_and_two_ranks_gpu(gpu):
    """The fused HIP rollout (encoder kernel, decode kernel with in-kernel Philox noise, env kernel, fused insert)
    at 2 ranks sharing the GPU vs 1 rank with twice the envs: bit-identical buffers."""
    one = spawn(_rollout_gpu_e16, world=1, gpu=True)[0]
    two = spawn(_rollout_gpu_e8, world=2, gpu=True)
    assert one["fused"] and two[0]["fused"]
    _assert_rank_split_equal(one, two)


# ------------------------------------------------------------------------------------------ overlapped gradient all-reduce
def _overlap_case(comm, overlap, gpu_fused=False):
    """One full PPO iteration with (overlap=True) the decoder's gradient slice all-reduced asynchronously under the
    encoder backward, or (False) the single blocking all-reduce of the flat buffer; the parameters afterwards.
    At >= 3 ranks the gradients go through the ordered reduction (all-gather + rank-order sum): a ring all-reduce's
    per-element summation order depends on the message's chunking, so one buffer and two slices can differ in the
    last bit (measured: 1.2e-7 at 4 gloo ranks), while the ordered sum cannot."""
    from mat_dcml_amd.config import get_config, parse_args
    from mat_dcml_amd.runner.dcml_runner import DCMLRunner
    comm.ordered = comm.world_size > 2
    argv = ["--n_workers", "32" if gpu_fused else "4", "--n_rollout_threads", "4", "--episode_length", "4",
            "--ppo_epoch", "2", "--num_mini_batch", "2", "--use_valuenorm", "--env_name", "DCML", "--seed", "5"]
    if overlap:
        argv.append("--grad_overlap")
    args = parse_args(argv, get_config(), warn=False)
    r = DCMLRunner({"all_args": args, "device": comm.device, "run_dir": None, "comm": comm})
    assert r.trainer.grad_overlap == overlap
    assert bool(r.trainer.fused) == gpu_fused
    if overlap:
        assert r.trainer._overlap_split() is not None   # the decoder's gradients are one contiguous slice
    r.warmup()
    r.train_iteration()
    flat = torch.cat([p.detach().reshape(-1) for p in r.policy.transformer.parameters()]).cpu().numpy().copy()
    return flat, r.trainer.collectives


def _overlap_on(comm):
    return _overlap_case(comm, True)


def _overlap_off(comm):
    return _overlap_case(comm, False)


@pytest.mark.parametrize("world", [2, 4])
def test_grad_overlap_gives_identical_parameters(world):
    """``--grad_overlap`` (decoder slice all-reduced while the encoder backward runs, then the rest)
    leaves every rank with parameters torch.equal to the single blocking all-reduce after a full PPO iteration
    (gloo, CPU ranks: the eager path's two-phase backward)."""
    import numpy as np
    on, off = spawn(_overlap_on, world=world), spawn(_overlap_off, world=world)
    for r in range(world):
        assert np.array_equal(on[r][0], off[r][0]), (r, np.abs(on[r][0] - off[r][0]).max())
        assert np.array_equal(on[r][0], on[0][0])
    # 2 epochs x (1 statistics + 2 minibatches x (2 overlapped collectives)) vs x 1
    assert on[0][1] == 2 * (1 + 2 * 2) and off[0][1] == 2 * (1 + 2)


def _overlap_on_gpu(comm):
    return _overlap_case(comm, True, gpu_fused=True)


def _overlap_off_gpu(comm):
    return _overlap_case(comm, False, gpu_fused=True)


@pytest.mark.gpu
def test_grad_overlap_fused_gpu_identical_parameters(gpu):
    """The fused trainer's overlapped schedule (decoder slice of the private workspace reduced right after dec_bwd
    and all-reduced under enc_bwd) at 2 ranks sharing the GPU: parameters equal to the blocking path's."""
    import numpy as np
    on, off = spawn(_overlap_on_gpu, world=2, gpu=True), spawn(_overlap_off_gpu, world=2, gpu=True)
    for r in range(2):
        assert np.array_equal(on[r][0], off[r][0]), (r, np.abs(on[r][0] - off[r][0]).max())
