"""One-shot peer-memory all-reduce (csrc/xgmi_allreduce.hip, parallel/oneshot.py) on the GPU box.

The box has one GPU, so the two ranks map each other's regions on the same device through HIP IPC; the protocol
(flags, buffer halves, bounded waits) is the same one that runs across the xGMI mesh of an 8-GPU node.  The group
for the handle exchange and the comparison all-reduce is gloo (RCCL wants one GPU per rank)."""
import os

import pytest
import torch

from test_dist import _runner_case_w32, spawn

N_ODD = 151_475   # not a multiple of the workgroup count or of 4


def _inputs(k, rank, n):
    g = torch.Generator().manual_seed(1000 * k + rank)
    return torch.randn(n, generator=g) * (1.0 + k)


def _oneshot_case(comm):
    import torch.distributed as dist
    from mat_dcml_amd.parallel.oneshot import OneShotAllReduce
    W, n, calls = comm.world_size, N_ODD, 12
    ar = OneShotAllReduce(comm, n)
    dev = comm.device
    outs = []
    for k in range(calls):   # back to back on one stream, no host sync: exercises both buffer halves
        x = _inputs(k, comm.rank, n).to(dev)
        outs.append(ar(x, scale=1.0 / W) if k % 2 else ar(x.clone(), out=torch.empty_like(x), scale=1.0 / W))
    torch.cuda.synchronize(dev)
    ar.check()
    exact, vs_dist = [], []
    for k in range(calls):
        s = torch.zeros(n)
        for r in range(W):      # the kernel's order: 0 + x_0 + x_1 + ... then one multiply by 1/W
            s = s + _inputs(k, r, n)
        ref = s * (1.0 / W)
        got = outs[k].cpu()
        exact.append(bool(torch.equal(got, ref)))
        t = _inputs(k, comm.rank, n)
        dist.all_reduce(t)
        vs_dist.append(float((got - t / W).abs().max()))
    digest = float(torch.stack([o.double().cpu().sum() for o in outs]).sum())
    ar.close()
    return exact, vs_dist, digest, ar.G


@pytest.mark.gpu
def test_oneshot_allreduce_matches_dist_all_reduce(gpu):
    out = spawn(_oneshot_case, world=2, gpu=True)
    for r in (0, 1):
        exact, vs_dist, digest, G = out[r]
        assert all(exact), exact                 # bit-exact vs the fp32 rank-order sum
        assert max(vs_dist) < 1e-5, vs_dist      # and vs torch.distributed.all_reduce
        assert G >= 32
    assert out[0][2] == out[1][2]                # every rank holds the same result


def _probe_case(comm):
    from mat_dcml_amd.parallel import oneshot
    chosen, ar, info = oneshot.probe(comm, 151_472)
    if ar is not None:
        ar.close()
    return chosen, info


@pytest.mark.gpu
def test_oneshot_probe_agrees_and_decides_identically(gpu):
    """The start-up probe (mode "auto"): one-shot result matches dist.all_reduce, both are timed, and every rank
    takes the same decision."""
    out = spawn(_probe_case, world=2, gpu=True)
    (c0, i0), (c1, i1) = out[0], out[1]
    assert c0 == c1 and c0 in ("oneshot", "rccl")
    assert i0["agree"] and i0["max_rel_err"] <= 1e-5, i0
    assert i0["oneshot_us"] > 0 and i0["backend_us"] > 0 and i0["backend"] == "gloo"
    print("probe:", i0)


def _runner_oneshot(comm):
    os.environ["MAT_DCML_ALLREDUCE"] = "oneshot"
    from mat_dcml_amd.config import get_config, parse_args
    from mat_dcml_amd.runner.dcml_runner import DCMLRunner
    args = parse_args(["--n_workers", "32", "--n_rollout_threads", "16", "--episode_length", "8", "--ppo_epoch", "2",
                       "--num_mini_batch", "2", "--use_valuenorm", "--env_name", "DCML"], get_config(), warn=False)
    r = DCMLRunner({"all_args": args, "device": comm.device, "run_dir": None, "comm": comm})
    r.warmup()
    for _ in range(2):
        r.train_iteration()
    flat = torch.cat([p.detach().reshape(-1) for p in r.policy.transformer.parameters()]).double().cpu()
    calls = comm.oneshot.calls if comm.oneshot is not None else 0
    return float(flat.sum()), float(flat.pow(2).sum()), bool(r.trainer.fused), \
        [float(t) for t in r.trainer.value_normalizer.running_mean_var()], r.trainer.grad_allreduce, calls


@pytest.mark.gpu
def test_dp_fused_trainer_with_oneshot_gradients(gpu):
    """The fused HIP trainer at 2 ranks with the gradient average on the one-shot kernel: ranks stay bit-identical
    and land where the gloo-averaged run lands."""
    a = spawn(_runner_oneshot, world=2, gpu=True)
    b = spawn(_runner_case_w32, world=2, gpu=True)
    assert a[0][2] and a[1][2]
    assert a[0][4] == a[1][4] == "oneshot" and a[0][5] == a[1][5] == 2 * 2 * 2   # iterations x ppo_epoch x minibatches
    assert a[0][0] == a[1][0] and a[0][1] == a[1][1]
    assert a[0][3] == pytest.approx(b[0][3], rel=1e-4, abs=1e-6)   # statistics path is unchanged
    assert abs(a[0][0] - b[0][0]) <= 1e-4 * max(1.0, abs(b[0][0]))
    assert abs(a[0][1] - b[0][1]) <= 1e-4 * max(1.0, abs(b[0][1]))


def _timeout_case(comm):
    """Rank 1 never joins the all-reduce: rank 0's bounded peer wait times out, its output is NaN (so the
    optimizer's non-finite guard skips the step), and both the synchronous check and the per-iteration poll raise."""
    from mat_dcml_amd.parallel.oneshot import OneShotAllReduce
    n = 4096
    ar = OneShotAllReduce(comm, n, wait_s=0.02)
    dev = comm.device
    res = (None, None, None)
    if comm.rank == 0:
        x = torch.ones(n, device=dev)
        y = ar(x, out=torch.empty_like(x))
        ar.poll()                       # queues the first asynchronous error-word copy
        torch.cuda.synchronize(dev)
        try:
            ar.poll()
            polled = False
        except RuntimeError:
            polled = True
        try:
            ar.check()
            raised = False
        except RuntimeError:
            raised = True
        res = (bool(torch.isnan(y).all()), raised, polled)
    comm.barrier()
    if comm.rank == 1:   # the timed-out rank flagged its peers too (bit 31): every rank's check raises
        try:
            ar.check()
            res = (None, False, ar.error_word())
        except RuntimeError:
            res = (None, True, ar.error_word())
    comm.barrier()
    ar.close()
    return res


@pytest.mark.gpu
def test_oneshot_missing_peer_poisons_output_and_raises(gpu):
    out = spawn(_timeout_case, world=2, gpu=True)
    assert out[0] == (True, True, True), out[0]
    assert out[1][1] and out[1][2] & 0x80000000 and out[1][2] & 1, out[1]   # flagged by rank 0
