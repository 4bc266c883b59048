"""ctypes bindings for the in-tree HIP library ``mat_dcml_amd/_lib/libmatdcml.so`` (gfx950).

The library is plain HIP C++ (``mat_dcml_amd/csrc/*.hip``) compiled by ``hipcc --offload-arch=gfx950``
(``mat_dcml_amd/csrc/build.py``); each entry point takes raw device pointers and the current HIP stream,
so launches are captured by hipGraphs exactly like torch's own kernels.

Policy: on a GPU tensor the HIP path is the default and a missing library is an ERROR (no silent eager
fallback) unless ``MAT_DCML_KERNELS=torch`` is set explicitly.  CPU tensors always take the torch path.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "_lib", os.environ.get("MAT_DCML_LIBNAME", "libmatdcml.so"))
_lib = None
_load_error = None


def mode():
    return os.environ.get("MAT_DCML_KERNELS", "auto").lower()


def _csrc():
    return os.path.join(os.path.dirname(_HERE), "csrc")


def _build_mod():
    import importlib.util
    spec = importlib.util.spec_from_file_location("_mat_dcml_build", os.path.join(_csrc(), "build.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def build_identity(L):
    """(source hash, flags hash) embedded in a loaded library (None for a library built before the guard)."""
    try:
        return tuple((ctypes.c_char * 17).in_dll(L, n).value.decode()   # const char[17] arrays, not pointers
                     for n in ("mdl_build_source_hash", "mdl_build_flags_hash"))
    except ValueError:
        return None


def check_build(L, src_dir=None, default_lib=None):
    """None when library ``L`` was built from the sources in ``src_dir`` (and, for the default library, with the
    default flags); otherwise the reason it is stale."""
    b = _build_mod()
    if os.path.basename(LIB_PATH).startswith("libmatdcml_ab_") and src_dir is None:
        # explicit A/B timing builds (scripts/build_ab.sh: another revision's sources, or timing-only variants) are
        # never loaded by the tests / bench / smoke, which use the default library
        return None
    got = build_identity(L)
    if got is None:
        return "the library carries no build identity (built before the staleness guard)"
    want = b.source_hash(src_dir or _csrc())
    if got[0] != want:
        return f"built from sources {got[0]}, the tree has {want}"
    if default_lib if default_lib is not None else LIB_PATH.endswith("libmatdcml.so"):
        wf = b.flags_hash()
        if got[1] != wf:
            return f"built with flags {got[1]}, the build would use {wf}"
    return None


BUILD_ID = None   # the loaded library's source hash (logged by bench.py / smoke)


class _BuildLock:
    """Exclusive ``flock`` on ``_lib/.build.lock``: the ranks of one node (``bench.py --gpus N``, torchrun) that find
    a stale library check and rebuild it one at a time, so the first rebuilds and the others see it fresh."""

    def __init__(self, lib_dir):
        self.path = os.path.join(lib_dir, ".build.lock")

    def __enter__(self):
        import fcntl
        os.makedirs(os.path.dirname(self.path), exist_ok=True)   # fresh checkout: nothing under _lib is tracked
        self.f = open(self.path, "a")
        fcntl.flock(self.f, fcntl.LOCK_EX)
        return self

    def __exit__(self, *exc):
        import fcntl
        fcntl.flock(self.f, fcntl.LOCK_UN)
        self.f.close()


def _sidecar_stale(b):
    """Why the default library must be rebuilt, judged from its sidecar identity file (no dlopen), or None."""
    if not os.path.exists(LIB_PATH):
        return "not built"
    got = b.sidecar(LIB_PATH)
    if got is None:
        return "no build identity sidecar"
    if got != (b.source_hash(), b.flags_hash()):
        return f"built from {got}, the tree has {(b.source_hash(), b.flags_hash())}"
    return None


def lib():
    """Load the HIP library, refusing a stale one: its embedded source / flags hash must match the tree.  When hipcc
    exists, the default library is checked (by its sidecar identity, before it is ever dlopen'ed) and rebuilt if
    stale, under a file lock shared by every process of the node; anything else stale is an error."""
    global _lib, _load_error, BUILD_ID
    if _lib is None:
        b = _build_mod()
        # only the default library is rebuilt: a named variant (A/B timing builds, MAT_DCML_LIBNAME) was built with
        # flags the environment of this process need not carry, so "stale" there means "leave it alone"
        if os.path.exists(b.HIPCC) and LIB_PATH == b.OUT and os.path.basename(LIB_PATH) == "libmatdcml.so":
            with _BuildLock(os.path.dirname(LIB_PATH)):
                why = _sidecar_stale(b)   # re-checked under the lock: another rank may have just rebuilt it
                if why is not None:
                    print(f"[kernels] {LIB_PATH} is stale ({why}): rebuilding", flush=True)
                    b.build()
        if not os.path.exists(LIB_PATH):
            _load_error = f"{LIB_PATH} not built (run python -c 'import __graft_entry__ as g; g.build()')"
            raise RuntimeError(_load_error)
        L = ctypes.CDLL(LIB_PATH)
        why = check_build(L)
        if why is not None:
            _load_error = f"stale native library {LIB_PATH}: {why}; rebuild it (python mat_dcml_amd/csrc/build.py)"
            raise RuntimeError(_load_error)
        BUILD_ID = (build_identity(L) or ("unidentified",))[0]   # A/B variants may predate the identity
        _lib = L
        _declare(_lib)
    return _lib


def available():
    """True when the HIP library is loaded.  On a GPU box a missing / unloadable library is an error, not a silent
    fall-back to the eager path (``MAT_DCML_KERNELS=torch`` selects the eager path explicitly)."""
    if mode() == "torch":
        return False
    try:
        lib()
        return True
    except Exception:
        if torch.cuda.is_available():
            raise
        return False


def use_hip(t: torch.Tensor) -> bool:
    if not t.is_cuda or mode() == "torch":
        return False
    lib()  # raises loudly when the extension is missing on a GPU run
    return True


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_CUR_DEV = getattr(torch._C, "_cuda_getDevice", None)


def _stream():
    """The current HIP stream of the current device as a ctypes pointer.  torch.cuda.current_stream() builds a Stream
    object (device-index resolution included): ~9 us of host time per launch, 4 launches per rollout step — the
    rollout's host side runs only ~1.5x ahead of the GPU, so the raw accessor is used where this torch has it."""
    if _RAW_STREAM is not None and _CUR_DEV is not None:
        return ctypes.c_void_p(_RAW_STREAM(_CUR_DEV()))
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def P(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


_SIGS = {}


def _declare(L):
    vp, i32, f32, i64, u64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_int64, ctypes.c_uint64
    ab = os.path.basename(LIB_PATH).startswith("libmatdcml_ab_")
    for name, args in _SIGS.items():
        try:
            fn = getattr(L, name)
        except AttributeError:
            if ab:   # an A/B build of an older revision: its missing entry points are never called by the A/B run
                continue
            raise
        fn.argtypes = args
        fn.restype = ctypes.c_int


def sig(name, *args):
    """Register an entry point's argument types.  Applied at load time, and immediately when the library is
    already loaded (modules that declare signatures may be imported after the first launch — without this, raw
    Python-int pointers would be passed as 32-bit C ints)."""
    _SIGS[name] = list(args)
    if _lib is not None:
        fn = getattr(_lib, name)
        fn.argtypes = list(args)
        fn.restype = ctypes.c_int


def check(rc, name):
    if rc != 0:
        raise RuntimeError(f"HIP kernel {name} failed with hipError {rc}")


# ----------------------------------------------------------------------------------------- RL ops
vp, i32, f32, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_int64
sig("mdl_gae_reverse_scan", vp, vp, vp, vp, vp, vp, i32, i32, i32, f32, f32, vp)


def gae_reverse_scan(rewards, value_preds, masks, meanstd, gamma, lam, adv_out, ret_out):
    """rewards (T, ..., n_obj), value_preds (T+1, ..., n_obj), masks (T+1, ..., 1) shared by the objectives,
    meanstd [means(n_obj) | stds(n_obj)] fp32."""
    T = rewards.shape[0]
    n = rewards[0].numel()
    n_obj = rewards.shape[-1]
    assert value_preds.shape[0] == T + 1 and masks.numel() * n_obj == (T + 1) * n and meanstd.numel() == 2 * n_obj
    for t in (rewards, value_preds, masks, adv_out, ret_out, meanstd):
        assert t.is_contiguous() and t.dtype == torch.float32
    check(lib().mdl_gae_reverse_scan(P(rewards), P(value_preds), P(masks), P(meanstd), P(adv_out), P(ret_out),
                                     T, n, n_obj, gamma, lam, _stream()), "gae_reverse_scan")


sig("mdl_gae_reverse_scan_vn", vp, vp, vp, vp, vp, vp, vp, f32, i32, vp, vp, i32, i32, i32, f32, f32, vp)


def gae_reverse_scan_vn(rewards, value_preds, masks, next_value, vn, gamma, lam, adv_out, ret_out):
    """gae_reverse_scan with the ValueNorm statistics computed in-kernel from ``vn``'s running moments (or none) and
    V(T) = next_value, which is also written into value_preds[-1]."""
    T = rewards.shape[0]
    n = rewards[0].numel()
    n_obj = rewards.shape[-1]
    assert value_preds.shape[0] == T + 1 and masks.numel() * n_obj == (T + 1) * n and next_value.numel() == n
    for t in (rewards, value_preds, masks, adv_out, ret_out, next_value):
        assert t.is_contiguous() and t.dtype == torch.float32
    rm = rmsq = deb = None
    nvn, eps = 1, 1e-5
    if vn is not None:
        rm, rmsq, deb = vn.running_mean, vn.running_mean_sq, vn.debiasing_term
        for t in (rm, rmsq, deb):
            assert t.is_contiguous() and t.dtype == torch.float32
        nvn, eps = rm.numel(), float(vn.epsilon)
    check(lib().mdl_gae_reverse_scan_vn(P(rewards), P(value_preds), P(masks), P(next_value), P(rm), P(rmsq), P(deb),
                                        eps, nvn, P(adv_out), P(ret_out), T, n, n_obj, gamma, lam, _stream()),
          "gae_reverse_scan_vn")


u32 = ctypes.c_uint32
sig("mdl_philox_fill", vp, i32, u32, u32, u32, u32, u32, vp)


def philox_fill(n, c1, c2, c3, k0, k1, device):
    out = torch.empty(n, 4, dtype=torch.int64, device=device)
    check(lib().mdl_philox_fill(P(out), n, c1, c2, c3, k0, k1, _stream()), "philox_fill")
    return out


sig("mdl_randperm", vp, i32, u32, u32, vp)


def randperm(n, device, generator=None, key=None):
    """Random permutation of [0, n) (int64, on ``device``) by one keyed-Feistel launch (csrc/rl_ops.hip; reference
    ``utils/philox.feistel_randperm``); the key is drawn from the CPU generator (``torch.manual_seed`` seeds it),
    so no device RNG launch either."""
    if key is None:
        g = generator if generator is not None and generator.device.type == "cpu" else None
        k = torch.randint(0, 2 ** 31 - 1, (2,), generator=g).tolist()
    else:
        k = [int(key[0]), int(key[1])]
    out = torch.empty(n, dtype=torch.int64, device=device)
    check(lib().mdl_randperm(P(out), int(n), int(k[0]), int(k[1]), _stream()), "randperm")
    return out


# ----------------------------------------------------------------------------------------- minibatch / adv stats
sig("mdl_masked_sums", vp, vp, i32, i32, vp, vp, vp)
_SUMS_WS = {}


def masked_sums(x, mask):
    """(Σx, Σx², count) over active entries as a device fp64[3] (fixed-order reduction, no host sync)."""
    assert x.is_contiguous() and mask.is_contiguous() and x.dtype == mask.dtype == torch.float32
    mdiv = x.numel() // mask.numel()
    assert mdiv * mask.numel() == x.numel()
    ws = _SUMS_WS.get(x.device)
    if ws is None:
        ws = _SUMS_WS[x.device] = torch.empty(3 * 240, dtype=torch.float64, device=x.device)
    out = torch.empty(3, dtype=torch.float64, device=x.device)
    check(lib().mdl_masked_sums(P(x), P(mask), x.numel(), mdiv, P(ws), P(out), _stream()), "masked_sums")
    return out


sig("mdl_mb_stats", vp, vp, vp, i32, i32, i32, i32, vp, vp, vp)
_MBS_WS = {}


def mb_stats(ret, active, perm, n_mb):
    """Per-minibatch (Σ ret_o, Σ ret_o², count, Σ active) of one epoch's partition ``perm`` (n_mb equal slices of
    rows; every row = ``ret.shape[1]`` tokens) as a device fp64 [n_mb, 2·n_obj + 2]."""
    assert ret.is_contiguous() and active.is_contiguous() and perm.dtype == torch.int64 and perm.is_contiguous()
    n_obj = ret.shape[-1]
    width = ret[0].numel() // n_obj
    mb = perm.numel() // n_mb
    K = 2 * n_obj + 2
    ws = _MBS_WS.get(ret.device)
    if ws is None or ws.numel() < n_mb * 32 * K:
        ws = _MBS_WS[ret.device] = torch.empty(max(n_mb, 16) * 32 * K, dtype=torch.float64, device=ret.device)
    out = torch.empty(n_mb, K, dtype=torch.float64, device=ret.device)
    check(lib().mdl_mb_stats(P(ret), P(active), P(perm), n_mb, mb, width, n_obj, P(ws), P(out), _stream()), "mb_stats")
    return out


class GatherEnt(ctypes.Structure):
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("width", ctypes.c_int), ("norm", ctypes.c_int)]


class GatherArgs(ctypes.Structure):
    _fields_ = [("e", GatherEnt * 10), ("idx", ctypes.c_void_p), ("sums", ctypes.c_void_p), ("rows", ctypes.c_int),
                ("n", ctypes.c_int), ("eps", ctypes.c_float)]


sig("mdl_gather_rows", vp, vp)


def gather_args(srcs, idx, norm_sums=None, norm_keys=(), eps=1e-5):
    """The GatherArgs of ``gather_rows`` and its freshly allocated outputs (the launch is the caller's: the standalone
    ``mdl_gather_rows`` or the fused update's adam_pack, csrc/ppo.hip).  The struct keeps raw pointers: the caller
    holds ``srcs``, ``idx`` and ``norm_sums`` until the launch has run."""
    assert idx.dtype == torch.int64 and idx.is_contiguous() and len(srcs) <= 10
    a = GatherArgs()
    out = {}
    for k, (name, src) in enumerate(srcs.items()):
        assert src.is_contiguous() and src.dtype == torch.float32
        dst = torch.empty((idx.numel(), *src.shape[1:]), dtype=torch.float32, device=src.device)
        width = src[0].numel()
        a.e[k] = GatherEnt(src.data_ptr(), dst.data_ptr(), width, int(name in norm_keys))
        out[name] = dst
    if norm_keys:
        assert norm_sums is not None and norm_sums.dtype == torch.float64
    a.idx, a.sums, a.rows, a.n, a.eps = idx.data_ptr(), norm_sums.data_ptr() if norm_sums is not None else 0, \
        idx.numel(), len(srcs), eps
    return a, out


def gather_rows(srcs, idx, norm_sums=None, norm_keys=(), eps=1e-5):
    """{name: src (N, …) fp32 contiguous} -> {name: src[idx]} in one launch; entries in ``norm_keys`` are
    standardised with ``norm_sums`` (from ``masked_sums``) on the fly."""
    a, out = gather_args(srcs, idx, norm_sums, norm_keys, eps)
    check(lib().mdl_gather_rows(ctypes.byref(a), _stream()), "gather_rows")
    return out


# ----------------------------------------------------------------------------------------- rollout insert
class InsSeg(ctypes.Structure):
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("n", ctypes.c_int)]


class InsArgs(ctypes.Structure):
    _fields_ = [("seg", InsSeg * 6), ("E", ctypes.c_int), ("A", ctypes.c_int), ("n_obj", ctypes.c_int)] + \
               [(n, ctypes.c_void_p) for n in ("reward", "delay", "pay", "done", "d_rew", "d_mask", "ep_r", "ep_d",
                                               "ep_p", "stats")]


sig("mdl_rollout_insert", ctypes.POINTER(InsArgs), vp)


def rollout_insert(copies, reward, delay, pay, done, rew_slot, mask_slot, ep_r, ep_d, ep_p, stats):
    """One launch: ``dst.copy_(src)`` for up to 6 (src, dst) pairs of contiguous f32 tensors, the agent-expanded
    rewards ((E, A, n_obj) slot; n_obj 2 = (-delay, -payment)) and masks, the episode sums and done statistics
    (runner/dcml_runner.py _track / insert)."""
    a = InsArgs()
    for k, (src, dst) in enumerate(copies):
        assert src.dtype == dst.dtype == torch.float32 and src.numel() == dst.numel()
        assert src.is_contiguous() and dst.is_contiguous()
        a.seg[k] = InsSeg(src.data_ptr(), dst.data_ptr(), src.numel())
    E, A, n_obj = rew_slot.shape
    a.E, a.A, a.n_obj = E, A, n_obj
    for n, t in (("reward", reward), ("delay", delay), ("pay", pay), ("done", done), ("d_rew", rew_slot),
                 ("d_mask", mask_slot), ("ep_r", ep_r), ("ep_d", ep_d), ("ep_p", ep_p), ("stats", stats)):
        assert t.is_contiguous(), n
        setattr(a, n, t.data_ptr())
    assert done.dtype == torch.bool and stats.dtype == torch.float64 and mask_slot.numel() == E * A
    check(lib().mdl_rollout_insert(ctypes.byref(a), _stream()), "rollout_insert")


class SmacInsArgs(ctypes.Structure):
    _fields_ = [("seg", InsSeg * 6), ("E", ctypes.c_int), ("A", ctypes.c_int)] + \
               [(n, ctypes.c_void_p) for n in ("reward", "dones", "won", "dead", "d_rew", "d_mask", "d_active", "ep_r",
                                               "stats")]


sig("mdl_smac_insert", ctypes.POINTER(SmacInsArgs), vp)


def smac_insert(copies, reward, dones, won, dead, rew_slot, mask_slot, active_slot, ep_r, stats):
    """One launch: the SMAC runner's _track_smac + _insert_smac (csrc/rl_ops.hip smac_insert_kernel)."""
    a = SmacInsArgs()
    for k, (src, dst) in enumerate(copies):
        assert src.dtype == dst.dtype == torch.float32 and src.numel() == dst.numel()
        assert src.is_contiguous() and dst.is_contiguous()
        a.seg[k] = InsSeg(src.data_ptr(), dst.data_ptr(), src.numel())
    E, A = dones.shape
    a.E, a.A = E, A
    for n, t in (("reward", reward), ("dones", dones), ("won", won), ("dead", dead), ("d_rew", rew_slot),
                 ("d_mask", mask_slot), ("d_active", active_slot), ("ep_r", ep_r), ("stats", stats)):
        assert t.is_contiguous(), n
        setattr(a, n, t.data_ptr())
    assert dones.dtype == torch.bool and won.dtype == torch.bool and stats.dtype == torch.float64
    assert reward.numel() == E and rew_slot.numel() == E * A and mask_slot.numel() == E * A
    assert active_slot.numel() == E * A and dead.dtype == torch.float32 and ep_r.numel() == E
    check(lib().mdl_smac_insert(ctypes.byref(a), _stream()), "smac_insert")


# ----------------------------------------------------------------------------------------- DCML env
class EnvCfg(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("E", "W", "A", "P", "obs_dim", "share_dim", "fixed", "preset",
                                            "max_disable", "max_slot_iters", "preset_rows", "shannon")] + \
               [("k0", ctypes.c_uint32), ("k1", ctypes.c_uint32)] + \
               [(n, ctypes.c_double) for n in ("r_min", "r_max", "c_min", "c_max", "r_hi", "c_hi", "pr_min", "pr_max",
                                               "rate", "freq", "bit_to_byte", "continue_prob", "alpha", "beta",
                                               "standalone_penalty", "fixed_k_ratio", "band", "noise", "mp_lo",
                                               "mp_hi", "wp_lo", "wp_hi", "d_lo", "d_hi", "ple")] + \
               [("master_feature", ctypes.c_float)]


class EnvState(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("gid", "profiles", "counter", "task_ctr", "R", "C", "master_pr",
                                               "worker_pr", "avail", "n_disable", "arrive", "lw", "obs", "share",
                                               "ava", "preset_idx", "preset_master", "preset_prs", "preset_disable",
                                               "rate", "up_rate")]


class StepOut(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("actions", "reward", "done", "delay", "payment", "dbg")]


sig("mdl_dcml_env_reset", ctypes.POINTER(EnvCfg), ctypes.POINTER(EnvState), vp)
sig("mdl_dcml_env_step", ctypes.POINTER(EnvCfg), ctypes.POINTER(EnvState), ctypes.POINTER(StepOut), vp)


def _env_structs(env):
    c = env.cfg
    ec = EnvCfg(E=env.E, W=env.W, A=env.A, P=env.P, obs_dim=c.obs_dim, share_dim=c.share_dim, fixed=int(env.fixed),
                preset=int(env.preset), max_disable=c.max_disable, max_slot_iters=c.max_slot_iters,
                preset_rows=int(env.preset_master.shape[0]) if env.preset else 0, k0=env.k0, k1=env.k1,
                r_min=c.r_min, r_max=c.r_max, c_min=c.c_min, c_max=c.c_max, r_hi=c.r_hi, c_hi=c.c_hi,
                pr_min=c.pr_min, pr_max=c.pr_max, rate=c.data_rate, freq=c.frequency, bit_to_byte=c.bit_to_byte,
                continue_prob=c.continue_prob, alpha=c.alpha, beta=c.beta, standalone_penalty=c.standalone_penalty,
                fixed_k_ratio=c.fixed_k_ratio, master_feature=c.master_feature, shannon=int(c.shannon),
                band=c.bandwidth_total / env.W, noise=10.0 ** (c.noise_dbm / 10.0), mp_lo=c.master_power[0],
                mp_hi=c.master_power[1], wp_lo=c.worker_power[0], wp_hi=c.worker_power[1], d_lo=c.distance[0],
                d_hi=c.distance[1], ple=c.path_loss_exp)
    pm = env.preset_master if env.preset else None
    pp = env.preset_prs if env.preset else None
    pd = env.preset_disable if env.preset else None
    es = EnvState(*[t.data_ptr() if t is not None else None for t in (
        env.gid, env.profiles, env.counter, env.task_ctr, env.R, env.C, env.master_pr, env.worker_pr, env.avail,
        env.n_disable, env.arrive, env.lw, env.obs, env.share, env.ava, env.preset_idx, pm, pp, pd, env.rate,
        env.up_rate)])
    return ec, es


def dcml_env_reset(env, mask=None):
    ec, es = _env_structs(env)
    check(lib().mdl_dcml_env_reset(ctypes.byref(ec), ctypes.byref(es), _stream()), "dcml_env_reset")


def dcml_env_step(env, actions):
    if not hasattr(env, "_out"):
        dev = env.device
        env._out = (torch.zeros(env.E, device=dev), torch.zeros(env.E, dtype=torch.bool, device=dev),
                    torch.zeros(env.E, device=dev), torch.zeros(env.E, device=dev))
    rew, done, delay, pay = env._out
    actions = actions.contiguous()
    ec, es = _env_structs(env)
    dbg = None
    if getattr(env, "record_debug", False):   # parity record (tests/test_gpu_env.py)
        dbg = torch.zeros(env.E, 6 + 3 * env.W, dtype=torch.float64, device=env.device)
        env.last_debug = dbg
    so = StepOut(actions.data_ptr(), rew.data_ptr(), done.data_ptr(), delay.data_ptr(), pay.data_ptr(),
                 dbg.data_ptr() if dbg is not None else None)
    check(lib().mdl_dcml_env_step(ctypes.byref(ec), ctypes.byref(es), ctypes.byref(so), _stream()), "dcml_env_step")
    return env.obs, env.share_view(), rew, done, delay, pay, env.ava


# ----------------------------------------------------------------------------------------- MuJoCo surrogate physics
class PlanarConsts(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("B", "J", "R", "nu", "nsub", "kind")] + \
               [(n, ctypes.c_float) for n in ("h", "mass", "root_I", "k_contact", "c_contact", "mu", "grav_y", "cn",
                                              "ct")]


sig("mdl_planar_step", vp, vp, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp)


def planar_step(consts, scal, act, p, th, v, w, q, qd, tau, f_end, f_root):
    """All sub-steps of one PlanarSim env step in one launch (csrc/planar_sim.hip); state tensors updated in place."""
    c = PlanarConsts(*scal)
    B, J = c.B, c.J
    for t, n in ((p, 2 * B), (th, B), (v, 2 * B), (w, B), (q, B * J), (qd, B * J), (tau, B * J), (f_end, 2 * B * J),
                 (f_root, 2 * B), (act, B * c.nu)):
        assert t.is_cuda and t.is_contiguous() and t.dtype == torch.float32 and t.numel() == n, (t.shape, n)
    assert consts.is_contiguous() and consts.dtype == torch.float32
    check(lib().mdl_planar_step(ctypes.byref(c), P(consts), consts.numel(), P(act), P(p), P(th), P(v), P(w), P(q),
                                P(qd), P(tau), P(f_end), P(f_root), _stream()), "planar_step")


# ----------------------------------------------------------------------------------------- SMAC-shaped env
class SmacCfg(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("E", "A", "N", "nA", "u", "limit", "obs_dim", "state_dim", "rao",
                                            "mode")] + \
               [("k0", ctypes.c_uint32), ("k1", ctypes.c_uint32), ("inv_reward_scale", ctypes.c_float)]


class SmacState(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("gid", "ep_ctr", "apos", "ahp", "epos", "ehp", "t", "last",
                                               "battles_won", "battles_game", "perm")]


class SmacOut(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("actions", "obs", "state", "ava", "reward", "dones", "won", "lost",
                                               "timeout", "dead_allies", "dead_enemies", "battles_won_out",
                                               "battles_game_out")]


sig("mdl_smac_env", ctypes.POINTER(SmacCfg), ctypes.POINTER(SmacState), ctypes.POINTER(SmacState), ctypes.POINTER(SmacOut), vp)


def smac_env(env, actions):
    """One launch of csrc/smac_env.hip: the step (``actions`` (E, A) policy rows) or, with ``actions=None``, the
    reset of every env; returns (obs, state, ava, reward (E,), dones (E, A) bool, info)."""
    E, A, N, sp = env.E, env.A, env.N, env.spec
    dev = env.device
    for name in ("apos", "ahp", "epos", "ehp"):
        t = getattr(env, name)
        if t.dtype != torch.float32 or not t.is_contiguous():
            setattr(env, name, t.float().contiguous())
    for name in ("t", "last", "perm", "ep_ctr", "gid"):
        t = getattr(env, name)
        if t.dtype != torch.int64 or not t.is_contiguous():
            setattr(env, name, t.long().contiguous())
    c = SmacCfg(E=E, A=A, N=N, nA=env.n_actions, u=sp.unit_type_bits, limit=sp.limit, obs_dim=sp.obs_dim,
                state_dim=sp.state_dim, rao=int(env.random_agent_order), mode=0 if actions is not None else 1,
                k0=env.k0, k1=env.k1, inv_reward_scale=1.0 / env.reward_scale)
    names = ("gid", "ep_ctr", "apos", "ahp", "epos", "ehp", "t", "last", "battles_won", "battles_game", "perm")
    # ping-pong state: the kernel reads the env's tensors and writes the spare copy, which then becomes the env's
    spare = getattr(env, "_smac_spare", None)
    if spare is None or any(spare[n].shape != getattr(env, n).shape for n in names[1:]):
        spare = env._smac_spare = {n: torch.empty_like(getattr(env, n)) for n in names[1:]}
    s = SmacState(*[getattr(env, n).data_ptr() for n in names])
    so = SmacState(env.gid.data_ptr(), *[spare[n].data_ptr() for n in names[1:]])
    f32 = dict(device=dev, dtype=torch.float32)
    obs = torch.empty(E, A, sp.obs_dim, **f32)
    state = torch.empty(E, A, sp.state_dim, **f32)
    ava = torch.empty(E, A, env.n_actions, **f32)
    reward = torch.empty(E, **f32)
    dones = torch.empty(E, A, dtype=torch.bool, device=dev)
    flags = torch.empty(3, E, dtype=torch.bool, device=dev)
    scal = torch.empty(4, E, **f32)
    act = None
    if actions is not None:
        act = actions.reshape(E, A)
        act = act if (act.dtype == torch.float32 and act.is_contiguous()) else act.float().contiguous()
    o = SmacOut(act.data_ptr() if act is not None else None, obs.data_ptr(), state.data_ptr(), ava.data_ptr(),
                reward.data_ptr(), dones.data_ptr(), flags[0].data_ptr(), flags[1].data_ptr(), flags[2].data_ptr(),
                scal[0].data_ptr(), scal[1].data_ptr(), scal[2].data_ptr(), scal[3].data_ptr())
    check(lib().mdl_smac_env(ctypes.byref(c), ctypes.byref(s), ctypes.byref(so), ctypes.byref(o), _stream()),
          "smac_env")
    for n in names[1:]:
        cur = getattr(env, n)
        setattr(env, n, spare[n])
        spare[n] = cur
    info = {"won": flags[0], "lost": flags[1], "bad_transition": flags[2], "battles_won": scal[2],
            "battles_game": scal[3], "dead_allies": scal[0], "dead_enemies": scal[1]}
    return obs, state, ava, reward, dones, info
