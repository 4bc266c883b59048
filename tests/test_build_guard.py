"""Native-library staleness guard: ``csrc/build.py`` embeds the source / flags hash of the
build in the library (``mdl_build_source_hash``, ``mdl_build_flags_hash``) and ``ops/kernels.lib()`` refuses or
rebuilds a library whose hash does not match the tree.  CPU only (loading the library needs no GPU)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mat_dcml_amd", "_lib", "libmatdcml.so")

pytestmark = pytest.mark.skipif(not os.path.exists(LIB), reason="native library not built")


def test_shipped_library_matches_tree():
    from mat_dcml_amd.ops import kernels
    L = kernels.lib()
    assert kernels.check_build(L) is None
    assert kernels.BUILD_ID == kernels._build_mod().source_hash()


def test_touched_source_reports_mismatch(tmp_path):
    from mat_dcml_amd.ops import kernels
    L = kernels.lib()
    src = os.path.join(ROOT, "mat_dcml_amd", "csrc")
    dst = tmp_path / "csrc"
    shutil.copytree(src, dst, ignore=shutil.ignore_patterns("__pycache__"))
    assert kernels.check_build(L, src_dir=str(dst)) is None        # an identical copy matches
    with open(dst / "ppo.hip", "a") as f:
        f.write("\n// touched\n")
    why = kernels.check_build(L, src_dir=str(dst))
    assert why is not None and "sources" in why


def test_stale_library_refused_without_hipcc(tmp_path):
    pkg = tmp_path / "mat_dcml_amd"
    shutil.copytree(os.path.join(ROOT, "mat_dcml_amd"), pkg,
                    ignore=shutil.ignore_patterns("__pycache__", "obj", "libmatdcml_*.so"))
    with open(pkg / "csrc" / "rl_ops.hip", "a") as f:
        f.write("\n// touched\n")
    code = ("from mat_dcml_amd.ops import kernels\n"
            "try:\n    kernels.lib()\nexcept RuntimeError as e:\n    print('REFUSED', e)\nelse:\n    print('LOADED')\n")
    env = dict(os.environ, HIPCC="/nonexistent/hipcc", PYTHONPATH=str(tmp_path))
    env.pop("MAT_DCML_LIBNAME", None)
    r = subprocess.run([sys.executable, "-c", code], cwd=str(tmp_path), env=env, capture_output=True, text=True,
                       timeout=300)
    assert "REFUSED stale native library" in r.stdout, r.stdout + r.stderr


FAKE_HIPCC = r'''#!/usr/bin/env python3
# hipcc stand-in for the rebuild test: a unit compile copies the cached object of the same source (any hash), the
# identity unit and the link go to the real hipcc.  Every call is logged.
import json, os, shutil, subprocess, sys
args = sys.argv[1:]
with open(os.environ["FAKE_HIPCC_LOG"], "a") as f:
    f.write(" ".join(os.path.basename(a) for a in args if a.endswith((".hip", ".cpp", ".so")) or ".so." in a) + "\n")
src = [a for a in args if a.endswith(".hip")]
if "-c" in args and src:
    out = args[args.index("-o") + 1]
    shutil.copy(json.loads(os.environ["FAKE_HIPCC_OBJ"])[os.path.basename(src[0])], out)
    sys.exit(0)
sys.exit(subprocess.call(["/opt/rocm/bin/hipcc"] + args))
'''


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc for the link")
def test_concurrent_ranks_rebuild_stale_library_once(tmp_path):
    """N ranks that find a stale library at once must rebuild it ONCE (file lock, re-check under it) and
    every rank must then load the fresh library (no dlclose / dlopen of a path whose old image may stay mapped)."""
    import json
    from mat_dcml_amd.ops import kernels
    b = kernels._build_mod()
    obj = {os.path.basename(s): os.path.join(b.OUT_DIR, "obj", os.path.basename(s) + "." + b._hash(s) + ".o")
           for s in b._sources()}   # the default build's cached objects of the untouched tree
    if not all(os.path.exists(o) for o in obj.values()):
        pytest.skip("no cached objects")
    obj = json.dumps(obj)
    pkg = tmp_path / "mat_dcml_amd"
    shutil.copytree(os.path.join(ROOT, "mat_dcml_amd"), pkg,
                    ignore=shutil.ignore_patterns("__pycache__", "obj", "libmatdcml_*.so"))
    with open(pkg / "csrc" / "rl_ops.hip", "a") as f:
        f.write("\n// touched\n")
    fake = tmp_path / "hipcc"
    fake.write_text(FAKE_HIPCC)
    fake.chmod(0o755)
    log = tmp_path / "hipcc.log"
    code = ("from mat_dcml_amd.ops import kernels\n"
            "kernels.lib()\nprint('LOADED', kernels.BUILD_ID)\n")
    env = dict(os.environ, HIPCC=str(fake), PYTHONPATH=str(tmp_path), FAKE_HIPCC_LOG=str(log), FAKE_HIPCC_OBJ=obj)
    env.pop("MAT_DCML_LIBNAME", None)
    procs = [subprocess.Popen([sys.executable, "-c", code], cwd=str(tmp_path), env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for _ in range(3)]
    outs = [p.communicate(timeout=600)[0] for p in procs]
    want = subprocess.run([sys.executable, "-c", "import sys; sys.path.insert(0, 'mat_dcml_amd/csrc'); import build; "
                           "print(build.source_hash())"], cwd=str(tmp_path), capture_output=True, text=True).stdout.strip()
    for o in outs:
        assert f"LOADED {want}" in o, o
    assert sum(o.count("rebuilding") for o in outs) == 1, outs
    links = [l for l in log.read_text().splitlines() if ".so" in l]
    assert len(links) == 1, log.read_text()


def test_missing_lib_dir_reaches_the_build(tmp_path):
    """on a fresh checkout nothing under ``_lib/`` exists; ``lib()`` must create the directory for its
    build lock and get as far as the build (here a failing stand-in hipcc) instead of dying on the lock file."""
    pkg = tmp_path / "mat_dcml_amd"
    shutil.copytree(os.path.join(ROOT, "mat_dcml_amd"), pkg, ignore=shutil.ignore_patterns("__pycache__", "_lib"))
    fake = tmp_path / "hipcc"
    fake.write_text("#!/bin/sh\necho fake-hipcc-called >&2\nexit 1\n")
    fake.chmod(0o755)
    code = ("from mat_dcml_amd.ops import kernels\n"
            "try:\n    kernels.lib()\nexcept FileNotFoundError as e:\n    print('LOCKFAIL', e)\n"
            "except Exception as e:\n    print('BUILDFAIL', type(e).__name__)\nelse:\n    print('LOADED')\n")
    env = dict(os.environ, HIPCC=str(fake), PYTHONPATH=str(tmp_path))
    env.pop("MAT_DCML_LIBNAME", None)
    r = subprocess.run([sys.executable, "-c", code], cwd=str(tmp_path), env=env, capture_output=True, text=True,
                       timeout=300)
    assert "LOCKFAIL" not in r.stdout, r.stdout + r.stderr
    assert (pkg / "_lib").is_dir()
    assert "rebuilding" in r.stdout and "BUILDFAIL" in r.stdout, r.stdout + r.stderr


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")
def test_kernel_arg_structs_match_ctypes(tmp_path):
    """The ctypes mirrors of the kernel argument structs (EncP / DecP / PPOArgs / AdamArgs / UpdArgs) must have the C
    structs' sizes and field offsets: a field appended on one side only shifts every later pointer (round 6 grew
    EncP / DecP / PPOArgs).  The C side is compiled for the host from the library's own headers."""
    import ctypes
    from mat_dcml_amd.ops import kernels, mat_train, ppo_fused
    csrc = os.path.join(ROOT, "mat_dcml_amd", "csrc")
    src = tmp_path / "sz.hip"
    # the PPO / Adam / update structs live in ppo.hip: include it (its kernels compile for the host side as stubs)
    src.write_text(f'''#include <cstdio>
#include <cstddef>
#include "{csrc}/mat_train_common.h"
#include "{csrc}/ppo.hip"
int main() {{
  printf("EncP %zu %zu %zu\\n", sizeof(EncP), offsetof(EncP, g_mode), offsetof(EncP, sidx));
  printf("DecP %zu %zu %zu\\n", sizeof(DecP), offsetof(DecP, g_mode), offsetof(DecP, sidx));
  printf("PPOArgs %zu %zu %zu\\n", sizeof(PPOArgs), offsetof(PPOArgs, n_lp), offsetof(PPOArgs, adv_eps));
  printf("AdamArgs %zu %zu %zu\\n", sizeof(AdamArgs), offsetof(AdamArgs, clip), offsetof(AdamArgs, npart));
  printf("UpdArgs %zu %zu %zu %zu\\n", sizeof(UpdArgs), offsetof(UpdArgs, a), offsetof(UpdArgs, bar), offsetof(UpdArgs, ga_wg));
  printf("GatherArgs %zu %zu %zu\\n", sizeof(GatherArgs), offsetof(GatherArgs, idx), offsetof(GatherArgs, eps));
}}
''')
    exe = tmp_path / "sz"
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-std=c++17", "-O0", "--offload-arch=gfx950", str(src), "-o", str(exe)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    # the host binary only prints sizeof / offsetof (no GPU needed)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60).stdout
    got = {l.split()[0]: tuple(int(x) for x in l.split()[1:]) for l in out.strip().splitlines()}
    want = {
        "EncP": (ctypes.sizeof(mat_train.EncP), mat_train.EncP.g_mode.offset, mat_train.EncP.sidx.offset),
        "DecP": (ctypes.sizeof(mat_train.DecP), mat_train.DecP.g_mode.offset, mat_train.DecP.sidx.offset),
        "PPOArgs": (ctypes.sizeof(ppo_fused.PPOArgs), ppo_fused.PPOArgs.n_lp.offset, ppo_fused.PPOArgs.adv_eps.offset),
        "AdamArgs": (ctypes.sizeof(ppo_fused.AdamArgs), ppo_fused.AdamArgs.clip.offset, ppo_fused.AdamArgs.npart.offset),
        "UpdArgs": (ctypes.sizeof(mat_train.UpdArgs), mat_train.UpdArgs.a.offset, mat_train.UpdArgs.bar.offset,
                    mat_train.UpdArgs.ga_wg.offset),
        "GatherArgs": (ctypes.sizeof(kernels.GatherArgs), kernels.GatherArgs.idx.offset, kernels.GatherArgs.eps.offset),
    }
    assert got == want, (got, want)
