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
