"""Host-code sanitizer run: the HIP library's host paths under ASan + UBSan, on the CPU.

Builds ``libmatdcml_hostsan.so`` (same sources, ``-Xarch_host -fsanitize=address,undefined``; objects cached by
content hash in ``_lib/obj``) and ``tests/native/host_checks.hip``, then runs the checks: Philox known answers,
decode / training tile geometry invariants over every agent count, and argument validation of the launch entry
points.  GPU-side ASan (xnack+) is not available on this pool; device-side races are covered by the bitwise
determinism harness (``test_gpu_determinism.py``)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
SAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined", "-Xarch_host",
       "-fno-sanitize=function", "-Xarch_host", "-fno-omit-frame-pointer"]


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_host_code_under_asan_ubsan(tmp_path):
    env = dict(os.environ, MAT_DCML_LIBNAME="libmatdcml_hostsan.so", MAT_DCML_EXTRA_FLAGS=" ".join(["-O1", "-g"] + SAN))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "mat_dcml_amd", "csrc", "build.py")], env=env,
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    exe = str(tmp_path / "host_checks")
    r = subprocess.run([HIPCC, "-O1", "-g", "-std=c++17", "--offload-arch=gfx950", *SAN,
                        os.path.join(ROOT, "tests", "native", "host_checks.hip"), "-o", exe, "-ldl"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    run_env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1",
                   UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, os.path.join(ROOT, "mat_dcml_amd", "_lib", "libmatdcml_hostsan.so")], cwd=ROOT,
                       env=run_env, capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "0 failures" in r.stdout
