"""Build the in-tree HIP library for gfx950: every ``*.hip`` in this directory -> ``../_lib/libmatdcml.so``.

Plain ``hipcc`` (no torch headers): each translation unit compiles in seconds and the result is loaded with
ctypes (``ops/kernels.py``).  Objects are cached by content hash under ``_lib/obj``.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
OUT_DIR = os.path.join(os.path.dirname(HERE), "_lib")
OUT = os.path.join(OUT_DIR, os.environ.get("MAT_DCML_LIBNAME", "libmatdcml.so"))
ARCH = os.environ.get("MAT_DCML_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=fast", "-munsafe-fp-atomics",
         "-Wno-unused-result", "-fvisibility=hidden"] + os.environ.get("MAT_DCML_EXTRA_FLAGS", "").split()


# Per-translation-unit scheduler choices, each measured on the 1-GPU bench (rocprofv3 kernel stats,
# scripts/ab_flags2.sh): the AMDGPU register-pressure trackers cut the decoder backward's VGPR spills 76 -> 6 and
# its time 676 -> 635 us per minibatch, but slow the decode kernel (323 -> 333 us), so only that unit uses them.
PER_FILE_FLAGS = {
    "mat_dec_ct_bwd.hip": ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"],
    # ... and the encoder forward (its saved-activation stores spilled 88 -> 63 instructions: 191 -> 178 us per
    # training minibatch, scripts/r4_ab7.sh); the decoder forward measured neutral with them
    "mat_enc_ct.hip": ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"],
    # the SMAC env must round every product / sum like the torch path: hip's __fmul_rn / __fadd_rn are plain
    # operators that -ffp-contract=fast still fuses into FMAs (battle positions drifted by an ulp)
    "smac_env.hip": ["-ffp-contract=off"],
    # MFMA results written straight to VGPRs: by default hipcc accumulates in AGPRs and copies every result to a VGPR
    # for the VALU work that follows (847 v_accvgpr moves per agent step in the one-wave decode, 131 with this form)
    # ... and the max-ILP scheduler for the latency-bound speculative decode (scripts/r5_sched.sh: 256 x 33 150.0 ->
    # 146.7 us, SMAC 135.2 -> 133.0 us, 256 x 129 749 -> 741 us; max-memory-clause and the register-pressure trackers
    # were slower; the training backward / forward measured neutral / slower with max-ilp)
    "mat_decode_wave.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1", "-mllvm", "-amdgpu-sched-strategy=max-ilp"],
    "mat_decode.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"],
}


FWD_TUS = ("mat_enc_ct.hip", "mat_dec_ct.hip")   # the training forward translation units


def _flags(src):
    # A/B variants: extra flags for the training backward / forward translation units only
    extra = os.environ.get("MAT_DCML_BWD_FLAGS", "").split() if src.endswith("_bwd.hip") else []
    if os.path.basename(src) in FWD_TUS:
        extra = os.environ.get("MAT_DCML_FWD_FLAGS", "").split()
    if os.path.basename(src) == "mat_enc_ct.hip":   # A/B: the encoder forward alone
        extra = extra + os.environ.get("MAT_DCML_ENCF_FLAGS", "").split()
    if os.path.basename(src) == "mat_decode_wave.hip":   # A/B: the one-wave / speculative decode
        extra = extra + os.environ.get("MAT_DCML_DECW_FLAGS", "").split()
    per_file = [] if os.environ.get("MAT_DCML_NO_PER_FILE_FLAGS") else PER_FILE_FLAGS.get(os.path.basename(src), [])
    return FLAGS + per_file + extra


def _sources():
    return sorted(os.path.join(HERE, f) for f in os.listdir(HERE) if f.endswith(".hip"))


def _deps(path, seen=None):
    """The translation unit and every local file it #includes (transitively), sorted."""
    seen = set() if seen is None else seen
    if path in seen or not os.path.exists(path):
        return seen
    seen.add(path)
    with open(path) as f:
        for line in f:
            m = re.match(r'\s*#\s*include\s+"([^"]+)"', line)
            if m:
                _deps(os.path.join(os.path.dirname(path), m.group(1)), seen)
    return seen


def _hash(path):
    """Object-cache key: the contents of the unit and its local includes, plus its flags (an edit to one kernel no
    longer rebuilds every other unit)."""
    h = hashlib.sha256()
    for p in [path] + sorted(_deps(path) - {path}):
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(_flags(path)).encode())
    return h.hexdigest()[:16]


def source_hash(src_dir=HERE):
    """Hash of every HIP source / header of ``src_dir`` (names + contents): the identity of the kernel sources a
    library was built from.  Embedded in the library as ``mdl_build_source_hash`` and checked by ``ops/kernels.lib()``
    before anything launches, so a stale ``.so`` shipped next to newer sources can never run silently."""
    h = hashlib.sha256()
    for f in sorted(os.listdir(src_dir)):
        if f.endswith((".h", ".hip")):
            h.update(f.encode() + b"\0")
            with open(os.path.join(src_dir, f), "rb") as fh:
                h.update(fh.read())
            h.update(b"\0")
    return h.hexdigest()[:16]


def flags_hash(srcs=None):
    """Hash of the compile flags of every translation unit (environment-dependent A/B flags included)."""
    h = hashlib.sha256()
    for src in srcs or _sources():
        h.update((os.path.basename(src) + ":" + " ".join(_flags(src)) + "\n").encode())
    return h.hexdigest()[:16]


def _tmp(path):
    """Per-process temporary name next to ``path`` (several ranks may build at once: os.replace of a shared
    ``.tmp`` name could move another process's half-written file into place)."""
    return f"{path}.{os.getpid()}.tmp"


def sidecar(out=None):
    """(source hash, flags hash) recorded next to a built library, or None."""
    try:
        with open((out or OUT) + ".buildinfo") as f:
            sh, fh = f.read().split()
        return sh, fh
    except (OSError, ValueError):
        return None


def _buildinfo(srcs):
    """A one-symbol-pair translation unit carrying the build identity (source hash, flags hash)."""
    sh, fh = source_hash(), flags_hash(srcs)
    os.makedirs(os.path.join(OUT_DIR, "obj"), exist_ok=True)
    obj = os.path.join(OUT_DIR, "obj", f"buildinfo_{sh}_{fh}.o")
    if not os.path.exists(obj):
        cpp = f"{obj[:-2]}.{os.getpid()}.cpp"
        with open(cpp, "w") as f:
            f.write(f'extern "C" __attribute__((visibility("default"))) const char mdl_build_source_hash[] = "{sh}";\n'
                    f'extern "C" __attribute__((visibility("default"))) const char mdl_build_flags_hash[] = "{fh}";\n')
        tmp = _tmp(obj)
        r = subprocess.run([HIPCC, "-O2", "-fPIC", "-c", cpp, "-o", tmp], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {cpp}:\n{r.stderr}")
        os.replace(tmp, obj)
        os.remove(cpp)
    return obj


def _compile(src):
    os.makedirs(os.path.join(OUT_DIR, "obj"), exist_ok=True)
    obj = os.path.join(OUT_DIR, "obj", os.path.basename(src) + "." + _hash(src) + ".o")
    if not os.path.exists(obj):
        tmp = _tmp(obj)
        cmd = [HIPCC, *_flags(src), "-c", src, "-o", tmp]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
        os.replace(tmp, obj)
    return obj


def build(verbose=True, jobs=None):
    srcs = _sources()
    jobs = jobs or min(8, len(srcs)) or 1
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(_compile, srcs))
    objs.append(_buildinfo(srcs))
    tmp = _tmp(OUT)
    cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    os.replace(tmp, OUT)
    # sidecar identity: lets ops/kernels.lib() decide "stale -> rebuild" BEFORE the library is ever dlopen'ed (a
    # dlclose + dlopen of one path can hand back the old image); the embedded symbols stay the authoritative check
    side = _tmp(OUT + ".buildinfo")
    with open(side, "w") as f:
        f.write(f"{source_hash()} {flags_hash(srcs)}\n")
    os.replace(side, OUT + ".buildinfo")
    if verbose:
        print(f"[build] {OUT} <- {', '.join(os.path.basename(s) for s in srcs)}")
    return OUT


def prune():
    """Delete the cached objects the current sources / flags no longer use (content-hashed names accumulate)."""
    keep = {os.path.basename(src) + "." + _hash(src) + ".o" for src in _sources()}
    keep.add(f"buildinfo_{source_hash()}_{flags_hash()}.o")
    d = os.path.join(OUT_DIR, "obj")
    gone = [f for f in os.listdir(d) if f not in keep] if os.path.isdir(d) else []
    for f in gone:
        os.remove(os.path.join(d, f))
    return len(gone)


if __name__ == "__main__":
    build()
    if "--prune" in sys.argv[1:]:
        print(f"[build] pruned {prune()} stale cached objects")
    sys.exit(0)
