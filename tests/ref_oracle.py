"""Import the read-only reference as a test oracle (SURVEY.md §4.2 harness).

The reference imports cleanly on CPU once ``absl.flags``, ``wandb``, ``tensorboardX`` and ``setproctitle``
are stubbed; its env reads ``data/`` relative to the CWD, so callers chdir into a scratch dir holding a
``data`` symlink.  Every test using this skips when ``/root/reference`` is absent (e.g. on the GPU box).
"""
import contextlib
import os
import sys
import types

REF = os.environ.get("MAT_DCML_REFERENCE", "/root/reference")


def available():
    return os.path.isdir(os.path.join(REF, "mat_src"))


def install_stubs():
    if "absl" not in sys.modules:
        absl = types.ModuleType("absl")
        flags = types.ModuleType("absl.flags")
        flags.FLAGS = lambda *a, **k: None
        absl.flags = flags
        sys.modules["absl"] = absl
        sys.modules["absl.flags"] = flags
    for name in ("wandb", "setproctitle"):
        if name not in sys.modules:
            m = types.ModuleType(name)
            m.setproctitle = lambda *a, **k: None
            m.init = lambda *a, **k: None
            m.log = lambda *a, **k: None
            sys.modules[name] = m
    if "tensorboardX" not in sys.modules:
        tb = types.ModuleType("tensorboardX")

        class SummaryWriter:
            def __init__(self, *a, **k):
                pass

            def add_scalars(self, *a, **k):
                pass

            def export_scalars_to_json(self, *a, **k):
                pass

            def close(self):
                pass
        tb.SummaryWriter = SummaryWriter
        sys.modules["tensorboardX"] = tb
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    for p in (os.path.join(REF, "mat_src"), REF):
        if p not in sys.path:
            sys.path.insert(0, p)


@contextlib.contextmanager
def ref_cwd(tmp_path):
    """chdir into tmp_path with a data -> reference/data symlink."""
    link = os.path.join(str(tmp_path), "data")
    if not os.path.exists(link):
        os.symlink(os.path.join(REF, "data"), link)
    old = os.getcwd()
    os.chdir(str(tmp_path))
    try:
        yield
    finally:
        os.chdir(old)
