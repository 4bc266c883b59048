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


def install_gym_stub():
    """Minimal ``gym`` for the reference MPE env (``environment.py`` / ``multi_discrete.py``): only the space
    classes and ``gym.Env`` it subclasses.  gym itself is not installed."""
    if "gym" in sys.modules:
        return
    import numpy as np
    gym = types.ModuleType("gym")
    spaces = types.ModuleType("gym.spaces")
    envs = types.ModuleType("gym.envs")
    reg = types.ModuleType("gym.envs.registration")

    class Space:
        pass

    class Discrete(Space):
        def __init__(self, n):
            self.n = n

    class Box(Space):
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.low, self.high, self.shape, self.dtype = low, high, shape, dtype

    class Tuple(Space):
        def __init__(self, spaces_):
            self.spaces = spaces_

    gym.Env, gym.Space = type("Env", (), {}), Space
    spaces.Discrete, spaces.Box, spaces.Tuple = Discrete, Box, Tuple
    reg.EnvSpec = type("EnvSpec", (), {})
    gym.spaces, gym.envs, envs.registration = spaces, envs, reg
    sys.modules.update({"gym": gym, "gym.spaces": spaces, "gym.envs": envs, "gym.envs.registration": reg})


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
