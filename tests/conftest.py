import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mat_dcml_amd.ops import kernels
    if not os.path.exists(kernels.LIB_PATH):
        from mat_dcml_amd.csrc.build import build
        build()
    return torch.device("cuda:0")


def perf_record(name, value, bound, unit="us"):
    """Print a GPU performance-guard measurement and append it to gpurun_out/perf_guards.jsonl (merged back from the
    GPU box), so every GPU run leaves the measured value next to its bound."""
    import json
    import time
    line = {"name": name, "value": round(float(value), 3), "bound": bound, "unit": unit, "time": time.time()}
    print(f"[perf] {name}: {value:.3f} {unit} (bound {bound} {unit})")
    try:
        d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "perf_guards.jsonl"), "a") as f:
            f.write(json.dumps(line) + "\n")
    except OSError:
        pass
