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


# Performance guards: a bound is 1.25x a recorded measurement, and the measured value is the MEDIAN of
# several timed windows, so the run-to-run jitter of a shared or throttled MI355X does not fail a guard.
GUARD_MARGIN = 1.25


def median_us(fn, iters=10, windows=5, warm=3):
    """Median over ``windows`` hipEvent windows of ``iters`` back-to-back calls: microseconds per call."""
    import torch
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(windows):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / iters * 1e3)
    return sorted(ts)[len(ts) // 2]
