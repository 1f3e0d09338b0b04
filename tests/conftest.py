"""pytest configuration: the `gpu` marker and shared helpers.

`-m "not gpu"` runs here (no GPU): oracle pinning, host logic, C-ABI symbol checks and the
host build of the device arithmetic (tests/hostsim).  `-m gpu` runs on an MI355X and calls
the HIP engine through the C ABI.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the engine's stream pool follows the hardware queues the process starts with; the tests run
# the configuration bench.py measures (10 queues).  Set before the first HIP call (libmbls never
# changes the environment itself).
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("MBLS_HW_QUEUES", "10")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")


HOSTSIM_SO = os.path.join(ROOT, "tests", "hostsim", "libhostsim.so")
HOSTSIM_SRC = os.path.join(ROOT, "tests", "hostsim", "hostsim.cpp")
CSRC = os.path.join(ROOT, "lambda_ethereum_consensus_amd", "csrc")


def build_hostsim(force=False, so=HOSTSIM_SO, extra=()):
    """Compile the device headers for the host (test-only library); `extra` adds flags (the
    UBSan build of tests/test_sanitizers.py)."""
    deps = [HOSTSIM_SRC] + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hpp")]
    if not force and os.path.exists(so):
        so_m = os.path.getmtime(so)
        if all(os.path.getmtime(d) <= so_m for d in deps):
            return so
    opt = "-O1" if extra else "-O2"
    cmd = ["hipcc", opt, "-fPIC", "-shared", "-std=c++17", *extra, "-I", CSRC, "-o", so, HOSTSIM_SRC]
    subprocess.run(cmd, check=True, timeout=900)
    return so


@pytest.fixture(scope="session")
def hostsim():
    import ctypes

    # MBLS_HOSTSIM_SO: a prebuilt variant (the sanitizer run points it at the UBSan build)
    return ctypes.CDLL(os.environ.get("MBLS_HOSTSIM_SO") or build_hostsim())
