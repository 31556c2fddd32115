import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
EXAMPLE = os.path.join(ROOT, "tests", "golden", "example")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: longer CPU test")


def _gpu_available():
    try:
        import torch  # noqa: F401
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_available():
        return
    skip = pytest.mark.skip(reason="no HIP device in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def built():
    """Build native artefacts once per session (no-op when up to date)."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "build/libpm_oracle.so"], check=True)
    lib = os.path.join(ROOT, "polymutt_amd", "lib", "libpolymutt.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "polymutt_amd")], check=True)
    return True


@pytest.fixture(scope="session")
def cpu_driver():
    """tests/native/build/cpu_polymutt: the product host driver with the CPU oracle as evaluator."""
    exe = os.path.join(ROOT, "tests", "native", "build", "cpu_polymutt")
    import __graft_entry__
    lib = os.path.join(ROOT, "tests", "native", "build", "libpm_cpu_driver.so")
    nat = os.path.join(ROOT, "tests", "native")
    srcs = [os.path.join(nat, f) for f in os.listdir(nat) if f.endswith((".cpp", ".h"))] + \
        [os.path.join(ROOT, "oracle", f) for f in ("pm_oracle.c", "pm_oracle.h")] + \
        [os.path.join(ROOT, "polymutt_amd", "host", f) for f in os.listdir(os.path.join(ROOT, "polymutt_amd", "host"))]
    if not os.path.exists(exe) or not os.path.exists(lib) or \
            max(os.path.getmtime(s) for s in srcs) > min(os.path.getmtime(exe), os.path.getmtime(lib)):
        __graft_entry__.build_cpu_driver()
    return exe
