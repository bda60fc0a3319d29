import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: large sizes")


def _ensure_built():
    lib = os.path.join(ROOT, "syzkaller_amd", "libsyzsig.so")
    orc = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(orc):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "all"], check=True)
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-j8", "-C", ROOT], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a GPU")
    from syzkaller_amd.device import Device

    return Device(0)


GOLDEN = os.path.join(ROOT, "tests", "golden")


def golden_names():
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz"))


def load_golden(name):
    import numpy as np

    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as f:
        return {k: f[k] for k in f.files}
