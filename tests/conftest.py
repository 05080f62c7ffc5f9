import os
import sys

# The product's stream layout: bench.py gives the process 8 HIP hardware queues before it touches the GPU (the
# latent-sharded step's RCCL streams would otherwise push the side stream onto the compute stream's queue,
# DESIGN.md section 6).  The GPU tests run under the same setting (set before anything imports torch).
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:  # (the box exports 4)
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

import pytest  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import crosscoder_amd  # noqa: E402,F401  (registers the package under its importable name)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm) GPU; runs through the HIP C-ABI library")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no ROCm device is visible")
    return torch.device("cuda:0")
