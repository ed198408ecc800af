import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")
# extra flags for the host builds of native code the tests compile (tests/native/*.cpp):
# `make asan-test` sets -fsanitize=address,undefined (the process preloads the runtimes)
NATIVE_FLAGS = os.environ.get("GF_NATIVE_SANITIZE", "").split()
BEIJING = (115.5, 117.6, 39.6, 41.1)
QPOINT = (116.414899, 39.920374)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle

    oracle.build()
    return oracle


_BUILD_CHECKED = []


def assert_product_build():
    """The library under test must be the product build: no unit compiled with tuning or
    experiment defines (gf_build_is_product).  GF_TEST_EXPERIMENT=1 lets
    an A/B arm's experiment library be parity-checked explicitly (tools/gpu_ab.sh)."""
    import spatialflink_amd._lib as L

    lib = L.lib()
    info = lib.gf_build_info().decode()
    if os.environ.get("GF_TEST_EXPERIMENT") == "1":
        return info
    assert lib.gf_build_is_product() == 1, f"not the product build: {info} ({L.LIB_PATH})"
    return info


@pytest.fixture(autouse=True)
def _product_build(request):
    """Every gpu-marked test runs against the product library only."""
    if request.node.get_closest_marker("gpu") is not None and not _BUILD_CHECKED:
        _BUILD_CHECKED.append(assert_product_build())
    yield


@pytest.fixture(scope="session")
def gpu():
    """Skip-free on the GPU box: a gpu-marked test must fail loudly if no device is visible."""
    import torch

    assert torch.cuda.is_available(), "gpu test needs a visible HIP device"
    import spatialflink_amd._lib as L

    L.lib()
    return torch.device("cuda", 0)
