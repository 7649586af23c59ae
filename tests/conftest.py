"""Shared test setup: import paths, the `gpu` marker, in-tree builds."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "dna-kmeres-parallel_amd")
ORACLE = os.path.join(REPO, "oracle")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")
    # build the in-tree libraries once if a fresh checkout lacks them (make is a no-op otherwise)
    if not os.path.exists(os.path.join(PKG, "lib", "libkmc.so")):
        subprocess.run(["make", "-s", "-j8", "-C", PKG], check=True)
    if not os.path.exists(os.path.join(ORACLE, "libkmc_oracle.so")):
        subprocess.run(["make", "-s", "-C", ORACLE, "all"], check=True)
    if os.path.isdir("/root/reference") and not os.path.exists(os.path.join(ORACLE, "_ref", "libref_cpu.so")):
        subprocess.run(["make", "-s", "-C", ORACLE, "ref"], check=True)


@pytest.fixture(scope="session")
def kmc():
    import kmc as _kmc
    return _kmc


@pytest.fixture(scope="session")
def oracle():
    import oracle as _oracle
    return _oracle


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected on a machine without a visible HIP device")
    return torch.device("cuda:0")


@pytest.fixture(autouse=True)
def _dense_status_clear(request):
    """After every GPU test: no dense call of the test left a deferred status in the
    device flag of either library (kmc_dense_status: a k = 8 spill overflow or a
    record of >= 2^31 windows); the tests that raise one on purpose consume it."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import kmc as _kmc
    import torch
    if not torch.cuda.is_available():
        return
    torch.cuda.synchronize()
    dv = torch.cuda.current_device()
    for L in (_kmc._lib, _kmc._diag_lib):
        if L is not None:
            assert L.kmc_dense_status(dv) == 0, "a dense call left a deferred error in kmc_dense_status"
