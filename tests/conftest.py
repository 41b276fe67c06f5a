import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs on the MI355X box)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import ref

    ref.lib()
    return ref


@pytest.fixture(scope="session")
def ecglib():
    from daos_amd import ecg

    # ECG_TEST_LIB: run the suite against an experimental build of libecg.so
    # (tools/build_exp.sh) -- A/B candidates must pass parity before timing
    if os.environ.get("ECG_TEST_LIB"):
        ecg.LIB_PATH = os.path.abspath(os.environ["ECG_TEST_LIB"])
    ecg.lib()
    return ecg


@pytest.fixture(scope="session")
def ctx(ecglib):
    if ecglib.device_count() < 1:
        pytest.fail("no gfx950 device visible: GPU tests must run on the MI355X box")
    c = ecglib.Context(0)
    yield c
    c.close()


@pytest.fixture(params=["cpu", "gpu"])
def route(request, ecglib):
    """Host-cell drop-in calls and host-cell queue requests on the product CPU
    path (the default: below the measured crossover) or forced onto the GPU
    staging path (crossover 0); device cells always take the GPU."""
    old = ecglib.dropin_crossover()
    ecglib.set_dropin_crossover((1 << 64) - 1 if request.param == "cpu" else 0)
    yield request.param
    ecglib.set_dropin_crossover(old)
