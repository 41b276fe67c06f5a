"""Runs the native C driver (tests/c/test_ecg_c.c): the C-ABI exercised from
C, plain, with ASan/UBSan and with ThreadSanitizer on the host code, checked
against the oracle.  Without a GPU only its host-side checks run; under -m
gpu the device paths (concurrent ISA-L calls from 12 pthreads, batched
encode/recover, queue on host cells and on device cells from 4 pthreads) --
plain, ASan/UBSan and TSan.  The TSan build runs with address-space
randomisation off (setarch -R): on the GPU boxes its runtime (gcc 11)
otherwise aborts at start-up on the kernel's high-entropy mmap layout
("unexpected memory mapping"), with or without PIE.  tests/c/tsan.supp
suppresses only reports with a frame in the uninstrumented ROCm runtime."""
import os
import platform
import shutil
import subprocess

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
BIN = os.path.join(ROOT, "build", "ctest")


@pytest.fixture(scope="module")
def cbins():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "c")], check=True)
    return os.path.join(BIN, "test_ecg_c"), os.path.join(BIN, "test_ecg_c_asan"), os.path.join(BIN, "test_ecg_c_tsan")


SUPP = os.path.join(ROOT, "tests", "c", "tsan.supp")


def _run(path, gpu):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:use_sigaltstack=0", UBSAN_OPTIONS="print_stacktrace=1",
               TSAN_OPTIONS=f"halt_on_error=1 suppressions={SUPP}")
    if not gpu:
        env["HIP_VISIBLE_DEVICES"] = ""       # host-only half
    cmd = [path]
    if path.endswith("_tsan") and shutil.which("setarch"):
        cmd = ["setarch", platform.machine(), "-R", path]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS" in r.stdout
    return r.stdout


def test_c_driver_host(cbins):
    for b in cbins:
        _run(b, gpu=False)


@pytest.mark.gpu
def test_c_driver_device(cbins):
    out = _run(cbins[0], gpu=True)
    assert "host-only" not in out


@pytest.mark.gpu
def test_c_driver_device_asan(cbins):
    out = _run(cbins[1], gpu=True)
    assert "host-only" not in out


@pytest.mark.gpu
def test_c_driver_device_tsan(cbins):
    """The device half under ThreadSanitizer: the queue's worker, completion
    threads and update stream with device-cell batches, the multi-device
    shard threads, 12 concurrent ISA-L callers on the GPU path."""
    out = _run(cbins[2], gpu=True)
    assert "host-only" not in out
