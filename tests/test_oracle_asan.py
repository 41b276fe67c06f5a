"""The oracle's own memory safety: tests/test_oracle.py (every restated
function, the recovery codec over every erasure pattern of every class, the
parity-first quirk) run against an AddressSanitizer/UBSan build of
libecg_oracle.so (oracle/Makefile `asan`).  A checker that reads past its
buffers could agree with anything; this keeps it honest."""
import os
import subprocess
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def test_oracle_suite_under_asan():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
    libasan = subprocess.run(["gcc", "-print-file-name=libasan.so"], check=True, capture_output=True,
                             text=True).stdout.strip()
    assert os.path.isabs(libasan), libasan
    env = dict(os.environ, LD_PRELOAD=libasan, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               ECG_ORACLE_LIB=os.path.join(ROOT, "oracle", "build", "libecg_oracle_asan.so"))
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_oracle.py")], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "passed" in r.stdout and "ERROR: AddressSanitizer" not in r.stderr
