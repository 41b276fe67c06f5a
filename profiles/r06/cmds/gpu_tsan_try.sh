set -o pipefail
O=gpurun_out/tsan_try
mkdir -p $O
make -s -C tests/c || exit 1
HIP_VISIBLE_DEVICES="" TSAN_OPTIONS="halt_on_error=1 suppressions=$PWD/tests/c/tsan.supp print_suppressions=1" timeout -k 10 300 setarch $(uname -m) -R build/ctest/test_ecg_c_tsan > $O/host.log 2>&1; echo "host rc=$?"
tail -25 $O/host.log
TSAN_OPTIONS="halt_on_error=1 suppressions=$PWD/tests/c/tsan.supp print_suppressions=1" timeout -k 10 600 setarch $(uname -m) -R build/ctest/test_ecg_c_tsan > $O/dev.log 2>&1; echo "dev rc=$?"
tail -25 $O/dev.log
