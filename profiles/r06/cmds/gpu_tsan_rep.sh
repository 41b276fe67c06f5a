# the C driver's device half under ThreadSanitizer, 4 runs (unlocked queue launches, host-cell routes)
set -o pipefail
O=gpurun_out/tsan_rep
mkdir -p $O
make -s -C tests/c || exit 1
for i in 1 2 3; do
  TSAN_OPTIONS="halt_on_error=1 suppressions=$PWD/tests/c/tsan.supp" timeout -k 10 600 setarch $(uname -m) -R build/ctest/test_ecg_c_tsan > $O/dev_$i.log 2>&1 || { echo "run $i failed"; tail -40 $O/dev_$i.log; exit 1; }
  tail -2 $O/dev_$i.log
done
