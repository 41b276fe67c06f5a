# queue tests after CPU-route batches close when a completion thread idles; one-request latency (queue vs drop-in)
set -o pipefail
O=gpurun_out/lat
mkdir -p $O
make -s -C tests/c queue_bench || exit 1
timeout -k 10 900 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_fuzz.py tests/test_gpu_update_ptrs.py tests/test_c_driver.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pytest.log | head -80; exit $rc; }
for C in 32768 131072 1048576; do
  for mode in "" update device devupdate; do
    QB_LATENCY=1 timeout -k 10 120 build/ctest/queue_bench $C 1 $mode 64 >> $O/latency.log 2>&1 || exit 1
  done
  QB_LATENCY=1 QB_CPU_QUEUE=1 timeout -k 10 120 build/ctest/queue_bench $C 1 >> $O/latency.log 2>&1 || exit 1
done
grep '^{' $O/latency.log
