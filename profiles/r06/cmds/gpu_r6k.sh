# device batches launched with the queue lock released: queue tests (+ C driver plain/ASan/TSan), call cost on a
# busy stream, queue phase timing (qt_tmp/ = -DECG_QUEUE_TIMING)
set -o pipefail
O=gpurun_out/r6k
mkdir -p $O
make -s -C tests/c queue_bench upd_latency || exit 1
timeout -k 10 900 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_update_ptrs.py tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_fuzz.py tests/test_c_driver.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 build/ctest/upd_latency > $O/upd_latency.log 2>&1 || exit 1
LD_LIBRARY_PATH=qt8 timeout -k 10 120 build/ctest/upd_latency > $O/upd_latency_memcpy.log 2>&1 || exit 1
cat $O/upd_latency*.log
for rep in 1 2; do
  for T in 1 16; do
    for mode in devupdate device; do
      echo "== T=$T $mode" >> $O/qt.log
      LD_LIBRARY_PATH=qt_tmp timeout -k 10 300 build/ctest/queue_bench 131072 $T $mode $((1024 / T)) >> $O/qt.log 2>&1 || exit 1
    done
  done
done
grep -v "timing" $O/qt.log
