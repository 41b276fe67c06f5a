# table upload by fetch kernel (qt_tmp/) vs hipMemcpyAsync (qt8/, -DECG_TABLE_MEMCPY); both -DECG_QUEUE_TIMING
set -o pipefail
O=gpurun_out/fetch
mkdir -p $O
make -s -C tests/c queue_bench upd_latency || exit 1
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_update_ptrs.py tests/test_gpu_ptrs.py tests/test_gpu_sgl.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for lib in qt_tmp qt8; do
  LD_LIBRARY_PATH=$lib timeout -k 10 120 build/ctest/upd_latency > $O/upd_latency_$lib.log 2>&1 || exit 1
done
for rep in 1 2; do
  for lib in qt_tmp qt8; do
    for T in 1 16; do
      for mode in devupdate device; do
        echo "== $lib $mode T=$T" >> $O/qt.log
        LD_LIBRARY_PATH=$lib timeout -k 10 300 build/ctest/queue_bench 131072 $T $mode $((1024 / T)) >> $O/qt.log 2>&1 || exit 1
      done
    done
  done
done
cat $O/upd_latency_*.log
grep -v "^{" $O/qt.log | head -0
cat $O/qt.log
