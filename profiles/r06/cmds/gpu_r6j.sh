# full GPU suite on the fetch-kernel + placement-cache build; queue timing with the placement cache on / off
set -o pipefail
O=gpurun_out/r6j
mkdir -p $O
make -s -C tests/c queue_bench || exit 1
timeout -k 10 1000 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
rc=$?; tail -5 $O/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
for rep in 1 2; do
  for ttl in 0 1000; do
    for mode in devupdate device; do
      echo "== ECG_PLACE_CACHE_US=$ttl $mode" >> $O/qt.log
      ECG_PLACE_CACHE_US=$ttl LD_LIBRARY_PATH=qt_tmp timeout -k 10 300 build/ctest/queue_bench 131072 16 $mode 64 >> $O/qt.log 2>&1 || exit 1
    done
  done
done
cat $O/qt.log
