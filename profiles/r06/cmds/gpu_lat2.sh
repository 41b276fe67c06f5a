# the lone-request tests; one-request latency of the final queue (host CPU route, CPU executor, device cells)
set -o pipefail
O=gpurun_out/lat2
mkdir -p $O
make -s -C tests/c queue_bench || exit 1
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu \
  "tests/test_gpu_parity.py::test_queue_host_cell_alone_closes_at_once" "tests/test_gpu_parity.py::test_queue_device_cell_alone_launches_at_once" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for C in 32768 131072 1048576; do
  for mode in "" update device devupdate; do
    QB_LATENCY=1 timeout -k 10 120 build/ctest/queue_bench $C 1 $mode 64 >> $O/latency.log 2>&1 || exit 1
  done
  QB_LATENCY=1 QB_CPU_QUEUE=1 timeout -k 10 120 build/ctest/queue_bench $C 1 >> $O/latency.log 2>&1 || exit 1
done
grep '^{' $O/latency.log
