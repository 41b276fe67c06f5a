set -o pipefail
O=gpurun_out/r6h
mkdir -p $O
make -s -C tests/c queue_bench || exit 1
QB_CPU_QUEUE=1 timeout -k 10 300 build/ctest/queue_bench 131072 16 update 32 > $O/qb_cpuqueue.log 2>&1 || exit 1
QB_CPU_QUEUE=1 timeout -k 10 300 build/ctest/queue_bench 131072 16 > $O/qb_cpuqueue_encode.log 2>&1 || exit 1
QB_CPU_QUEUE=1 timeout -k 10 300 build/ctest/queue_bench 1048576 16 update 16 > $O/qb_cpuqueue_1m.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_queue_cpu.py tests/test_c_driver.py tests/test_gpu_parity.py tests/test_gpu_update_ptrs.py tests/test_gpu_multi.py > $O/pytest_queue.log 2>&1 || exit 1
echo ALLDONE
