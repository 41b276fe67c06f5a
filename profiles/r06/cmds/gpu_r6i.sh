set -o pipefail
O=gpurun_out/r6i
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_update_ptrs.py tests/test_c_driver.py -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
