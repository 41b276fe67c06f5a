# queue after: one update stream per device, scratch grown in steps
set -o pipefail
mkdir -p gpurun_out/r6g
make -s -C tests/c queue_bench || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_update_ptrs.py tests/test_gpu_parity.py -k "queue or update" -x -q --timeout 180 --timeout-method thread > gpurun_out/r6g/t.log 2>&1 || { tail -20 gpurun_out/r6g/t.log; exit 1; }
tail -2 gpurun_out/r6g/t.log
for C in 131072 1048576; do
  for rep in 1 2; do
    timeout -k 10 300 build/ctest/queue_bench $C 16 device 64 >> gpurun_out/r6g/qb.log 2>&1 || exit 1
    timeout -k 10 300 build/ctest/queue_bench $C 16 devupdate 64 >> gpurun_out/r6g/qb.log 2>&1 || exit 1
  done
done
QB_VERIFY=1 timeout -k 10 120 build/ctest/queue_bench 131072 16 devupdate 16 >> gpurun_out/r6g/qb.log 2>&1 || exit 1
cat gpurun_out/r6g/qb.log
echo ALLDONE
