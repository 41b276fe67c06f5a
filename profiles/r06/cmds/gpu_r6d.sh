# full GPU suite + default bench line
set -o pipefail
mkdir -p gpurun_out/r6d
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r6d/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r6d/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r6d/gpu_tests.log
timeout -k 10 900 python -u bench.py > gpurun_out/r6d/bench.log 2>&1 || { tail -30 gpurun_out/r6d/bench.log; exit 1; }
echo ALLDONE
