#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_c_driver.py -q -x -p no:cacheprovider > gpurun_out/stage_tests.log 2>&1
rc=$?; tail -2 gpurun_out/stage_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_pcie.py > gpurun_out/pcie.log 2>&1 || exit $?
grep -E '^\{' gpurun_out/pcie.log | cut -c1-900
timeout -k 10 300 python bench.py --workload rebuild_stream_8p2 --steps 5 --warmup 1 > gpurun_out/host.log 2>&1 || exit $?
grep -oE '"value": [0-9.]+|"frac_of_h2d": [0-9.]+' gpurun_out/host.log
bash tools/gpu_run.sh qbench dropin > gpurun_out/qd.log 2>&1 || exit $?
cat gpurun_out/qbench.jsonl | cut -c1-300
cat gpurun_out/bench_dropin.jsonl | cut -c1-300
