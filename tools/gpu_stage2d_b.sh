#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -x -p no:cacheprovider -k "queue or host or isal" > gpurun_out/stage_tests.log 2>&1
rc=$?; tail -2 gpurun_out/stage_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_run.sh qbench dropin > gpurun_out/qd.log 2>&1 || exit $?
cat gpurun_out/qbench.jsonl | cut -c1-250
cat gpurun_out/bench_dropin.jsonl | cut -c1-400
