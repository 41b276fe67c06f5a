#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -x -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/tune11.jsonl
for n in "" "" 3 6; do
	ECG_FUSED_COLS=$n timeout -k 10 240 python tools/tune11.py >> gpurun_out/tune11.jsonl 2> gpurun_out/tune11.err || exit $?
done
cat gpurun_out/tune11.jsonl
timeout -k 10 300 python tools/bench_csum.py > gpurun_out/bench_csum.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_rebuild.py > gpurun_out/bench_rebuild.log 2>&1 || exit $?
tail -3 gpurun_out/bench_rebuild.log
