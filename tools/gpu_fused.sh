#!/bin/bash
# Fused checksum tuning + parity tests for one gpurun call (each step bounded).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_csum.py tests/test_migrate.py tests/test_gpu_graph.py -q -x \
	-p no:cacheprovider > gpurun_out/fused_tests.log 2>&1
rc=$?; tail -3 gpurun_out/fused_tests.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/tune11.jsonl
for n in "" 1 2 4 8; do
	ECG_FUSED_COLS=$n timeout -k 10 240 python tools/tune11.py >> gpurun_out/tune11.jsonl 2> gpurun_out/tune11.err || exit $?
done
cat gpurun_out/tune11.jsonl
