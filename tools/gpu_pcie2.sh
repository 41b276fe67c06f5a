#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -k "host" -p no:cacheprovider > gpurun_out/host_tests.log 2>&1
rc=$?; tail -2 gpurun_out/host_tests.log; [ $rc -eq 0 ] || exit $rc
for parts in 1 0; do
	ECG_ENC_H2D_PARTS=$parts timeout -k 10 300 python tools/bench_pcie.py > gpurun_out/pcie_$parts.log 2>&1 || exit $?
	echo "parts=$parts"; grep -E '^\{' gpurun_out/pcie_$parts.log | cut -c1-700
	ECG_ENC_H2D_PARTS=$parts timeout -k 10 300 python bench.py --workload rebuild_stream_8p2 --steps 5 --warmup 1 > gpurun_out/host_$parts.log 2>&1 || exit $?
	grep -oE '"value": [0-9.]+' gpurun_out/host_$parts.log
done
