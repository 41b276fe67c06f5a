#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for parts in 3 0; do
	ECG_ENC_H2D_PARTS=$parts timeout -k 10 300 python tools/bench_pcie.py > gpurun_out/pcie_$parts.log 2>&1 || exit $?
	echo "parts=$parts"; grep -E '^\{' gpurun_out/pcie_$parts.log | cut -c1-330
done
