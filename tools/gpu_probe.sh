#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for n in "" 8; do
	ECG_FUSED_COLS=$n timeout -k 10 240 python tools/fused_probe.py 2>/dev/null || exit $?
done
