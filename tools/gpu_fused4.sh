#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rm -f gpurun_out/tune11.jsonl
for n in "" 1 2 4 8 16 32; do
	ECG_FUSED_COLS=$n timeout -k 10 240 python tools/tune11.py >> gpurun_out/tune11.jsonl 2> gpurun_out/tune11.err || exit $?
done
cat gpurun_out/tune11.jsonl
