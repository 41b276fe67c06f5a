#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python tools/tune12.py > gpurun_out/tune12.json 2> gpurun_out/tune12.err || exit $?
cat gpurun_out/tune12.json
