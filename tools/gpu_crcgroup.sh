#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_csum.py tests/test_migrate.py tests/test_gpu_sgl.py -q -x -p no:cacheprovider > gpurun_out/csum_tests.log 2>&1
rc=$?; tail -4 gpurun_out/csum_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_csum.py > gpurun_out/bench_csum.log 2>&1 || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/bench_csum.json"))
for k, v in d.items():
    if k.startswith(("crc", "adler", "enc_8p2")):
        print(k, v)
PY
