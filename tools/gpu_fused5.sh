#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_csum.py tests/test_migrate.py tests/test_gpu_graph.py -q -x -p no:cacheprovider > gpurun_out/csum_tests.log 2>&1
rc=$?; tail -1 gpurun_out/csum_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_csum.py > gpurun_out/bench_csum.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_rebuild.py > gpurun_out/bench_rebuild.log 2>&1 || exit $?
timeout -k 10 500 python tools/tune12.py > gpurun_out/tune12.json 2> gpurun_out/tune12.err || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/bench_csum.json"))
for k, v in d.items():
    if k.startswith(("enc_", "rec_")):
        print(k, v)
print(open("gpurun_out/tune12.json").read()[:3000])
PY
tail -3 gpurun_out/bench_rebuild.log
