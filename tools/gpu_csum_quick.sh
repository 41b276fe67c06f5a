#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_csum.py tests/test_migrate.py -q -x -p no:cacheprovider > gpurun_out/fused_tests.log 2>&1
rc=$?; tail -2 gpurun_out/fused_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_csum.py > gpurun_out/bench_csum.log 2>&1 || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/bench_csum.json"))
for k, v in d.items():
    if k.startswith(("enc_", "rec_")):
        print(k, v["fused_ms"], round(v.get("fused_overhead_vs_encode", v.get("fused_overhead")), 4))
PY
