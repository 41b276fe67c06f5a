#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 5 --no-cpu > gpurun_out/bench_a.log 2>&1 || exit $?
python - <<'PY'
import json
l = [x for x in open("gpurun_out/bench_a.log") if x.startswith("{")][0]
d = json.loads(l)["detail"]
print("bench", d["EC_8P2_1MiB_encode"]["ms"], d["EC_8P2_1MiB_encode_crc32_32KiB_fused"], d["EC_8P2_1MiB_rebuild_parity_shard_crc32"]["ms"])
PY
timeout -k 10 240 python tools/tune11.py > gpurun_out/tune11_a.log 2>&1 || exit $?
cut -c1-400 gpurun_out/tune11_a.log
ECG_FUSED_COLS=8 timeout -k 10 300 python bench.py --steps 5 --no-cpu > gpurun_out/bench_b.log 2>&1 || exit $?
python - <<'PY'
import json
l = [x for x in open("gpurun_out/bench_b.log") if x.startswith("{")][0]
d = json.loads(l)["detail"]
print("bench cols8", d["EC_8P2_1MiB_encode"]["ms"], d["EC_8P2_1MiB_encode_crc32_32KiB_fused"], d["EC_8P2_1MiB_rebuild_parity_shard_crc32"]["ms"])
PY
