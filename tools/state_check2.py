"""EC_16P2 128 KiB x 1024 encode after bench.py's EC_8P2 detail rows
(profiles/r03/tuner_check/): which preceding row makes the capped launch slow.
Sequence per argv: e = the EC_8P2 encode row, d = the decode row, then the
EC_16P2 row, then explicit uncapped / cap-2 blocks on fresh buffers.
usage: python tools/state_check2.py ed|e|d|-.  Bench infrastructure."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402
import bench  # noqa: E402
from tools.state_check import bufs, measure  # noqa: E402


def main():
    ctx = ecg.Context(0)
    seq = sys.argv[1] if len(sys.argv) > 1 else "ed"
    ceil = {"copy": 5700.0, "read": 6800.0, "write": 5900.0}
    pre = [s for s in bench.DETAIL_SHAPES[:2] if (s[5] == "enc" and "e" in seq) or (s[5] == "dec" and "d" in seq)]
    res = {"seq": seq}
    if pre:
        res["pre"] = {k: (v["ms"], v.get("launch_tuner")) for k, v in
                      bench.detail_rows(ctx, ceil, shapes=pre, csum=False).items()}
    r = bench.detail_rows(ctx, ceil, shapes=bench.DETAIL_SHAPES[2:3], csum=False)["EC_16P2_128KiB_encode"]
    res["row16"] = (r["ms"], r.get("launch_tuner"))
    ctx.set_autotune(0)
    res["explicit"] = measure(ctx, bufs(ctx, 7))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
