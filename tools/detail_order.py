"""bench.py's detail rows in a fresh process, with (`ceil`) or without
(`noceil`) bench's streaming-ceiling launches before them: what the rows'
launch-tuner decisions and times depend on (profiles/r03/tuner_check/).
usage: python tools/detail_order.py ceil|noceil.  Bench infrastructure."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402
import bench  # noqa: E402


def main():
    ctx = ecg.Context(0)
    mode = sys.argv[1] if len(sys.argv) > 1 else "ceil"
    if mode == "ceil":
        ceil = bench.measured_ceilings(ctx)
    else:
        ceil = {"copy": 5700.0, "read": 6800.0, "write": 5900.0}
    det = bench.detail_rows(ctx, ceil)
    print(mode, json.dumps({k: (v.get("ms"), v.get("launch_tuner")) for k, v in det.items()
                            if "EC_" in k and "crc" not in k and "rebuild" not in k}), flush=True)


if __name__ == "__main__":
    main()
