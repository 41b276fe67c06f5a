"""EC_16P2 128 KiB x 1024 encode: the launch tuner's decided launches vs
an explicit cap of the same value, in one fresh process, several blocks of
back-to-back launches each (profiles/r03/tuner_check/).  usage: python
tools/state_check3.py.  Bench infrastructure."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402
import bench  # noqa: E402
from tools.state_check import K, P, C, S, bufs  # noqa: E402


def main():
    ctx = ecg.Context(0)
    data, par, pitch = bufs(ctx, 7)

    def enc():
        ctx.encode(K, P, C, S, data.ptr, K * C, par.ptr, pitch, C)

    res = {"auto": [bench.time_kernel(ctx, enc, 11, warm=10)]}
    res["tuner"] = ctx.tune_state(K, P, C, S, K * C, C)
    res["auto"] += [bench.time_kernel(ctx, enc, 15, warm=0) for _ in range(3)]
    ctx.set_wg_per_cu(2)
    res["cap2"] = [bench.time_kernel(ctx, enc, 15, warm=0) for _ in range(3)]
    ctx.set_wg_per_cu(0)
    res["auto_again"] = [bench.time_kernel(ctx, enc, 15, warm=0) for _ in range(3)]
    ctx.set_wg_per_cu(255)
    res["uncapped"] = [bench.time_kernel(ctx, enc, 15, warm=0) for _ in range(3)]
    ctx.set_wg_per_cu(2)
    res["cap2_again"] = [bench.time_kernel(ctx, enc, 15, warm=0) for _ in range(3)]
    print(json.dumps({k: [round(x, 4) for x in v] if k != "tuner" else v for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
