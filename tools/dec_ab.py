"""Headline decode geometry A/B: the EC_4P2 1 MiB x 1024 in-place {d0,d1}
recovery (BASELINE configs[1], the bench's decode launch) under every launch
order x blocks-per-CU cap, beside the headline encode, timed in interleaved
rounds like bench.py (time_interleaved).  One JSON line per geometry, ms of
the median launch.  Results never depend on the geometry (include/ecg.h);
this only asks whether the decode's 2.6 % gap to the encode is a launch-shape
effect.  Bench infrastructure.
usage: python tools/dec_ab.py [iters]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from bench import fill_device, time_interleaved  # noqa: E402
from daos_amd import ecg  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 9
    k, p, C, S = 4, 2, 1 << 20, 1024
    ctx = ecg.Context(0)
    ctx.set_autotune(0)
    data = ctx.alloc(S * k * C)
    par = ctx.alloc(p * (S * C + 4096))
    stripes = ctx.alloc(S * (k + p) * C)
    fill_device(ctx, data, S * k * C, 1)
    fill_device(ctx, stripes, S * (k + p) * C, 2)
    ctx.sync()

    def enc():
        ctx.encode(k, p, C, S, data.ptr, k * C, par.ptr, S * C + 4096, C)

    def dec():
        ctx.recover(k, p, C, S, stripes.ptr, (k + p) * C, [0, 1])

    for order in (0, 1, 2, 3):
        for cap in (0, 2, 3, 4, 6, 8):
            ctx.set_order(order)
            ctx.set_wg_per_cu(cap)
            e, d = time_interleaved(ctx, [enc, dec], iters)
            print(json.dumps({"order": order, "wg_per_cu": cap, "enc_ms": round(e, 4), "dec_ms": round(d, 4),
                              "dec_over_enc": round(d / e, 4)}), flush=True)
    data.free()
    par.free()
    stripes.free()
    ctx.close()


if __name__ == "__main__":
    main()
