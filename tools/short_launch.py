"""How much of a short product launch is fixed cost (EC_2P1
128 KiB x 1024 stripes, a ~66 us launch, ran 0.76 of the HBM spec where the
long launches run 0.80).

For EC_2P1 (and EC_8P2 as a control) with 128 KiB cells, client layout, the
launch time is measured over a range of batch sizes S -- back to back on one
stream, HIP events around `reps` launches -- and fitted as T(S) = a + b*S:
b is the streaming cost per stripe (its bytes / b = the asymptotic rate), a
the fixed cost per launch (dispatch of the first blocks, ramp-up, the last
wave's tail, the gap to the next launch).  At S = 1024 the fraction a / T is
what no block order can remove.  The block -> item orders of ecg_set_launch_order
(0 = 2D grid, 1-3 = 1D, 2 and 3 XCD-blocked) are timed at S = 1024 too.

Run under `rocprofv3 --kernel-trace --stats` as well: the kernel durations
there exclude the inter-launch gap, so (events - trace) per launch = the gap,
and the trace's own intercept = ramp + tail inside the kernel.
Prints one JSON line per measurement and a summary line."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--shapes", default="2,1;8,2")
    args = ap.parse_args()
    ctx = ecg.Context(0)
    C = 128 << 10
    sizes = [64, 128, 256, 512, 1024, 2048, 4096, 8192]
    smax = max(sizes)
    summary = {}
    for shape in args.shapes.split(";"):
        k, p = (int(x) for x in shape.split(","))
        data = ctx.alloc(smax * k * C)
        par = ctx.alloc(p * (smax * C + 4096))
        data.fill(0x5A)
        pitch = smax * C + 4096
        st = ctx.stream()
        e0, e1 = ctx.event(), ctx.event()

        def run(S, reps):
            for _ in range(20):
                ctx.encode(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C, st)
            ctx.record(e0, st)
            for _ in range(reps):
                ctx.encode(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C, st)
            ctx.record(e1, st)
            ctx.sync(st)
            return ctx.elapsed_ms(e0, e1) / reps * 1e3      # us per launch

        rows = []
        for S in sizes:
            us = run(S, args.reps)
            byts = S * (k + p) * C
            r = {"shape": f"EC_{k}P{p}", "C": C, "S": S, "us": round(us, 3),
                 "GBps": round(byts / us / 1e3, 1), "frac_spec": round(byts / us / 1e3 / 8000, 4),
                 "kernel": ecg.last_kernel()}
            rows.append(r)
            print(json.dumps(r), flush=True)
        x = np.array([r["S"] for r in rows], float)
        y = np.array([r["us"] for r in rows], float)
        b, a = np.polyfit(x, y, 1)
        per = (k + p) * C
        t1024 = a + b * 1024
        s = {"fixed_us": round(a, 2), "us_per_stripe": round(b, 5),
             "asymptotic_GBps": round(per / b / 1e3, 1), "asymptotic_frac_spec": round(per / b / 1e3 / 8000, 4),
             "S1024_fit_us": round(t1024, 2), "S1024_fixed_share": round(a / t1024, 4),
             "S1024_bound_frac_spec": round(per * 1024 / t1024 / 1e3 / 8000, 4)}
        orders = {}
        for order in (0, 1, 2, 3):
            ctx.set_order(order)
            orders[order] = round(run(1024, args.reps), 3)
        ctx.set_order(0)
        s["S1024_us_by_order"] = orders
        summary[f"EC_{k}P{p}"] = s
        print(json.dumps({"fit": f"EC_{k}P{p}", **s}), flush=True)
        ctx.destroy_event(e0)
        ctx.destroy_event(e1)
        ctx.destroy_stream(st)
        data.free()
        par.free()
    print(json.dumps({"summary": summary}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
