"""Block -> (stripe, column) order sweep of ecg_mm_kernel (ecg_set_launch_order)
on the shapes that trail the headline: EC_8P2 1 MiB decode {d0,d1} in the
recovery layout, EC_8P2 1 MiB encode and EC_16P2 128 KiB encode in the client
layout, plus the EC_4P2 headline pair.  Median kernel time of 9 launches per
(shape, order), interleaved A/B in one process; outputs of every order are
compared with order 0's on sampled stripes.  -> gpurun_out/tune14.json.
Bench infrastructure (no oracle)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402
from tools.datagen import stripe_bytes  # noqa: E402

PAD = 4096


def main():
    ctx = ecg.Context(0)
    a, b = ctx.event(), ctx.event()

    def timed(fn, reps=9):
        fn()
        ctx.sync()
        ts = []
        for _ in range(reps):
            ctx.record(a)
            fn()
            ctx.record(b)
            ts.append(ctx.elapsed_ms(a, b))
        ts.sort()
        return ts[len(ts) // 2]

    blk = stripe_bytes(256 << 20, 14)
    res = {}
    shapes = (("EC_8P2_1MiB_decode_d0d1", 8, 2, 1 << 20, 512, "dec"),
              ("EC_8P2_1MiB_encode", 8, 2, 1 << 20, 512, "enc"),
              ("EC_16P2_128KiB_encode", 16, 2, 128 << 10, 1024, "enc"),
              ("EC_16P2_128KiB_encode_x4", 16, 2, 128 << 10, 4096, "enc"),
              ("EC_4P2_1MiB_encode", 4, 2, 1 << 20, 1024, "enc"),
              ("EC_4P2_1MiB_decode_d0d1", 4, 2, 1 << 20, 1024, "dec"))
    for name, k, p, C, S, mode in shapes:
        st = (k + p) * C
        buf = ctx.alloc(S * st)
        for off in range(0, S * st, blk.size):
            buf.upload(blk[: min(blk.size, S * st - off)], offset=off)
        par = ctx.alloc(p * (S * C + PAD)) if mode == "enc" else None
        if mode == "enc":
            pitch = S * C + PAD
            fn = lambda: ctx.encode(k, p, C, S, buf.ptr, k * C, par.ptr, pitch, C)      # noqa: E731
            out = lambda s: np.concatenate([par.download(C, offset=r * pitch + s * C) for r in range(p)])  # noqa: E731
            alg = (k + p) * C * S
        else:
            ctx.encode(k, p, C, S, buf.ptr, st, buf.ptr + k * C, C, st)
            fn = lambda: ctx.recover(k, p, C, S, buf.ptr, st, [0, 1])                   # noqa: E731
            out = lambda s: buf.download(2 * C, offset=s * st)                           # noqa: E731
            alg = (k + 2) * C * S
        row = {}
        ref = None
        for rnd in range(2):                   # two interleaved rounds: drift shows up
            for order in (0, 1, 2, 3):
                ctx.set_order(order)
                if mode == "enc":
                    par.fill(0)
                ms = timed(fn)
                key = f"o{order}"
                row.setdefault(key, []).append(round(ms, 4))
                samp = np.concatenate([out(s) for s in (0, S // 3, S - 1)])
                if ref is None:
                    ref = samp
                row[f"{key}_same"] = bool(np.array_equal(samp, ref)) and row.get(f"{key}_same", True)
        ctx.set_order(0)
        for order in range(4):
            best = min(row[f"o{order}"])
            row[f"o{order}_TBps"] = round(alg / best / 1e9, 3)
        res[name] = row
        print(name, json.dumps(row), flush=True)
        buf.free()
        if par is not None:
            par.free()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "tune14.json"), "w"), indent=1)
    ctx.close()


if __name__ == "__main__":
    main()
