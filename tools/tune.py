"""Kernel tuning sweep on the GPU box (one process, interleaved rounds).

For each shape: every tuning variant (launch variant 16+v, see ecg.h) x grid
shape, R rounds interleaved so DVFS/device drift hits all variants alike
(cdna_hip_programming.md §5.4 rule 24).  Also measures this box's streaming
copy / read / write rates.  Writes gpurun_out/tune.json.
"""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from daos_amd import ecg  # noqa: E402


def main():
    rounds = int(os.environ.get("TUNE_ROUNDS", "5"))
    ctx = ecg.Context(0)
    a, b = ctx.event(), ctx.event()

    def timed(fn):
        ctx.record(a)
        fn()
        ctx.record(b)
        return ctx.elapsed_ms(a, b)

    out = {"stream": {}, "shapes": {}}
    n = 4 << 30
    x, y = ctx.alloc(n), ctx.alloc(n)
    x.fill(7)
    for mode, name, nbytes in ((0, "copy", 2 * n), (1, "read", n), (2, "write", n)):
        ms = []
        for _ in range(10):
            ms.append(timed(lambda: ctx.copy_kernel(y.ptr, x.ptr, n, mode)))
        ms.sort()
        out["stream"][name] = round(nbytes / ms[len(ms) // 2] / 1e6, 1)
    x.free()
    y.free()
    print("stream GB/s:", out["stream"], flush=True)

    shapes = [
        ("4P2_enc_client", 4, 2, 1 << 20, 1024, "enc_client"),
        ("4P2_dec_d0d1", 4, 2, 1 << 20, 1024, "dec"),
        ("8P2_enc_client", 8, 2, 1 << 20, 512, "enc_client"),
        ("8P2_enc_inplace", 8, 2, 1 << 20, 512, "enc_inplace"),
        ("16P2_enc_128K", 16, 2, 128 << 10, 1024, "enc_inplace"),
    ]
    variants = [0] + [16 + v for v in range(1, 8)]
    grids = [(0, 0), (256, 16), (256, 64), (256, 128), (128, 64), (64, 256), (32, 256)]
    for name, k, p, C, S, mode in shapes:
        st = (k + p) * C
        buf = ctx.alloc(S * st)
        par = ctx.alloc(p * S * C)
        buf.fill(0x5A)
        if mode == "enc_client":
            fn = lambda: ctx.encode(k, p, C, S, buf.ptr, k * C, par.ptr, S * C, C)
            alg = (k + p) * C * S
        elif mode == "enc_inplace":
            fn = lambda: ctx.encode(k, p, C, S, buf.ptr, st, buf.ptr + k * C, C, st)
            alg = (k + p) * C * S
        else:
            fn = lambda: ctx.recover(k, p, C, S, buf.ptr, st, [0, 1])
            alg = (k + 2) * C * S
        res = {}
        for r in range(rounds):
            for v in variants:
                for gx, gy in grids:
                    if v != 0 and (gx, gy) != (0, 0) and k == 16:
                        continue
                    ctx.set_launch(gx, gy, v)
                    try:
                        ms = timed(fn)
                    except ecg.EcgError as e:
                        res.setdefault(f"v{v}_g{gx}x{gy}", []).append(str(e))
                        continue
                    res.setdefault(f"v{v}_g{gx}x{gy}", []).append(ms)
        ctx.set_launch(0, 0, 0)
        summ = {}
        for key, ms in res.items():
            ms = [m for m in ms if isinstance(m, float)]
            if not ms:
                continue
            ms.sort()
            med = ms[len(ms) // 2]
            summ[key] = {"ms": round(med, 4), "GBps": round(alg / med / 1e6, 1)}
        best = sorted(summ.items(), key=lambda kv: kv[1]["ms"])[:6]
        out["shapes"][name] = {"alg_bytes": alg, "default": summ.get("v0_g0x0"), "best": best, "all": summ}
        print(name, "default", summ.get("v0_g0x0"), "best", best[:4], flush=True)
        buf.free()
        par.free()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "tune.json"), "w"), indent=1)
    ctx.close()


if __name__ == "__main__":
    t0 = time.time()
    main()
    print(f"tune done in {time.time() - t0:.1f}s")
