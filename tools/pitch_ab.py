"""EC_16P2 128 KiB x 1024 encode with the data cells at padded pitches (cell j
of stripe s at s*stride + j*pitch, pitch = C + pad, stride = k*pitch): does the
power-of-two cell stride of the client layout [S][k][C] cost channel
parallelism?  Tuner off, uncapped and at 2 blocks per CU; median of 30
back-to-back launches after 40.  -> gpurun_out/pitch_ab.json.  Bench
infrastructure."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("ECG_AUTOTUNE", "0")
from daos_amd import ecg  # noqa: E402


def timed(ctx, fn, iters=30, warm=40):
    for _ in range(warm):
        fn()
    ctx.sync()
    evs = [ctx.event() for _ in range(iters + 1)]
    ctx.record(evs[0])
    for i in range(iters):
        fn()
        ctx.record(evs[i + 1])
    ms = sorted(ctx.elapsed_ms(evs[i], evs[i + 1]) for i in range(iters))
    for e in evs:
        ctx.destroy_event(e)
    return ms[iters // 2]


def main():
    ctx = ecg.Context(0)
    k, p, C, S = 16, 2, 128 << 10, 1024
    coef = ecg.cauchy1(k, p)[k:]
    res = {}
    for pad in (0, 256, 4096, 65536, 128 << 10):
        pitch = C + pad
        stride = k * pitch
        data = ctx.alloc(S * stride + 64)
        data.fill(0x3C)
        prow = S * C + 4096
        par = ctx.alloc(p * prow)
        fn = lambda: ctx.matmul(coef, C, S, data.ptr, [j * pitch for j in range(k)], stride, par.ptr,
                                [r * prow for r in range(p)], C, 0)
        for cap in (0, 2):
            ctx.set_wg_per_cu(cap)
            ms = timed(ctx, fn)
            alg = (k + p) * C * S
            res[f"pad{pad}_cap{cap}"] = {"ms": round(ms, 4), "alg_GBps": round(alg / ms / 1e6, 1),
                                         "kernel": ecg.last_kernel()}
            print(f"pad {pad} cap {cap}", res[f"pad{pad}_cap{cap}"], flush=True)
        ctx.set_wg_per_cu(0)
        data.free()
        par.free()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "pitch_ab.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
