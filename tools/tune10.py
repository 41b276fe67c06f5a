"""(Experiment, round 1; the half-width kernel was measured and removed --
profiles/r01/tune10_half_width.json)  Full-width (16 B per
lane, 4 KiB columns) vs half-width (8 B per lane, 2 KiB columns, variant 5)
product kernels at EC_8P2 / EC_16P2, client and
recovery layouts; the half-width outputs are checked byte for byte against
the full-width ones.  -> gpurun_out/tune10.json."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from daos_amd import ecg  # noqa: E402
from tools.datagen import stripe_bytes  # noqa: E402


def main():
    ctx = ecg.Context(0)
    a, b = ctx.event(), ctx.event()

    def timed(fn, reps=9):
        fn()
        ctx.sync()
        ts = []
        for _ in range(reps):
            ctx.record(a); fn(); ctx.record(b)
            ts.append(ctx.elapsed_ms(a, b))
        ts.sort()
        return ts[len(ts) // 2]

    blk = stripe_bytes(256 << 20, 11)
    res = {}
    for k, p, C, S in ((16, 2, 128 << 10, 1024), (16, 2, 1 << 20, 256), (8, 2, 1 << 20, 512),
                       (8, 2, 128 << 10, 2048), (16, 3, 128 << 10, 1024)):
        tag = f"{k}p{p}_{C >> 10}K"
        data = ctx.alloc(S * k * C)
        for off in range(0, S * k * C, blk.size):
            data.upload(blk[: min(blk.size, S * k * C - off)], offset=off)
        pitch = S * C + 4096
        par = ctx.alloc(p * pitch)
        st = ctx.alloc(S * (k + p) * C)
        st.fill(0x37)
        alg = (k + p) * C * S
        row = {}
        outs = {}
        for var in (0, 5):
            ctx.set_launch(0, 0, var)
            ms = timed(lambda: ctx.encode(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C))
            row[f"client_v{var}_GBps"] = round(alg / ms / 1e6, 1)
            row[f"client_v{var}_kernel"] = ecg.last_kernel()
            outs[var] = par.download()
            ms = timed(lambda: ctx.encode(k, p, C, S, st.ptr, (k + p) * C, st.ptr + k * C, C, (k + p) * C))
            row[f"inplace_v{var}_GBps"] = round(alg / ms / 1e6, 1)
            ms = timed(lambda: ctx.recover(k, p, C, S, st.ptr, (k + p) * C, [0, 1]))
            row[f"decode_d0d1_v{var}_GBps"] = round((k + 2) * C * S / ms / 1e6, 1)
        ctx.set_launch(0, 0, 0)
        row["half_equals_full"] = bool(np.array_equal(outs[0], outs[5]))
        res[tag] = row
        print(tag, row, flush=True)
        data.free(); par.free(); st.free()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "tune10.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
