"""Default (one item per block) vs persistent pipelined kernel (variant 3),
resident-block sweep, random data, interleaved rounds -> gpurun_out/tune7.json"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg
from tools.datagen import stripe_bytes


def fill(buf):
    blk = stripe_bytes(256 << 20, 5)
    off = 0
    while off < buf.nbytes:
        n = min(blk.size, buf.nbytes - off)
        buf.upload(blk[:n], offset=off)
        off += n


def main():
    ctx = ecg.Context(0)
    a, b = ctx.event(), ctx.event()

    def timed(fn):
        ctx.record(a); fn(); ctx.record(b)
        return ctx.elapsed_ms(a, b)

    shapes = [
        ("4P2_enc_client", 4, 2, 1 << 20, 1024, "enc_client"),
        ("4P2_dec_d0d1", 4, 2, 1 << 20, 1024, "dec"),
        ("8P2_enc_client", 8, 2, 1 << 20, 512, "enc_client"),
        ("8P2_enc_inplace", 8, 2, 1 << 20, 512, "enc_inplace"),
        ("8P2_dec_d0d1", 8, 2, 1 << 20, 512, "dec"),
        ("16P2_enc_128K", 16, 2, 128 << 10, 1024, "enc_inplace"),
        ("16P2_enc_1M", 16, 2, 1 << 20, 256, "enc_inplace"),
    ]
    out = {}
    for name, k, p, C, S, mode in shapes:
        st = (k + p) * C
        buf = ctx.alloc(S * st)
        par = ctx.alloc(p * (S * C + 4096))
        fill(buf)
        if mode == "enc_client":
            fn = lambda: ctx.encode(k, p, C, S, buf.ptr, k * C, par.ptr, S * C + 4096, C)
            alg = (k + p) * C * S
        elif mode == "enc_inplace":
            fn = lambda: ctx.encode(k, p, C, S, buf.ptr, st, buf.ptr + k * C, C, st)
            alg = (k + p) * C * S
        else:
            ctx.encode(k, p, C, S, buf.ptr, st, buf.ptr + k * C, C, st)
            fn = lambda: ctx.recover(k, p, C, S, buf.ptr, st, [0, 1])
            alg = (k + 2) * C * S
        cfgs = [(0, 0), (0, 4)]
        res = {}
        for _ in range(7):
            for gx, v in cfgs:
                ctx.set_launch(gx, 0, v)
                res.setdefault(f"v{v}_g{gx}", []).append(timed(fn))
        ctx.set_launch(0, 0, 0)
        summ = {}
        for key, ms in res.items():
            ms.sort()
            summ[key] = round(alg / ms[len(ms) // 2] / 1e6, 1)
        out[name] = summ
        best = max(summ.items(), key=lambda kv: kv[1])
        print(name, "default", summ["v0_g0"], "best", best, flush=True)
        buf.free(); par.free()
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "tune7.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
