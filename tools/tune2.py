"""Finer sweep: grid shapes x {default, 2-stripe} per layout, plus stream
kernel block counts.  One process, interleaved rounds.  -> gpurun_out/tune2.json"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg


def main():
    rounds = 5
    ctx = ecg.Context(0)
    a, b = ctx.event(), ctx.event()

    def timed(fn):
        ctx.record(a); fn(); ctx.record(b)
        return ctx.elapsed_ms(a, b)

    out = {"stream": {}, "shapes": {}}
    n = 4 << 30
    x, y = ctx.alloc(n), ctx.alloc(n)
    x.fill(7)
    res = {}
    for _ in range(rounds):
        for mode, name, nb in ((0, "copy", 2 * n), (1, "read", n), (2, "write", n)):
            for blocks in (512, 2048, 16384, 65536, 262144, 1048576):
                ctx.set_launch(blocks, 0, 0)
                ms = timed(lambda: ctx.copy_kernel(y.ptr, x.ptr, n, mode))
                res.setdefault((name, blocks), []).append(nb / ms / 1e6)
    ctx.set_launch(0, 0, 0)
    for (name, blocks), v in sorted(res.items()):
        v.sort()
        out["stream"][f"{name}_b{blocks}"] = round(v[len(v) // 2], 1)
    x.free(); y.free()
    print("stream", json.dumps(out["stream"]), flush=True)

    shapes = [
        ("4P2_enc_client", 4, 2, 1 << 20, 1024, "enc_client"),
        ("4P2_dec_d0d1", 4, 2, 1 << 20, 1024, "dec"),
        ("8P2_enc_client", 8, 2, 1 << 20, 512, "enc_client"),
        ("8P2_enc_inplace", 8, 2, 1 << 20, 512, "enc_inplace"),
        ("8P2_dec_d0d1", 8, 2, 1 << 20, 512, "dec"),
        ("16P2_enc_128K", 16, 2, 128 << 10, 1024, "enc_inplace"),
    ]
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
        nch = (C + 4095) // 4096
        gxs = sorted({g for g in (8, 16, 32, 64, 128, 256) if g <= nch} | {nch})
        res = {}
        for _ in range(rounds):
            for v in (0, 1):
                for gx in gxs:
                    for gy in (16, 32, 64, 128, 256, 512, 1024):
                        if gx * gy < 1024 or gx * gy > 262144:
                            continue
                        ctx.set_launch(gx, gy, v)
                        res.setdefault(f"v{v}_g{gx}x{gy}", []).append(timed(fn))
            ctx.set_launch(0, 0, 0)
            res.setdefault("default", []).append(timed(fn))
        summ = {}
        for key, ms in res.items():
            ms.sort()
            med = ms[len(ms) // 2]
            summ[key] = {"ms": round(med, 4), "GBps": round(alg / med / 1e6, 1)}
        best = sorted(summ.items(), key=lambda kv: kv[1]["ms"])[:8]
        out["shapes"][name] = {"alg": alg, "default": summ["default"], "best": best, "all": summ}
        print(name, "default", summ["default"], "best", best[:5], flush=True)
        buf.free(); par.free()
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "tune2.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
