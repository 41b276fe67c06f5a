"""HBM aliasing: parity-row pitch (client layout) and cell pitch (recovery
layout) sweeps, random data, interleaved rounds -> gpurun_out/tune6.json"""
import json, os, sys
import numpy as np
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

    out = {}
    C = 1 << 20
    pads = (0, 256, 1024, 4096, 8192, 12288, 65536 + 4096)
    for k, p, S in ((8, 2, 512), (4, 2, 1024), (16, 2, 256)):
        maxp = max(pads)
        data = ctx.alloc(S * (k + p) * (C + maxp) + maxp)
        par = ctx.alloc(p * (S * C + maxp))
        fill(data)
        en = ecg.cauchy1(k, p)
        res = {}
        for _ in range(7):
            for pad in pads:
                fn = lambda: ctx.encode(k, p, C, S, data.ptr, k * C, par.ptr, S * C + pad, C)
                res.setdefault(f"{k}P{p}_client_ppad{pad}", []).append(((k + p) * C * S, timed(fn)))
                pitch = C + pad
                st = (k + p) * pitch
                fn = lambda: ctx.matmul(en[k:], C, S, data.ptr, [j * pitch for j in range(k)], st,
                                        data.ptr, [(k + r) * pitch for r in range(p)], st)
                res.setdefault(f"{k}P{p}_inplace_cellpad{pad}", []).append(((k + p) * C * S, timed(fn)))
                rows, dec, _ = ecg.recov_matrix(k, p, [0, 1])
                fn = lambda: ctx.matmul(rows, C, S, data.ptr, [int(d) * pitch for d in dec], st,
                                        data.ptr, [0, pitch], st)
                res.setdefault(f"{k}P{p}_decode_cellpad{pad}", []).append(((k + 2) * C * S, timed(fn)))
        for key, v in res.items():
            ms = sorted(x[1] for x in v)
            out[key] = round(v[0][0] / ms[len(ms) // 2] / 1e6, 1)
        data.free(); par.free()
    print(json.dumps(out, indent=0))
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "tune6.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
