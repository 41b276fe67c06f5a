"""Client-layout encode: parity-row stride S*C (power of two) vs padded
strides; data stripe stride k*C vs padded.  Interleaved rounds, random data.
-> gpurun_out/tune5.json"""
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

    out = {}
    for k, p, S in ((8, 2, 512), (4, 2, 1024)):
        C = 1 << 20
        pads = (0, 4096, 65536, 1 << 20, 3 << 20)
        data = ctx.alloc(S * (k * C + max(pads)))
        par = ctx.alloc(p * (S * C + max(pads)))
        fill(data)
        res = {}
        for _ in range(7):
            for dpad in (0, 4096):
                for ppad in pads:
                    fn = lambda: ctx.encode(k, p, C, S, data.ptr, k * C + dpad, par.ptr, S * C + ppad, C)
                    res.setdefault(f"{k}P{p}_dpad{dpad}_ppad{ppad}", []).append(timed(fn))
            st = (k + p) * C
            fn = lambda: ctx.encode(k, p, C, S, data.ptr, st, data.ptr + k * C, C, st)
            res.setdefault(f"{k}P{p}_inplace", []).append(timed(fn))
        for key, ms in res.items():
            ms.sort()
            out[key] = round((k + p) * C * S / ms[len(ms) // 2] / 1e6, 1)
        data.free(); par.free()
    print(json.dumps(out, indent=0))
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "tune5.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
