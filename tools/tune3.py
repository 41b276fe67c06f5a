"""Data-dependence of HBM-bound kernel time (zeros / constant / random
bytes), interleaved rounds in one process -> gpurun_out/tune3.json."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg
from tools.datagen import stripe_bytes


def fill(buf, kind):
    if kind == "zero":
        buf.fill(0)
    elif kind == "const":
        buf.fill(0x5A)
    else:
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

    n = 4 << 30
    cases = {}
    bufs = {}
    for kind in ("zero", "const", "rand"):
        x, y = ctx.alloc(n), ctx.alloc(n)
        fill(x, kind); fill(y, kind)
        bufs[kind] = (x, y)
    res = {}
    k, p, C = 8, 2, 1 << 20
    S = n // ((k + p) * C)
    st = (k + p) * C
    for r in range(7):
        for kind, (x, y) in bufs.items():
            for mode, name, nb in ((0, "copy", 2 * n), (1, "read", n), (2, "write", n)):
                for blocks in (512, 262144):
                    ctx.set_launch(blocks, 0, 0)
                    res.setdefault(f"{name}_b{blocks}_{kind}", []).append(nb / timed(lambda: ctx.copy_kernel(y.ptr, x.ptr, n, mode)) / 1e6)
            ctx.set_launch(0, 0, 0)
            for v in (0, 20):
                ctx.set_launch(0, 0, v)
                res.setdefault(f"8P2enc_v{v}_{kind}", []).append((k + p) * C * S / timed(lambda: ctx.encode(k, p, C, S, x.ptr, st, x.ptr + k * C, C, st)) / 1e6)
                res.setdefault(f"4P2enc_client_v{v}_{kind}", []).append(6 * C * 600 / timed(lambda: ctx.encode(4, 2, C, 600, x.ptr, 4 * C, y.ptr, 600 * C, C)) / 1e6)
            ctx.set_launch(0, 0, 0)
    out = {}
    for key, v in sorted(res.items()):
        v.sort()
        out[key] = round(v[len(v) // 2], 1)
    print(json.dumps(out, indent=0))
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "tune3.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
