"""Chunked-checksum kernel sweep (include/ecg_csum.h) on device-resident data:
every DAOS hash type x chunk sizes x grid caps, plus the rebuild pattern
(EC_8P2 encode, then crc of the regenerated parity cells).
-> gpurun_out/bench_csum.json.  Bench infrastructure (no oracle)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402
from tools.datagen import stripe_bytes  # noqa: E402

NAMES = {1: "crc16", 2: "crc32", 3: "crc64", 7: "adler32"}


def main():
    ctx = ecg.Context(0)
    a, b = ctx.event(), ctx.event()
    L = ecg.lib()

    def timed(fn, reps=7):
        ts = []
        for _ in range(reps):
            ctx.record(a)
            fn()
            ctx.record(b)
            ts.append(ctx.elapsed_ms(a, b))
        ts.sort()
        return ts[len(ts) // 2]

    C, n = 1 << 20, 1024                      # 1 GiB of 1 MiB cells
    buf = ctx.alloc(C * n)
    blk = stripe_bytes(256 << 20, 9)
    for off in range(0, C * n, blk.size):
        buf.upload(blk[: min(blk.size, C * n - off)], offset=off)
    out = ctx.alloc(n * (C // 4096) * 8)
    res = {}
    for htype in (1, 2, 3, 7):
        for cs in (4096, 16384, 32768, 1 << 20):
            for blocks in (0, 1024, 2048, 8192, 65536):
                L.ecg_set_csum_launch(ctx.h, blocks)
                ms = timed(lambda: ctx.csum_extents(htype, cs, 1, 0, C, buf.ptr, C, n, out.ptr))
                res[f"{NAMES[htype]}_cs{cs >> 10}K_b{blocks}"] = {
                    "ms": round(ms, 4), "GBps": round(C * n / ms / 1e6, 1), "kernel": L.ecg_last_kernel().decode()}
        L.ecg_set_csum_launch(ctx.h, 0)
    # rebuild pattern: EC_8P2 encode of 64 stripes then crc32 of the parity cells
    k, p, S = 8, 2, 64
    data = ctx.alloc(S * k * C)
    par = ctx.alloc(p * S * C + 4096)
    data.fill(0x3C)
    enc = timed(lambda: ctx.encode(k, p, C, S, data.ptr, k * C, par.ptr, S * C + 4096, C))
    crc = timed(lambda: ctx.csum_extents(2, 32768, 1, 0, C, par.ptr, C, p * S, out.ptr))
    res["rebuild_8p2_encode_ms"] = round(enc, 4)
    res["rebuild_8p2_parity_crc32_ms"] = round(crc, 4)
    print(json.dumps(res, indent=0))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "bench_csum.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
