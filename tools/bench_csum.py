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
        for cs in (4096, 32768, 1 << 20):
            for blocks in (0, 8192):
                L.ecg_set_csum_launch(ctx.h, blocks)
                ms = timed(lambda: ctx.csum_extents(htype, cs, 1, 0, C, buf.ptr, C, n, out.ptr))
                res[f"{NAMES[htype]}_cs{cs >> 10}K_b{blocks}"] = {
                    "ms": round(ms, 4), "GBps": round(C * n / ms / 1e6, 1), "kernel": L.ecg_last_kernel().decode()}
        L.ecg_set_csum_launch(ctx.h, 0)
    # rebuild pattern: encode alone / encode then checksum launches / fused
    for (k, p, C2, S, tag) in ((8, 2, 1 << 20, 256, "8p2_1M"), (4, 2, 1 << 20, 512, "4p2_1M"),
                               (16, 2, 128 << 10, 1024, "16p2_128K")):
        data = ctx.alloc(S * k * C2)
        par = ctx.alloc(p * S * C2 + 4096)
        cs_out = ctx.alloc(p * S * (C2 // 32768) * 8)
        for off in range(0, S * k * C2, blk.size):      # random bytes everywhere: CRC lookups are data-dependent
            data.upload(blk[: min(blk.size, S * k * C2 - off)], offset=off)
        pitch = S * C2 + 4096
        enc = timed(lambda: ctx.encode(k, p, C2, S, data.ptr, k * C2, par.ptr, pitch, C2))
        for htype in ((1, 2, 3) if tag == "8p2_1M" else (2,)):
            def two_pass():
                ctx.encode(k, p, C2, S, data.ptr, k * C2, par.ptr, pitch, C2)
                for r in range(p):
                    ctx.csum_extents(htype, 32768, 1, 0, C2, par.ptr + r * pitch, C2, S, cs_out.ptr)
            sep = timed(two_pass)
            fus = timed(lambda: ctx.encode_csum(k, p, C2, S, data.ptr, k * C2, par.ptr, pitch, C2, htype, 32768, 1,
                                                cs_out.ptr))
            alg = (k + p) * C2 * S
            res[f"enc_{tag}_{NAMES[htype]}"] = {
                "encode_ms": round(enc, 4), "encode_then_csum_ms": round(sep, 4), "fused_ms": round(fus, 4),
                "encode_GBps": round(alg / enc / 1e6, 1), "fused_GBps": round(alg / fus / 1e6, 1),
                "fused_overhead_vs_encode": round(fus / enc - 1, 4), "fused_kernel": L.ecg_last_kernel().decode()}
        if tag == "8p2_1M":
            st = ctx.alloc(S * (k + p) * C2)
            for off in range(0, S * (k + p) * C2, blk.size):
                st.upload(blk[: min(blk.size, S * (k + p) * C2 - off)], offset=off)
            rec = timed(lambda: ctx.recover(k, p, C2, S, st.ptr, (k + p) * C2, [0, 1]))
            recf = timed(lambda: ctx.recover_csum(k, p, C2, S, st.ptr, (k + p) * C2, [0, 1], 2, 32768, 1,
                                                  cs_out.ptr))
            res["rec_8p2_1M_crc32"] = {"recover_ms": round(rec, 4), "fused_ms": round(recf, 4),
                                      "fused_overhead": round(recf / rec - 1, 4)}
            st.free()
        data.free(); par.free(); cs_out.free()
    print(json.dumps(res, indent=0))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "bench_csum.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
