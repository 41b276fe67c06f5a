"""Fused product + checksum variants timed the way bench.py's fused rows are:
back-to-back blocks of each configuration (20 warm launches, 21 timed, events
at every boundary), all configurations forward then in reverse order, the
mean of the two medians.  EC_8P2 x 512, 1 MiB cells, 32 KiB chunks, random
data; table kinds and columns per item of crc32 / crc64 (ecg_set_csum_variant,
ecg_set_fused_cols) against the plain encode.  -> gpurun_out/fused_blocked.json.
Bench infrastructure."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402
from tools.datagen import stripe_bytes  # noqa: E402
import bench  # noqa: E402


def main():
    ctx = ecg.Context(0)
    L = ecg.lib()
    k, p, C, S = 8, 2, 1 << 20, 512
    data = ctx.alloc(k * S * C)
    blk = stripe_bytes(256 << 20, 13)
    for off in range(0, data.nbytes, blk.size):
        data.upload(blk, offset=off)
    pitch = S * C + 4096
    par = ctx.alloc(p * pitch)
    out = ctx.alloc(p * S * 32 * 8)

    def fused(htype, cols, var):
        def fn():
            L.ecg_set_fused_cols(ctx.h, cols)
            L.ecg_set_csum_variant(ctx.h, var)
            ctx.encode_csum(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C, htype, 32768, 1, out.ptr)
            L.ecg_set_fused_cols(ctx.h, 0)
            L.ecg_set_csum_variant(ctx.h, 0)
        return fn

    cfgs = [("encode", lambda: ctx.encode(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C))]
    for hn, h in (("crc32", ecg.HASH_CRC32), ("crc64", ecg.HASH_CRC64)):
        cfgs += [(f"{hn}_default", fused(h, 0, 0)),
                 (f"{hn}_bytes_c2", fused(h, 2, 256 | 16)),
                 (f"{hn}_bytes_c4", fused(h, 4, 256 | 16)),
                 (f"{hn}_nib_tb4_c4", fused(h, 4, 256 | 1024)),
                 (f"{hn}_5bit_c4", fused(h, 4, 256 | 32)),
                 (f"{hn}_s16_c4", fused(h, 4, 256 | 64))]
    ts = {n: [] for n, _ in cfgs}
    for order in (cfgs, cfgs[::-1]):
        for n, fn in order:
            ts[n].append(bench.time_kernel(ctx, fn, 21, warm=20))
            print(n, round(ts[n][-1], 4), flush=True)
    res = {n: round(sum(v) / len(v), 4) for n, v in ts.items()}
    enc = res["encode"]
    res.update({n + "_overhead": round(v / enc - 1, 4) for n, v in list(res.items()) if n != "encode"})
    print(json.dumps(res))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "fused_blocked.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
