"""Where the fused product+checksum time goes: the same launch timed with
the production library and with experimental builds (ECG_EXP_NO_MULMOD:
per-item reduction multiply removed; ECG_EXP_NO_CRC: CRC lookups removed),
random data, EC_8P2 / EC_4P2 1 MiB cells, crc32 / crc64 32 KiB chunks.
Checksums of the experimental builds are wrong by construction.
usage: python tools/fused_cost.py [path/to/libecg.so]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402

if len(sys.argv) > 1:
    ecg.LIB_PATH = os.path.abspath(sys.argv[1])
import bench  # noqa: E402

COLS = [int(c) for c in os.environ.get("FUSED_COST_COLS", "0").split(",")]


def main():
    ctx = ecg.Context(0)
    C = 1 << 20
    res = {"lib": os.path.basename(ecg.LIB_PATH)}
    for k, p, S in ((8, 2, 512), (4, 2, 1024), (8, 1, 512)):
        data = ctx.alloc(S * k * C)
        bench.fill_device(ctx, data, S * k * C, 8)
        pitch = S * C + bench.PARITY_ROW_PAD
        par = ctx.alloc(p * pitch)
        out = ctx.alloc(p * S * (C // 4096) * 8)
        for _ in range(50):
            ctx.encode(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C)
        res[f"{k}p{p}_enc"] = round(bench.time_kernel(
            ctx, lambda: ctx.encode(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C), 9), 4)
        for h, hn in ((ecg.HASH_CRC32, "crc32"), (ecg.HASH_CRC64, "crc64")):
            for n in COLS:
                ecg.lib().ecg_set_fused_cols(ctx.h, n)
                res[f"{k}p{p}_{hn}_c{n}"] = round(bench.time_kernel(
                    ctx, lambda: ctx.encode_csum(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C, h, 32768, 1,
                                                 out.ptr), 9), 4)
            ecg.lib().ecg_set_fused_cols(ctx.h, 0)
        data.free()
        par.free()
        out.free()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
