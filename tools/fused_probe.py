"""Why does bench.py's fused row differ from tune11?  Same process, same
shapes: time encode and fused crc32/32 KiB under different data seeds,
output-buffer sizes and allocation orders (prints one JSON line)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402
import bench  # noqa: E402


def main():
    ctx = ecg.Context(0)
    k, p, C, S = 8, 2, 1 << 20, 512
    res = {"cols": os.environ.get("ECG_FUSED_COLS", "auto")}
    for seed in (8, 5):
        data = ctx.alloc(S * k * C)
        bench.fill_device(ctx, data, S * k * C, seed)
        pitch = S * C + bench.PARITY_ROW_PAD
        par = ctx.alloc(p * pitch)
        for osz in ("exact", "big"):
            out = ctx.alloc(p * S * (C // 32768) * 4 if osz == "exact" else p * S * (C // 4096) * 8)
            enc = bench.time_kernel(ctx, lambda: ctx.encode(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C), 7)
            fus = bench.time_kernel(ctx, lambda: ctx.encode_csum(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C,
                                                                 ecg.HASH_CRC32, 32768, 1, out.ptr), 7)
            res[f"seed{seed}_{osz}"] = [round(enc, 4), round(fus, 4), round(fus / enc - 1, 3)]
            out.free()
        par.free()
        data.free()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
