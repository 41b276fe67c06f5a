"""Fused product + checksum with fewer, longer-lived workgroups: columns per
item x stripes handled in parallel (grid y; the kernel's stripe loop strides
beyond it), so each workgroup stages the CRC tables once for many items.
Random data, EC_8P2 x 512 and EC_4P2 x 1024, 1 MiB cells, crc32 32 KiB chunks;
A/B interleaved, medians -> one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402
import bench  # noqa: E402


def main():
    ctx = ecg.Context(0)
    L = ecg.lib()
    C = 1 << 20
    res = {}
    for k, p, S in ((8, 2, 512), (4, 2, 1024)):
        data = ctx.alloc(S * k * C)
        bench.fill_device(ctx, data, S * k * C, 8)
        pitch = S * C + bench.PARITY_ROW_PAD
        par = ctx.alloc(p * pitch)
        out = ctx.alloc(p * S * (C // 4096) * 8)
        for _ in range(50):
            ctx.encode(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C)
        cases = [("enc", 0, 0)]
        for cols in (1, 2, 4, 8):
            for gy in (0, 256, 128, 64, 32):
                cases.append((f"c{cols}_gy{gy}", cols, gy))
        samples = {n: [] for n, _, _ in cases}
        for _ in range(3):
            for name, cols, gy in cases:
                if name == "enc":
                    ctx.set_launch(0, 0, 0)
                    fn = lambda: ctx.encode(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C)  # noqa: E731
                else:
                    L.ecg_set_fused_cols(ctx.h, cols)
                    ctx.set_launch(0, gy, 0)
                    fn = (lambda: ctx.encode_csum(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C, ecg.HASH_CRC32,
                                                  32768, 1, out.ptr))
                samples[name].append(bench.time_kernel(ctx, fn, 7))
        ctx.set_launch(0, 0, 0)
        L.ecg_set_fused_cols(ctx.h, 0)
        for n, v in samples.items():
            v.sort()
            res[f"{k}p{p}_{n}"] = round(v[1], 4)
        data.free()
        par.free()
        out.free()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
