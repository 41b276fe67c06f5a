"""Fused product + checksum with fewer, longer-lived workgroups (round 3
tables: crc64 stages ~28 KiB per workgroup): grid y capped at G stripes, the
kernel's stripe loop striding, so each workgroup stages its tables once per
S/G stripes.  Interleaved with the plain encode, medians; EC_8P2 x 512 and
EC_4P2 x 1024, 1 MiB cells, 32 KiB chunks, crc32 / crc64 defaults.
usage: python tools/fused_grid.py -> gpurun_out/fused_grid.json.  Bench infrastructure."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402
import bench  # noqa: E402


def main():
    ctx = ecg.Context(0)
    C = 1 << 20
    res = {}
    for k, p, S in ((8, 2, 512), (4, 2, 1024)):
        data = ctx.alloc(S * k * C)
        bench.fill_device(ctx, data, S * k * C, 8)
        pitch = S * C + bench.PARITY_ROW_PAD
        par = ctx.alloc(p * pitch)
        out = ctx.alloc(p * S * (C // 32768) * 8)
        names, fns = ["enc"], [lambda: ctx.encode(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C)]
        for hn, ht in (("crc32", ecg.HASH_CRC32), ("crc64", ecg.HASH_CRC64)):
            for gy in (0, 128, 64, 32, 16):
                def fn(ht=ht, gy=gy):
                    ctx.set_launch(0, gy, 0)
                    ctx.encode_csum(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C, ht, 32768, 1, out.ptr)
                    ctx.set_launch(0, 0, 0)
                names.append(f"{hn}_gy{gy}")
                fns.append(fn)
        ms = bench.time_interleaved(ctx, fns, 15, warm=10)
        row = {n: round(m, 4) for n, m in zip(names, ms)}
        for n in names[1:]:
            row[n + "_overhead"] = round(row[n] / row["enc"] - 1, 4)
        res[f"{k}P{p}_x{S}"] = row
        print(k, p, json.dumps(row), flush=True)
        data.free()
        par.free()
        out.free()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "fused_grid.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
