"""Fused product + checksum, columns per work item (ecg_set_fused_cols),
A/B interleaved in one process on random data everywhere (CRC lookups are
data-dependent), after a long warm-up: EC_8P2 and EC_4P2 1 MiB cells,
crc32 / crc64, 32 KiB and 1 MiB chunks, plus the parity-shard rebuild.
Medians over rounds -> one JSON line."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402
import bench  # noqa: E402

COLS = (0, 2, 4, 8, 16)


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
        enc = lambda: ctx.encode(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C)  # noqa: E731
        for _ in range(50):
            enc()
        ctx.sync()
        cases = [("enc", None, None)]
        for h, hn in ((ecg.HASH_CRC32, "crc32"), (ecg.HASH_CRC64, "crc64")):
            for cs in (32768, 1 << 20):
                for n in COLS:
                    cases.append((f"{hn}_cs{cs >> 10}K_cols{n}", (h, cs), n))
        if k == 8:
            for n in COLS:
                cases.append((f"shard_crc32_cols{n}", "shard", n))
        pieces = (ecg.MigratePiece * S)()
        npc = ctypes.c_uint32()
        samples = {name: [] for name, _, _ in cases}
        for _ in range(3):
            for name, what, n in cases:
                L.ecg_set_fused_cols(ctx.h, n or 0)
                if what is None:
                    fn = enc
                elif what == "shard":
                    def fn():
                        ecg._chk(L.ecg_migrate_update_parity(
                            ctx.h, (37 << 24) | 1, C, 1, k + p - 1, data.ptr, 0, S * k * C, 1, ecg.HASH_CRC32,
                            32768, par.ptr, out.ptr, pieces, S, ctypes.byref(npc), None), "shard")
                else:
                    h, cs = what
                    fn = (lambda h=h, cs=cs: ctx.encode_csum(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C, h, cs,
                                                             1, out.ptr))
                samples[name].append(bench.time_kernel(ctx, fn, 7))
        L.ecg_set_fused_cols(ctx.h, 0)
        for name, v in samples.items():
            v.sort()
            res[f"{k}p{p}_{name}"] = round(v[len(v) // 2], 4)
        data.free()
        par.free()
        out.free()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
