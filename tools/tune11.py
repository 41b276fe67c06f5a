"""Fused product+checksum: columns per work item (ECG_FUSED_COLS, read once
per process) x checksum chunk size, EC_8P2 / EC_4P2 1 MiB cells, crc32 and
crc64, plus the parity-shard rebuild -> one JSON line per process
(tools/gpu_fused.sh runs it for several settings)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402
from tools.datagen import stripe_bytes  # noqa: E402


def main():
    ctx = ecg.Context(0)
    a, b = ctx.event(), ctx.event()

    def timed(fn, reps=9):
        fn()
        ts = []
        for _ in range(reps):
            ctx.record(a)
            fn()
            ctx.record(b)
            ts.append(ctx.elapsed_ms(a, b))
        ts.sort()
        return ts[len(ts) // 2]

    res = {"ECG_FUSED_COLS": os.environ.get("ECG_FUSED_COLS", "auto")}
    C = 1 << 20
    for k, p, S in ((8, 2, 512), (4, 2, 1024)):
        data = ctx.alloc(S * k * C)
        blk = stripe_bytes(256 << 20, 5)
        for off in range(0, S * k * C, blk.size):      # random everywhere: CRC lookups are data-dependent
            data.upload(blk[: min(blk.size, S * k * C - off)], offset=off)
        pitch = S * C + 4096
        par = ctx.alloc(p * pitch)
        out = ctx.alloc(p * S * (C // 4096) * 8)
        res[f"{k}p{p}_encode_ms"] = timed(lambda: ctx.encode(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C))
        for h, hn in ((ecg.HASH_CRC32, "crc32"), (ecg.HASH_CRC64, "crc64")):
            for cs in (4096, 8192, 32768, 1 << 20):
                if h == ecg.HASH_CRC64 and cs not in (32768,):
                    continue
                res[f"{k}p{p}_{hn}_cs{cs >> 10}K_ms"] = timed(
                    lambda: ctx.encode_csum(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C, h, cs, 1, out.ptr))
        if k == 8:
            pieces = (ecg.MigratePiece * S)()
            npc = ctypes.c_uint32()

            def shard():
                ecg._chk(ecg.lib().ecg_migrate_update_parity(
                    ctx.h, (37 << 24) | 1, C, 1, k + p - 1, data.ptr, 0, S * k * C, 1, ecg.HASH_CRC32, 32768,
                    par.ptr, out.ptr, pieces, S, ctypes.byref(npc), None), "migrate_update_parity")

            res["8p2_shard_rebuild_crc32_ms"] = timed(shard)
        data.free()
        par.free()
        out.free()
    res = {kk: (round(v, 4) if isinstance(v, float) else v) for kk, v in res.items()}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
