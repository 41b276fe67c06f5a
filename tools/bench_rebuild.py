"""Rebuild of one parity shard on device-resident fetched stripes
(ecg_migrate_update_parity, migrate_update_parity restated): the kept parity
row and its crc32 chunk checksums (32 KiB chunks, fused) vs the full encode
with checksums of every parity row (ecg_encode_csum, what obj_ec_encode_buf +
the csummer would compute) and the plain encode.  Algorithmic bytes: (k + 1)
cells per stripe for the shard rebuild, (k + p) for the full encode.
-> gpurun_out/bench_rebuild.json.  Bench infrastructure (no oracle)."""
import ctypes as ct
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402
from tools.datagen import stripe_bytes  # noqa: E402

OC = {(8, 2): (37 << 24) | 1, (16, 2): (39 << 24) | 1, (4, 2): (35 << 24) | 1}


def main():
    ctx = ecg.Context(0)
    L = ecg.lib()
    a, b = ctx.event(), ctx.event()

    def timed(fn, reps=9):
        fn()
        ctx.sync()
        ts = []
        for _ in range(reps):
            ctx.record(a); fn(); ctx.record(b)
            ts.append(ctx.elapsed_ms(a, b))
        ts.sort()
        return ts[len(ts) // 2]

    blk = stripe_bytes(256 << 20, 12)
    res = {}
    for k, p, C, S in ((8, 2, 1 << 20, 512), (16, 2, 128 << 10, 1024), (4, 2, 1 << 20, 1024)):
        data = ctx.alloc(S * k * C)
        for off in range(0, S * k * C, blk.size):
            data.upload(blk[: min(blk.size, S * k * C - off)], offset=off)
        pitch = S * C + 4096
        par = ctx.alloc(p * pitch)
        nch = C // 32768
        cs = ctx.alloc(p * S * nch * 4)
        pieces = (ecg.MigratePiece * S)()
        n = ct.c_uint32()

        def shard():
            rc = L.ecg_migrate_update_parity(ctx.h, OC[(k, p)], C, 1, k + p - 1, data.ptr, 0, S * k * C, 1, 2,
                                             32768, par.ptr, cs.ptr, pieces, S, ct.byref(n), None)
            assert rc == 0, L.ecg_strerror()

        t_shard = timed(shard)
        kern = ecg.last_kernel()
        t0 = time.perf_counter()
        for _ in range(10):
            shard()
        ctx.sync()
        wall = (time.perf_counter() - t0) / 10 * 1e3
        t_full = timed(lambda: ctx.encode_csum(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C, 2, 32768, 1,
                                               cs.ptr))
        t_enc = timed(lambda: ctx.encode(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C))
        res[f"EC_{k}P{p}_{C >> 10}KiB_x{S}"] = {
            "shard_rebuild_crc32_ms": round(t_shard, 4), "shard_rebuild_kernel": kern,
            "shard_rebuild_alg_GBps": round((k + 1) * C * S / t_shard / 1e6, 1),
            "shard_rebuild_wall_ms_per_call": round(wall, 4),
            "full_encode_crc32_ms": round(t_full, 4),
            "full_encode_crc32_alg_GBps": round((k + p) * C * S / t_full / 1e6, 1),
            "encode_only_ms": round(t_enc, 4),
            "shard_vs_full_encode_crc32": round(t_shard / t_full, 3)}
        print(k, p, res[f"EC_{k}P{p}_{C >> 10}KiB_x{S}"], flush=True)
        data.free(); par.free(); cs.free()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "bench_rebuild.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
