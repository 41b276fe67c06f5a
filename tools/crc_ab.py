"""A/B of the CRC lookup tables: 5-bit conflict-free tables (default) vs the
byte tables (ecg_set_csum_variant bit 4), in one process, interleaved:
  * standalone kernels over 1 GiB of 1 MiB cells, 4 / 32 / 1024 KiB chunks;
  * fused encode + checksums (EC_8P2 x 512 and EC_4P2 x 1024, 1 MiB cells,
    32 KiB chunks) and the parity-shard rebuild row <8,1> against the plain
    encode.
Median of 7 launches after 3 warm-up launches.  -> gpurun_out/crc_ab.json.  Bench infrastructure."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402
from tools.datagen import stripe_bytes  # noqa: E402

NAMES = {1: "crc16", 2: "crc32", 3: "crc64"}


def main():
    ctx = ecg.Context(0)
    L = ecg.lib()
    a, b = ctx.event(), ctx.event()

    def timed(fn, reps=7):
        for _ in range(3):
            fn()
        ctx.sync()
        ts = []
        for _ in range(reps):
            ctx.record(a)
            fn()
            ctx.record(b)
            ts.append(ctx.elapsed_ms(a, b))
        ts.sort()
        return ts[len(ts) // 2]

    C, n = 1 << 20, 1024
    buf = ctx.alloc(C * n)
    blk = stripe_bytes(256 << 20, 11)
    for off in range(0, C * n, blk.size):
        buf.upload(blk[: min(blk.size, C * n - off)], offset=off)
    out = ctx.alloc(n * (C // 4096) * 8)
    res = {}
    for htype in (1, 2, 3) if "fused-only" not in sys.argv else ():
        for cs in (4096, 32768, 1 << 20):
            row = {}
            for rnd in range(2):
                for tag, var in (("dflt", 0), ("bytes", 16), ("f5", 32)):
                    L.ecg_set_csum_variant(ctx.h, var)
                    ms = timed(lambda: ctx.csum_extents(htype, cs, 1, 0, C, buf.ptr, C, n, out.ptr))
                    row.setdefault(tag, []).append(round(C * n / ms / 1e9, 3))
                    row[f"{tag}_kernel"] = L.ecg_last_kernel().decode()
            res[f"{NAMES[htype]}_cs{cs >> 10}K_TBps"] = row
            print(NAMES[htype], cs, row, flush=True)
    L.ecg_set_csum_variant(ctx.h, 0)
    par = ctx.alloc(2 * (256 * C + 4096))
    for k, p, S in ((8, 2, 128), (4, 2, 256)):          # data k*S*C = 1 GiB = buf
        pitch = S * C + 4096
        assert k * S * C <= buf.nbytes and p * pitch <= par.nbytes
        assert p * S * (C // 32768) * 8 <= out.nbytes
        row = {"encode_ms": []}
        for rnd in range(2):
            row["encode_ms"].append(round(timed(lambda: ctx.encode(k, p, C, S, buf.ptr, k * C, par.ptr, pitch, C)), 4))
            for hname, htype in (("crc32", 2), ("crc64", 3)):
                for tag, var in (("dflt", 0), ("wg_tb0", 32 | 256), ("wg_tb1", 16 | 256), ("wave_tb0", 160),
                                 ("wave_tb1", 144)):
                    L.ecg_set_csum_variant(ctx.h, var)
                    try:
                        ms = timed(lambda: ctx.encode_csum(k, p, C, S, buf.ptr, k * C, par.ptr, pitch, C, htype, 32768,
                                                           1, out.ptr))
                    except ecg.EcgError:          # that table kind is not instantiated for this shape
                        continue
                    row.setdefault(f"{hname}_{tag}_ms", []).append(round(ms, 4))
                    row[f"{hname}_{tag}_kernel"] = L.ecg_last_kernel().decode()
            L.ecg_set_csum_variant(ctx.h, 0)
        enc = min(row["encode_ms"])
        for key in list(row):
            if key.endswith("_ms") and key != "encode_ms":
                row[key.replace("_ms", "_overhead")] = round(min(row[key]) / enc - 1, 4)
        res[f"fused_EC_{k}P{p}_1MiB_x{S}"] = row
        print(k, p, row, flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "crc_ab.json"), "w"), indent=1)
    ctx.close()


if __name__ == "__main__":
    main()
