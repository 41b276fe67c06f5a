"""Fused product + checksum: columns-per-item sweep (ecg_set_fused_cols) for
EC_8P2 x 128 and EC_4P2 x 256 (1 MiB cells, 1 GiB of data), crc32 / crc64
over 32 KiB chunks, against the plain encode, interleaved in one process.
-> gpurun_out/fused_sweep.json.  Bench infrastructure."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402
from tools.datagen import stripe_bytes  # noqa: E402


def main():
    ctx = ecg.Context(0)
    L = ecg.lib()
    a, b = ctx.event(), ctx.event()

    def timed(fn, reps=7):
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

    C = 1 << 20
    buf = ctx.alloc(1 << 30)
    blk = stripe_bytes(256 << 20, 12)
    for off in range(0, 1 << 30, blk.size):
        buf.upload(blk, offset=off)
    out = ctx.alloc(1 << 22)
    par = ctx.alloc(2 * (256 * C + 4096))
    res = {}
    for k, p, S in ((8, 2, 128), (4, 2, 256)):
        pitch = S * C + 4096
        assert k * S * C <= buf.nbytes and p * pitch <= par.nbytes and p * S * 32 * 8 <= out.nbytes
        row = {"encode_ms": []}
        for rnd in range(2):
            row["encode_ms"].append(round(timed(lambda: ctx.encode(k, p, C, S, buf.ptr, k * C, par.ptr, pitch, C)), 4))
            for hname, htype in (("crc32", 2), ("crc64", 3)):
                for cols in (2, 4, 8):
                    L.ecg_set_fused_cols(ctx.h, cols)
                    ms = timed(lambda: ctx.encode_csum(k, p, C, S, buf.ptr, k * C, par.ptr, pitch, C, htype, 32768, 1,
                                                       out.ptr))
                    row.setdefault(f"{hname}_c{cols}", []).append(round(ms, 4))
                L.ecg_set_fused_cols(ctx.h, 0)
        enc = min(row["encode_ms"])
        row["overhead"] = {key: round(min(v) / enc - 1, 4) for key, v in row.items() if key.startswith("crc")}
        res[f"EC_{k}P{p}_x{S}"] = row
        print(k, p, json.dumps(row), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "fused_sweep.json"), "w"), indent=1)
    ctx.close()


if __name__ == "__main__":
    main()
