"""Fused product + checksum: columns per work item (ecg_set_fused_cols 1 / 2 /
4 / 8; 1 = one 4 KiB column per workgroup, the plain kernel's shape) for crc32
and crc64 against the plain encode, EC_8P2 x 512 and EC_4P2 x 1024 (1 MiB
cells, 32 KiB chunks, random data); configurations rotated every round, median
of 21 after 10 warm-up rounds.  Env AB_SHAPES="k,p,S ...", AB_COLS="2,4",
AB_HASH="crc32" narrow it.  -> gpurun_out/fused_cols_ab.json.  Bench infrastructure."""
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
    C = 1 << 20
    buf = ctx.alloc(4 << 30)
    blk = stripe_bytes(256 << 20, 13)
    for off in range(0, buf.nbytes, blk.size):
        buf.upload(blk, offset=off)
    par = ctx.alloc(2 * (1024 * C + 4096))
    out = ctx.alloc(2 * 1024 * 32 * 8)
    res = {}
    shapes = [tuple(int(x) for x in a.split(",")) for a in os.environ.get("AB_SHAPES", "").split()]
    colset = [int(x) for x in os.environ.get("AB_COLS", "1,2,4,8,0").split(",")]
    hashes = [(h, hn) for h, hn in ((ecg.HASH_CRC32, "crc32"), (ecg.HASH_CRC64, "crc64"))
              if hn in os.environ.get("AB_HASH", "crc32,crc64")]
    for k, p, S in shapes or ((8, 2, 512), (4, 2, 1024)):
        pitch = S * C + 4096
        if not (k * S * C <= buf.nbytes and p * pitch <= par.nbytes and p * S * 32 * 8 <= out.nbytes):
            raise SystemExit(f"fused_cols_ab: shape {k},{p},{S} exceeds the buffers")

        def fused(cols, htype, var=0, k=k, p=p, S=S, pitch=pitch):
            def fn():
                L.ecg_set_fused_cols(ctx.h, cols)
                L.ecg_set_csum_variant(ctx.h, var)
                ctx.encode_csum(k, p, C, S, buf.ptr, k * C, par.ptr, pitch, C, htype, 32768, 1, out.ptr)
                L.ecg_set_fused_cols(ctx.h, 0)
                L.ecg_set_csum_variant(ctx.h, 0)
            return fn
        cfgs = [("encode", lambda k=k, p=p, S=S, pitch=pitch: ctx.encode(k, p, C, S, buf.ptr, k * C, par.ptr, pitch, C))]
        for h, hn in hashes:
            for cols in colset:
                cfgs.append((f"{hn}_c{cols}", fused(cols, h, 256 if cols else 0)))
        ts = {n: [] for n, _ in cfgs}
        for rnd in range(31):
            order = cfgs[rnd % len(cfgs):] + cfgs[:rnd % len(cfgs)]
            for n, fn in order:
                ctx.record(a)
                fn()
                ctx.record(b)
                ms = ctx.elapsed_ms(a, b)
                if rnd >= 10:
                    ts[n].append(ms)
        row = {}
        for n, v in ts.items():
            v.sort()
            row[n + "_ms"] = round(v[len(v) // 2], 4)
        for n in list(row):
            if n != "encode_ms":
                row[n.replace("_ms", "_overhead")] = round(row[n] / row["encode_ms"] - 1, 4)
        res[f"{k}P{p}_x{S}"] = row
        print(k, p, row, flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "fused_cols_ab.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
