"""Fused product + crc32 / crc64 table kinds: the 5-bit tables (crc32's
default), the byte tables (bit 4; crc64's default), and the s16 byte tables
with SDWA addresses + nibble column shift (bit 9, TB 3; with AB_OLD_KINDS=1),
and the positional nibble tables (bit 10, TB 4), against each hash's default, in one process, the order of the
configurations rotated every round so neither always follows the plain
encode (tools/fused_libs.py keeps a fixed order and showed a ~1-2 % position
bias); median of 21 rounds after 10 warm-up rounds, random cells, 1 MiB
cells, 32 KiB chunks.  usage: python tools/fused_tables_ab.py [k,p,S ...]
-> gpurun_out/fused_tables_ab.json.  Bench infrastructure."""
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
    shapes = [tuple(int(x) for x in a.split(",")) for a in sys.argv[1:]] or [(8, 2, 512), (8, 3, 512)]
    # every buffer sized for the largest shape (a shape past a buffer's end
    # would read or write out of bounds: refuse it instead)
    data_bytes = max(k * S * C for k, p, S in shapes)
    par_bytes = max(p * (S * C + 4096) for k, p, S in shapes)
    out_bytes = max(p * S * (C // 32768) * 8 for k, p, S in shapes)
    if data_bytes > (8 << 30) or par_bytes > (4 << 30):
        raise SystemExit(f"fused_tables_ab: shapes too large ({data_bytes} B data, {par_bytes} B parity)")
    buf = ctx.alloc(data_bytes)
    blk = stripe_bytes(256 << 20, 13)
    for off in range(0, buf.nbytes, blk.size):
        buf.upload(blk[:min(blk.size, buf.nbytes - off)], offset=off)
    par = ctx.alloc(par_bytes)
    out = ctx.alloc(out_bytes)
    res = {}
    for k, p, S in shapes:
        pitch = S * C + 4096
        assert k * S * C <= buf.nbytes and p * pitch <= par.nbytes and p * S * (C // 32768) * 8 <= out.nbytes

        def fused(variant, htype=ecg.HASH_CRC32, k=k, p=p, S=S, pitch=pitch):
            def fn():
                L.ecg_set_csum_variant(ctx.h, variant)
                ctx.encode_csum(k, p, C, S, buf.ptr, k * C, par.ptr, pitch, C, htype, 32768, 1, out.ptr)
                L.ecg_set_csum_variant(ctx.h, 0)
            return fn
        cfgs = [("encode", lambda k=k, p=p, S=S, pitch=pitch: ctx.encode(k, p, C, S, buf.ptr, k * C, par.ptr,
                                                                          pitch, C)),
                ("crc32_dflt", fused(0)), ("crc32_tb4", fused(1024)),
                ("crc64_dflt", fused(0, ecg.HASH_CRC64)), ("crc64_tb4", fused(1024, ecg.HASH_CRC64))]
        if os.environ.get("AB_OLD_KINDS"):
            cfgs += [("crc32_5bit", fused(32)), ("crc32_bytes", fused(16)), ("crc32_tb3", fused(512)),
                     ("crc64_tb3", fused(512 | 256, ecg.HASH_CRC64))]
        # a configuration this shape has no instantiation for is dropped
        ok = []
        for n, fn in cfgs:
            try:
                fn()
                ok.append((n, fn))
            except ecg.EcgError:
                L.ecg_set_csum_variant(ctx.h, 0)
        cfgs = ok
        ts = {n: [] for n, _ in cfgs}
        for rnd in range(31):
            order = cfgs[rnd % len(cfgs):] + cfgs[:rnd % len(cfgs)]
            for n, fn in order:
                ctx.record(a)
                fn()
                ctx.record(b)
                if rnd >= 10:
                    ts[n].append(ctx.elapsed_ms(a, b))
                else:
                    ctx.elapsed_ms(a, b)
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
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "fused_tables_ab.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
