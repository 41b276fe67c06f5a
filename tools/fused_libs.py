"""Fused product + checksum kernels timed with several builds of libecg.so
(one subprocess per library, interleaved twice), e.g. -DECG_EXP_NO_CRC (the
CRC lookups compiled out) and -DECG_EXP_NO_MULMOD (the per-item multiply
compiled out): EC_8P2 x 512 and EC_4P2 x 1024 (1 MiB cells, random data,
32 KiB chunks), crc32 / crc64, columns per item 4 / 8 / 16 and the
default, against the plain encode, interleaved launch by launch; median of
15 after 3 warm-up launches each.
usage: python tools/fused_libs.py lib1.so lib2.so ...  -> gpurun_out/fused_libs.json.
Bench infrastructure."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, sys
sys.path.insert(0, %r)
from daos_amd import ecg
ecg.LIB_PATH = sys.argv[1]
from tools.datagen import stripe_bytes
ctx = ecg.Context(0)
L = ecg.lib()
a, b = ctx.event(), ctx.event()
C = 1 << 20
buf = ctx.alloc(4 << 30)
blk = stripe_bytes(256 << 20, 13)
for off in range(0, buf.nbytes, blk.size):
    buf.upload(blk, offset=off)
par = ctx.alloc(2 * (1024 * C + 4096))
out = ctx.alloc(1 << 22)

def cfg(k, p, S, htype, cols, variant=0):
    pitch = S * C + 4096
    if htype == 0:
        return lambda: ctx.encode(k, p, C, S, buf.ptr, k * C, par.ptr, pitch, C)
    def fn():
        L.ecg_set_fused_cols(ctx.h, cols)
        L.ecg_set_csum_variant(ctx.h, variant)
        ctx.encode_csum(k, p, C, S, buf.ptr, k * C, par.ptr, pitch, C, htype, 32768, 1, out.ptr)
        L.ecg_set_csum_variant(ctx.h, 0)
    return fn

# configurations interleaved launch by launch (the box's clocks drift over a
# long run; back-to-back blocks of one configuration would absorb the drift)
res = {}
for k, p, S in ((8, 2, 512), (4, 2, 1024)):
    assert k * S * C <= buf.nbytes and 2 * (S * C + 4096) <= par.nbytes and p * S * 32 * 8 <= out.nbytes
    tag = "%%dP%%d_x%%d" %% (k, p, S)
    cfgs = [(tag + "_encode_ms", cfg(k, p, S, 0, 0))]
    for hname, htype in (("crc32", 2), ("crc64", 3)):
        for cols in (0, 4, 8):
            cfgs.append(("%%s_%%s_c%%d_ms" %% (tag, hname, cols), cfg(k, p, S, htype, cols)))
        # the wave-per-chunk kernel (csum_variant 128) and the workgroup kernel (256)
        cfgs.append(("%%s_%%s_wave_ms" %% (tag, hname), cfg(k, p, S, htype, 0, 128)))
        cfgs.append(("%%s_%%s_wg_ms" %% (tag, hname), cfg(k, p, S, htype, 0, 256)))
        # the workgroup kernel with the 5-bit tables (32) / the byte tables (16)
        cfgs.append(("%%s_%%s_wg5_ms" %% (tag, hname), cfg(k, p, S, htype, 0, 256 | 32)))
        cfgs.append(("%%s_%%s_wgb_ms" %% (tag, hname), cfg(k, p, S, htype, 0, 256 | 16)))
    ts = {n: [] for n, _ in cfgs}
    for n, fn in cfgs:
        for _ in range(3):
            fn()
        if "crc" in n:
            res[n.replace("_ms", "_kernel")] = L.ecg_last_kernel().decode()
    ctx.sync()
    for rep in range(15):
        for n, fn in cfgs:
            ctx.record(a); fn(); ctx.record(b); ts[n].append(ctx.elapsed_ms(a, b))
    for n, v in ts.items():
        v.sort()
        res[n] = round(v[len(v) // 2], 4)
    L.ecg_set_fused_cols(ctx.h, 0)
print(json.dumps(res))
''' % ROOT


def main():
    libs = sys.argv[1:]
    out = {}
    for rnd in range(int(os.environ.get("FUSED_ROUNDS", "2"))):
        for lib in libs:
            r = subprocess.run([sys.executable, "-c", CHILD, lib], capture_output=True, text=True, timeout=400)
            if r.returncode != 0:
                print(r.stdout, r.stderr, flush=True)
                raise SystemExit(r.returncode)
            row = json.loads(r.stdout.strip().splitlines()[-1])
            out.setdefault(lib, []).append(row)
            print(lib, rnd, json.dumps({k: v for k, v in row.items() if k.endswith("_ms")}), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "fused_libs.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
