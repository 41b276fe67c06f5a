"""Fused product + checksum kernels timed with several builds of libecg.so
(one subprocess per library, interleaved twice), e.g. -DECG_EXP_NO_CRC (the
CRC lookups compiled out) and -DECG_EXP_NO_MULMOD (the per-item multiply
compiled out): EC_8P2 x 512 and EC_4P2 x 1024 (1 MiB cells, random data,
32 KiB chunks), crc32 / crc64, columns per item 2 / 4 / 8 / 16 and the
default, against the plain encode.  Median of 15 after 5 warm-up launches.
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

def timed(fn, reps=15):
    for _ in range(5):
        fn()
    ctx.sync()
    ts = []
    for _ in range(reps):
        ctx.record(a); fn(); ctx.record(b); ts.append(ctx.elapsed_ms(a, b))
    ts.sort()
    return ts[reps // 2]

res = {}
for k, p, S in ((8, 2, 512), (4, 2, 1024)):
    pitch = S * C + 4096
    assert k * S * C <= buf.nbytes and p * pitch <= par.nbytes and p * S * 32 * 8 <= out.nbytes
    tag = "%%dP%%d_x%%d" %% (k, p, S)
    res[tag + "_encode_ms"] = round(timed(lambda: ctx.encode(k, p, C, S, buf.ptr, k * C, par.ptr, pitch, C)), 4)
    for hname, htype in (("crc32", 2), ("crc64", 3)):
        for cols in (0, 2, 4, 8, 16):
            L.ecg_set_fused_cols(ctx.h, cols)
            ms = timed(lambda: ctx.encode_csum(k, p, C, S, buf.ptr, k * C, par.ptr, pitch, C, htype, 32768, 1, out.ptr))
            res["%%s_%%s_c%%d_ms" %% (tag, hname, cols)] = round(ms, 4)
            res["%%s_%%s_c%%d_kernel" %% (tag, hname, cols)] = L.ecg_last_kernel().decode()
        L.ecg_set_fused_cols(ctx.h, 0)
print(json.dumps(res))
''' % ROOT


def main():
    libs = sys.argv[1:]
    out = {}
    for rnd in range(2):
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
