"""Standalone CRC kernels (crc16/32/64, 4 / 32 / 1024 KiB chunks over 1 GiB of
1 MiB cells) timed with several builds of libecg.so, one subprocess per
library, interleaved three times; median of 15 launches after 5 warm-up.  usage: python tools/crc_libs.py lib1.so lib2.so ...
-> gpurun_out/crc_libs.json.  Bench infrastructure."""
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
a, b = ctx.event(), ctx.event()
C, n = 1 << 20, 1024
buf = ctx.alloc(C * n)
blk = stripe_bytes(256 << 20, 11)
for off in range(0, C * n, blk.size):
    buf.upload(blk, offset=off)
out = ctx.alloc(n * (C // 4096) * 8)
res = {}
for htype, name in ((1, "crc16"), (2, "crc32"), (3, "crc64")):
    for cs in (4096, 32768, 1 << 20):
        fn = lambda: ctx.csum_extents(htype, cs, 1, 0, C, buf.ptr, C, n, out.ptr)
        for _ in range(5):
            fn()
        ctx.sync()
        ts = []
        for _ in range(15):
            ctx.record(a); fn(); ctx.record(b); ts.append(ctx.elapsed_ms(a, b))
        ts.sort()
        res[f"{name}_cs{cs >> 10}K"] = round(C * n / ts[7] / 1e9, 3)
print(json.dumps(res))
''' % ROOT


def main():
    libs = sys.argv[1:]
    res = {}
    for rnd in range(3):
        for lib in libs:
            r = subprocess.run([sys.executable, "-c", CHILD, os.path.abspath(lib)], capture_output=True, text=True,
                               timeout=300)
            if r.returncode != 0:
                print(r.stderr[-2000:], flush=True)
                raise SystemExit(r.returncode)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            for key, v in d.items():
                res.setdefault(lib, {}).setdefault(key, []).append(v)
            print(lib, d, flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "crc_libs.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
