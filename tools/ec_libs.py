"""EC product kernels timed with several builds of libecg.so (one subprocess
per library, interleaved twice): the BASELINE shapes, device-resident, plus the
box's streaming read / write rates.  Used with experimental builds that change
the kernel body, e.g. -DECG_EXP_XOR_ONLY (the GF multiply replaced by a plain
XOR: the same loads, stores, grid and registers for the addresses, so it
measures what this access pattern can stream).
usage: python tools/ec_libs.py lib1.so lib2.so ...  -> gpurun_out/ec_libs.json.
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
ctx = ecg.Context(0)
a, b = ctx.event(), ctx.event()
MiB = 1 << 20
buf = ctx.alloc(13 << 30)
buf.fill(0x5A)
ctx.sync()

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
for name, mode in (("read", 1), ("write", 2)):
    n = 4 << 30
    ms = timed(lambda: ctx.copy_kernel(buf.ptr + n, buf.ptr, n, mode))
    res["stream_" + name + "_GBps"] = round(n / ms / 1e6, 1)
for k, p, C, S in ((4, 2, MiB, 1024), (8, 2, MiB, 512), (16, 2, 128 << 10, 1024), (16, 2, 128 << 10, 4096),
                   (2, 1, 128 << 10, 1024)):
    tag = "%%dP%%d_%%dK_x%%d" %% (k, p, C >> 10, S)
    pitch = S * C + 4096
    data, par = buf.ptr, buf.ptr + k * S * C
    assert k * S * C + p * pitch <= buf.nbytes and S * (k + p) * C <= buf.nbytes
    alg = (k + p) * C * S
    ms = timed(lambda: ctx.encode(k, p, C, S, data, k * C, par, pitch, C))
    res[tag + "_enc_GBps"] = round(alg / ms / 1e6, 1)
    ms = timed(lambda: ctx.recover(k, p, C, S, buf.ptr, (k + p) * C, [0, 1] if p >= 2 else [0]))
    res[tag + "_dec_GBps"] = round(alg / ms / 1e6 if p >= 2 else (k + 1) * C * S / ms / 1e6, 1)
res["kernel"] = ecg.lib().ecg_last_kernel().decode()
print(json.dumps(res))
''' % ROOT


def main():
    libs = sys.argv[1:]
    out = {}
    for rnd in range(int(os.environ.get("EC_ROUNDS", "2"))):
        for lib in libs:
            r = subprocess.run([sys.executable, "-c", CHILD, lib], capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                print(r.stdout, r.stderr, flush=True)
                raise SystemExit(r.returncode)
            row = json.loads(r.stdout.strip().splitlines()[-1])
            out.setdefault(lib, []).append(row)
            print(lib, rnd, row, flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "ec_libs.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
