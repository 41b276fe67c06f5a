"""A/B of product-kernel builds (tools/build_exp.sh) on the device-resident
EC shapes, timed as bench.py times its detail rows: launches back to back on
one stream with an event at every boundary (no host wait between launches),
the median of 30 after 40 warm-up launches.  One subprocess per library and
round, libraries rotated every round (the box's clocks drift over a run).
The launch tuner is off (ECG_AUTOTUNE=0); every plain shape is timed
uncapped and at its candidate blocks-per-CU cap (k = 16: 2, k = 8: 3).
EC_OPS (default "enc,dec") picks the shapes: enc, dec, crc32, crc64 (the
fused encode + parity checksums), enc3 / dec3 (three parity rows / erasures),
upd1 .. upd4 (delta parity update of 1-4 cells per stripe).
EC_ORDERS (default "0") times each shape under the listed 1D item orders
(ecg_set_launch_order: 1 stripe-fastest, 2 / 3 XCD-blocked).
usage: [EC_OPS=...] python tools/ec_ab.py NAME=lib.so ... -> gpurun_out/ec_ab.json.
Bench infrastructure."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, os, sys
sys.path.insert(0, %r)
from daos_amd import ecg
ecg.LIB_PATH = sys.argv[1]
ctx = ecg.Context(0)
MiB = 1 << 20

def timed(fn, iters=30, warm=40):
    for _ in range(warm):
        fn()
    ctx.sync()
    evs = [ctx.event() for _ in range(iters + 1)]
    ctx.record(evs[0])
    for i in range(iters):
        fn()
        ctx.record(evs[i + 1])
    ms = sorted(ctx.elapsed_ms(evs[i], evs[i + 1]) for i in range(iters))
    for e in evs:
        ctx.destroy_event(e)
    return ms[iters // 2]

SHAPES = ((16, 2, 128 << 10, 1024, "enc", 0), (16, 2, 128 << 10, 1024, "dec", 0),
          (16, 2, 128 << 10, 4096, "enc", 0), (8, 2, MiB, 512, "enc", 0),
          (8, 2, MiB, 512, "dec", 0), (4, 2, MiB, 1024, "enc", 0), (4, 2, MiB, 1024, "dec", 0),
          (8, 2, MiB, 512, "enc", 8), (8, 2, MiB, 512, "enc", 4),
          (8, 2, MiB, 512, "crc32", 0), (8, 2, MiB, 512, "crc64", 0), (4, 2, MiB, 1024, "crc64", 0),
          (8, 3, MiB, 512, "enc3", 0), (8, 3, MiB, 512, "dec3", 0), (4, 3, MiB, 1024, "enc3", 0),
          (16, 3, 128 << 10, 1024, "enc3", 0),
          (8, 2, MiB, 512, "upd1", 0), (8, 2, MiB, 512, "upd2", 0), (8, 2, MiB, 512, "upd3", 0),
          (8, 2, MiB, 512, "upd4", 0), (4, 2, MiB, 1024, "upd1", 0),
          (16, 2, 128 << 10, 1024, "upd1", 0))
ops = os.environ.get("EC_OPS", "enc,dec").split(",")
orders = [int(o) for o in os.environ.get("EC_ORDERS", "0").split(",")]
res = {}
for k, p, C, S, op, off in (s for s in SHAPES if s[4] in ops):
    if op.startswith("upd"):
        # delta parity update of n cells per stripe: parity ^= coef * (old ^ new)
        n = int(op[3:])
        cells = [3, 6, 0, 5][:n] if k > 6 else [0, 1, 2, 3][:n]
        old, new = ctx.alloc(S * n * C), ctx.alloc(S * n * C)
        old.fill(0x11)
        new.fill(0x5E)
        pitch = S * C + 4096
        par = ctx.alloc(p * pitch + 64)
        fn = lambda: ctx.update(k, p, C, S, cells, old.ptr, new.ptr, n * C, par.ptr, pitch, C)
        bufs = (old, new, par)
        rows = p
        alg_over = (2 * n + 2 * p) * C * S
    elif op.startswith("crc"):
        # encode + checksums of the parity over 32 KiB chunks (the fused kernel), back to back
        data = ctx.alloc(S * k * C + 64)
        pitch = S * C + 4096
        par = ctx.alloc(p * pitch + 64)
        out = ctx.alloc(p * S * (C // 32768) * 8)
        data.fill(0x3C)
        ht = ecg.HASH_CRC32 if op == "crc32" else ecg.HASH_CRC64
        fn = lambda: ctx.encode_csum(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C, ht, 32768, 1, out.ptr)
        bufs = (data, par, out)
        rows = p
    elif op in ("enc", "enc3"):
        data = ctx.alloc(S * k * C + 64)
        pitch = S * C + 4096
        par = ctx.alloc(p * pitch + 64)
        data.fill(0x3C)
        fn = lambda: ctx.encode(k, p, C, S, data.ptr, k * C, par.ptr + off, pitch, C)
        bufs = (data, par)
        rows = p
    else:
        img = ctx.alloc(S * (k + p) * C)
        img.fill(0x3C)
        errs = [0, 1, 2] if op == "dec3" else [0, 1]
        fn = lambda: ctx.recover(k, p, C, S, img.ptr, (k + p) * C, errs)
        bufs = (img,)
        rows = len(errs)
    alg = alg_over if op.startswith("upd") else (k + rows) * C * S
    for cap in ((255, 2) if k >= 16 else (255, 3) if k >= 8 else (255,)):
        if (off or op.startswith("crc") or op.startswith("upd")) and cap != 255:
            continue
        for order in orders:
            ctx.set_wg_per_cu(cap)
            ctx.set_order(order)
            ms = timed(fn)
            tag = "EC_%%dP%%d_%%dK_x%%d_%%s%%s_cap%%s%%s" %% (k, p, C >> 10, S, op, "_off%%d" %% off if off else "",
                                                  cap if cap != 255 else "none", "_o%%d" %% order if order else "")
            res[tag] = {"ms": round(ms, 4), "GBps": round(alg / ms / 1e6, 1), "kernel": ecg.last_kernel()}
    ctx.set_wg_per_cu(0)
    ctx.set_order(0)
    for b in bufs:
        b.free()
print(json.dumps(res))
''' % ROOT


def main():
    libs = [a.split("=", 1) for a in sys.argv[1:]]
    rounds = int(os.environ.get("EC_ROUNDS", "3"))
    out = {name: [] for name, _ in libs}
    env = dict(os.environ, ECG_AUTOTUNE="0")
    for rnd in range(rounds):
        order = libs[rnd % len(libs):] + libs[:rnd % len(libs)]
        for name, lib in order:
            r = subprocess.run([sys.executable, "-c", CHILD, os.path.abspath(lib)], capture_output=True, text=True,
                               timeout=300, env=env)
            if r.returncode != 0:
                print(r.stdout, r.stderr, flush=True)
                raise SystemExit(r.returncode)
            row = json.loads(r.stdout.strip().splitlines()[-1])
            out[name].append(row)
            print(name, rnd, json.dumps({k: v["ms"] for k, v in row.items()}), flush=True)
    summary = {}
    for name, rows in out.items():
        for tag in rows[0]:
            ms = sorted(r[tag]["ms"] for r in rows)
            summary.setdefault(tag, {})[name] = {"ms_median": ms[len(ms) // 2], "ms_all": ms,
                                                 "kernel": rows[0][tag]["kernel"]}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "ec_ab.json"), "w") as f:
        json.dump({"runs": out, "summary": summary}, f, indent=1)
    for tag, per in summary.items():
        print(tag, {n: v["ms_median"] for n, v in per.items()})


if __name__ == "__main__":
    main()
