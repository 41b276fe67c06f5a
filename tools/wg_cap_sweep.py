"""Product-kernel blocks-per-CU caps (ecg_set_wg_per_cu) swept over the EC
classes, device-resident: encode in the client layout (data [S][k][C] ->
parity [p][S][C] at the padded pitch) and 2-erasure (1 for p = 1) decode in
the recovery layout [S][k+p][C]; caps interleaved launch by launch (the box's
clock drifts over a run), median of 9 after 5 warm-up launches, 3 rounds.
Cells hold seeded random bytes (--const: 0x5A everywhere, as the first sweep);
--b2b times each cap's launches back to back instead (as bench.py's rows).
usage: python tools/wg_cap_sweep.py [caps...] [--const] [--b2b] -> gpurun_out/wg_cap_sweep.json
(algorithmic GB/s).  Bench infrastructure."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402

UNCAPPED = 255
MiB = 1 << 20
SHAPES = [(2, 1, 128 << 10, 1024), (4, 2, MiB, 1024), (4, 3, MiB, 1024), (8, 1, MiB, 512), (8, 2, MiB, 512),
          (8, 3, MiB, 512), (16, 1, 128 << 10, 2048), (16, 2, 128 << 10, 1024), (16, 2, 128 << 10, 4096),
          (16, 3, 128 << 10, 1024), (16, 2, MiB, 256)]


def main():
    caps = [int(c) for c in sys.argv[1:] if not c.startswith("--")] or [UNCAPPED, 2, 3, 4, 5, 6]
    ctx = ecg.Context(0)
    a, b = ctx.event(), ctx.event()
    buf = ctx.alloc(13 << 30)
    if "--const" in sys.argv[1:]:          # constant bytes (the first sweep's fill)
        buf.fill(0x5A)
    else:                                  # seeded random bytes, as bench.py's rows
        from tools.datagen import stripe_bytes

        blk = stripe_bytes(256 << 20, 7)
        for off in range(0, buf.nbytes, blk.size):
            buf.upload(blk[: min(blk.size, buf.nbytes - off)], offset=off)
    ctx.sync()
    res = {}
    for rnd in range(3):
        for k, p, C, S in SHAPES:
            pitch = S * C + 4096
            data, par = buf.ptr, buf.ptr + k * S * C
            assert k * S * C + p * pitch <= buf.nbytes and S * (k + p) * C <= buf.nbytes
            errs = [0, 1] if p >= 2 else [0]
            ops = {"enc": (lambda: ctx.encode(k, p, C, S, data, k * C, par, pitch, C), (k + p) * C * S),
                   "dec": (lambda: ctx.recover(k, p, C, S, buf.ptr, (k + p) * C, errs), (k + len(errs)) * C * S)}
            for op, (fn, alg) in ops.items():
                tag = f"{k}P{p}_{C >> 10}K_x{S}_{op}"
                for cap in caps:
                    ctx.set_wg_per_cu(cap)
                    for _ in range(5):
                        fn()
                ctx.sync()
                ts = {cap: [] for cap in caps}
                if "--b2b" in sys.argv[1:]:       # each cap's launches back to back, as bench.py
                    for cap in caps:
                        ctx.set_wg_per_cu(cap)
                        for _ in range(3):
                            fn()
                        for _ in range(9):
                            ctx.record(a)
                            fn()
                            ctx.record(b)
                            ts[cap].append(ctx.elapsed_ms(a, b))
                else:
                    for _ in range(9):
                        for cap in caps:
                            ctx.set_wg_per_cu(cap)
                            ctx.record(a)
                            fn()
                            ctx.record(b)
                            ts[cap].append(ctx.elapsed_ms(a, b))
                row = res.setdefault(tag, {})
                for cap, v in ts.items():
                    v.sort()
                    row.setdefault(str(cap), []).append(round(alg / v[len(v) // 2] / 1e6, 1))
                best = max(row, key=lambda c: sum(row[c]) / len(row[c]))
                print(rnd, tag, {c: row[c][-1] for c in row}, "best", best, flush=True)
    ctx.set_wg_per_cu(0)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "wg_cap_sweep.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
