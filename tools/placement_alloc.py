"""Is the blocks-per-CU cap's gain a property of the allocation?  (The
in-allocation sweep, tools/placement_sweep.py, shows the same gain at every
relative offset.)  EC_16P2 128 KiB x 1024 encode and EC_8P2 1 MiB x 512
{d0,d1} decode on SEPARATELY allocated buffers, as bench.py and DAOS
(obj_ec_pbufs_init, ref:src/object/cli_ec.c:75-97) allocate them, over 6
allocation trials (each trial frees the buffers and allocates again behind a
spacer of a different size, so the buffers land elsewhere); per trial the
caps timed interleaved (alternating launches) and back to back (5 launches
of one cap, then the other), median of 7.
usage: python tools/placement_alloc.py -> gpurun_out/placement_alloc.json.  Bench infrastructure."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402
from tools.datagen import stripe_bytes  # noqa: E402

KiB, MiB = 1 << 10, 1 << 20


def fill(buf, blk):
    for off in range(0, buf.nbytes, blk.size):
        buf.upload(blk[:min(blk.size, buf.nbytes - off)], offset=off)


def main():
    ctx = ecg.Context(0)
    a, b = ctx.event(), ctx.event()
    blk = stripe_bytes(256 << 20, 19)

    def timed(fn, cap):
        ctx.set_wg_per_cu(cap)
        ctx.record(a)
        fn()
        ctx.record(b)
        return ctx.elapsed_ms(a, b)

    res = []
    for trial, spacer in enumerate((0, 4 * KiB, 2 * MiB + 4 * KiB, 64 * MiB, 1 << 30, 3 * MiB)):
        sp = ctx.alloc(spacer) if spacer else None
        k, p, C, S = 16, 2, 128 * KiB, 1024
        pitch = S * C + 4 * KiB
        data = ctx.alloc(k * S * C)
        par = ctx.alloc(p * pitch)
        fill(data, blk)
        k8, p8, C8, S8 = 8, 2, MiB, 512
        st = ctx.alloc(S8 * (k8 + p8) * C8)
        fill(st, blk)
        ctx.sync()
        cases = {
            "enc16": (lambda: ctx.encode(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C), (k + p) * C * S, 2),
            "dec8": (lambda: ctx.recover(k8, p8, C8, S8, st.ptr, (k8 + p8) * C8, [0, 1]), (k8 + 2) * C8 * S8, 3),
        }
        row = {"trial": trial, "spacer": spacer, "data_mod_2M": data.ptr % (2 * MiB), "par_mod_2M": par.ptr % (2 * MiB),
               "par_minus_data": par.ptr - data.ptr}
        for name, (fn, alg, cap) in cases.items():
            for _ in range(3):
                timed(fn, 255)
                timed(fn, cap)
            il = {255: [], cap: []}
            for _ in range(7):
                for c in (255, cap):
                    il[c].append(timed(fn, c))
            bb = {255: [], cap: []}
            for _ in range(2):
                for c in (255, cap):
                    for _ in range(5):
                        bb[c].append(timed(fn, c))
            for mode, t in (("il", il), ("b2b", bb)):
                for c, v in t.items():
                    v.sort()
                    row[f"{name}_{mode}_cap{c}_GBps"] = round(alg / v[len(v) // 2] / 1e6, 1)
        ctx.set_wg_per_cu(0)
        print(row, flush=True)
        res.append(row)
        for buf in (data, par, st) + ((sp,) if sp else ()):
            buf.free()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "placement_alloc.json"), "w"), indent=1)
    ctx.close()


if __name__ == "__main__":
    main()
