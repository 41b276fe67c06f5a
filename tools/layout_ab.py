"""Parity-row placement A/B (VERDICT r04 item 4 follow-up): client-layout
encode of EC_4P2 1 MiB x 1024 and EC_8P2 1 MiB x 512 with the p parity rows
  padded    one buffer, pitch S*C + 4 KiB (the headline's layout)
  unpadded  one buffer, pitch S*C
  sepN      p separate hipMalloc allocations, the N-th placement (dummy
            allocations of 2 MiB * N between them move the rows' relative
            offset), as obj_ec_pbufs_init allocates oer_pbufs
            (ref:src/object/cli_ec.c:75-97)
and, for each, the kernel's block orders 0-3 (ecg_set_launch_order: 2D grid /
stripe-fastest / XCD-blocked) -- does a traversal order undo an unlucky
placement?  Launches interleaved (bench.time_interleaved), medians in ms;
prints one JSON line per shape.  Bench infrastructure."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from daos_amd import ecg  # noqa: E402


def main():
    ctx = ecg.Context(0)
    out = []
    for name, k, p, C, S in (("EC_4P2_1MiB_x1024", 4, 2, 1 << 20, 1024), ("EC_8P2_1MiB_x512", 8, 2, 1 << 20, 512)):
        data = ctx.alloc(S * k * C)
        bench.fill_device(ctx, data, S * k * C, 10)
        padded = ctx.alloc(p * (S * C + 4096))
        unpadded = ctx.alloc(p * S * C)
        coef = ecg.cauchy1(k, p)[k:]
        soff = [j * C for j in range(k)]
        layouts = {"padded": lambda: ctx.encode(k, p, C, S, data.ptr, k * C, padded.ptr, S * C + 4096, C),
                   "unpadded": lambda: ctx.encode(k, p, C, S, data.ptr, k * C, unpadded.ptr, S * C, C)}
        keep = []
        for n in range(3):
            rows = []
            for r in range(p):
                rows.append(ctx.alloc(S * C))
                if r < p - 1 and n:
                    keep.append(ctx.alloc(n * (2 << 20)))
            keep += rows
            base = min(b.ptr for b in rows)
            doff = [b.ptr - base for b in rows]
            layouts[f"sep{n}"] = (lambda base=base, doff=doff:
                                  ctx.matmul(coef, C, S, data.ptr, soff, k * C, base, doff, C))
            layouts[f"sep{n}_offsets_MiB"] = [round(d / 2 ** 20, 3) for d in doff]
        fns = {kk: v for kk, v in layouts.items() if callable(v)}
        res = {"shape": name}
        for order in range(4):
            ctx.set_order(order)
            ms = dict(zip(fns, bench.time_interleaved(ctx, list(fns.values()), 11, warm=20)))
            res[f"order{order}"] = {kk: {"ms": round(v, 4), "of_padded_order0": None} for kk, v in ms.items()}
        ctx.set_order(0)
        ref = res["order0"]["padded"]["ms"]
        for order in range(4):
            for kk, v in res[f"order{order}"].items():
                v["of_padded_order0"] = round(ref / v["ms"], 4)
        res["sep_offsets_MiB"] = {kk: v for kk, v in layouts.items() if not callable(v)}
        out.append(res)
        print(json.dumps(res), flush=True)
        for b in [data, padded, unpadded] + keep:
            b.free()
    ctx.close()


if __name__ == "__main__":
    main()
