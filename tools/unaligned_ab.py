"""Misaligned operands: the launch's own choice (variant 0: funnel-shifted
source dwords for sources at any byte, misaligned dword stores for
destinations at any byte; before round 4's change, a bytewise head + shifted
body or the byte kernel) against dword lanes issued at the misaligned
addresses themselves for the sources too (variant 3).  (Round 5's runs also
timed variants 4 -- 16-byte lanes at the misaligned addresses -- and 5 -- the
g2 lanes before they became the k = 8 default; both launch variants were
removed from the product afterwards, their logs are in
profiles/r05/unaligned_ab/.)  Client-layout encode, EC_8P2 1 MiB x 512 and EC_4P2 / EC_16P2 /
EC_2P1 rows; ECG_TEST_LIB = an experimental build, UNALIGNED_CASES = a
comma list of case names, UNALIGNED_TAG = output file suffix;
median of 20 back-to-back launches after 10; both variants' parity compared
byte for byte.  usage: python tools/unaligned_ab.py -> gpurun_out/unaligned_ab.json.
Bench infrastructure."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("ECG_AUTOTUNE", "0")
from daos_amd import ecg  # noqa: E402

if os.environ.get("ECG_TEST_LIB"):	# an experimental build (tools/build_exp.sh)
    ecg.LIB_PATH = os.path.abspath(os.environ["ECG_TEST_LIB"])

MiB = 1 << 20
VARIANTS = tuple(int(v) for v in os.environ.get("UNALIGNED_VARIANTS", "0,3").split(","))


def timed(ctx, fn, iters=20, warm=10):
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


def main():
    ctx = ecg.Context(0)
    C = MiB
    res = {}
    # name, (k, p), stripes, data offset, parity offset, extra parity row pitch, cell bytes
    # (cells short of 1 MiB: every cell ends in a partial 4 KiB column)
    cases = (("aligned", (8, 2), 512, 0, 0, 0, C), ("data_off1", (8, 2), 512, 1, 0, 0, C),
             ("data_off4", (8, 2), 512, 4, 0, 0, C), ("data_off8", (8, 2), 512, 8, 0, 0, C),
             ("parity_off1", (8, 2), 512, 0, 1, 0, C), ("parity_off8", (8, 2), 512, 0, 8, 0, C),
             ("parity_off2_data_off1", (8, 2), 512, 1, 2, 0, C), ("parity_off1_unequal", (8, 2), 64, 0, 1, 1, C),
             ("data_off3_parity_off1_unequal", (8, 2), 64, 3, 1, 1, C),
             ("aligned_C-16", (8, 2), 512, 0, 0, 0, C - 16), ("aligned_C-4", (8, 2), 512, 0, 0, 0, C - 4),
             ("data_off1_C-4", (8, 2), 512, 1, 0, 0, C - 4), ("C-3", (8, 2), 512, 0, 0, 0, C - 3),
             ("4p2_aligned", (4, 2), 1024, 0, 0, 0, C), ("4p2_data_off1", (4, 2), 1024, 1, 0, 0, C),
             ("4p2_data_off4", (4, 2), 1024, 4, 0, 0, C),
             ("16p2_128K_aligned", (16, 2), 1024, 0, 0, 0, 128 << 10),
             ("16p2_128K_data_off1", (16, 2), 1024, 1, 0, 0, 128 << 10),
             ("16p2_128K_data_off4", (16, 2), 1024, 4, 0, 0, 128 << 10),
             ("2p1_128K_data_off1", (2, 1), 1024, 1, 0, 0, 128 << 10))
    only = os.environ.get("UNALIGNED_CASES")
    for name, (k, p), S, doff, poff, extra, C in cases:
        if only and name not in only.split(","):
            continue
        data = ctx.alloc(S * k * C + 64)
        data.fill(0x3C)
        data.upload(np.random.default_rng(S + doff).integers(0, 256, 64 * MiB, dtype=np.uint8))
        pitch = S * C + 4096 + extra
        par = ctx.alloc(p * pitch + 64)
        row = {"k": k, "p": p, "cell_bytes": C, "stripes": S}
        outs = {}
        for variant in VARIANTS:
            ctx.set_launch(0, 0, variant)
            fn = lambda: ctx.encode(k, p, C, S, data.ptr + doff, k * C, par.ptr + poff, pitch, C)
            par.fill(0)
            ms = timed(ctx, fn)
            alg = (k + p) * C * S
            row[f"v{variant}"] = {"ms": round(ms, 4), "alg_GBps": round(alg / ms / 1e6, 1),
                                  "kernel": ecg.last_kernel()}
            outs[variant] = par.download()
        ctx.set_launch(0, 0, 0)
        for v in VARIANTS[1:]:
            row[f"v{v}_over_v0"] = round(row["v0"]["ms"] / row[f"v{v}"]["ms"], 4)
        row["equal"] = all(bool(np.array_equal(outs[VARIANTS[0]], outs[v])) for v in VARIANTS[1:])
        res[name] = row
        print(name, json.dumps(row), flush=True)
        data.free()
        par.free()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    tag = os.environ.get("UNALIGNED_TAG", "")
    with open(os.path.join(ROOT, "gpurun_out", f"unaligned_ab{tag}.json"), "w") as f:
        json.dump(res, f, indent=1)
    assert all(r["equal"] for r in res.values()), "a variant's parity differs"


if __name__ == "__main__":
    main()
