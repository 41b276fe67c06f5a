"""Where the EC_16P2 / EC_8P2-decode gap to the measured mix comes from:
the kernels' rate against the relative placement of their streams in HBM
(VERDICT r02 item 7).  Device-resident, seeded random bytes, one big
allocation carved by offsets:
  * enc16: EC_16P2 128 KiB x 1024 encode, data [S][k][C] at the arena start,
    parity rows [p][S][C] (pitch S*C + 4 KiB) at data_end + delta;
  * dec8:  EC_8P2 1 MiB x 512 {d0,d1} decode in [S][k+p][C] at arena + delta;
delta over 4 KiB steps to 256 KiB and the powers of two to 64 MiB, each with
the product kernel uncapped and at 2 (k = 16) / 3 (k = 8) blocks per CU.
Every configuration's launches are interleaved round by round (the clock
drifts over a run); median of 7 after 3 warm-up rounds.
usage: python tools/placement_sweep.py -> gpurun_out/placement_sweep.json.
Bench infrastructure."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402
from tools.datagen import stripe_bytes  # noqa: E402

KiB, MiB = 1 << 10, 1 << 20
DELTAS = list(range(0, 256 * KiB, 4 * KiB)) + [256 * KiB << i for i in range(9)]


def main():
    ctx = ecg.Context(0)
    a, b = ctx.event(), ctx.event()
    arena = ctx.alloc(7 << 30)
    blk = stripe_bytes(256 << 20, 17)
    for off in range(0, arena.nbytes, blk.size):
        arena.upload(blk[:min(blk.size, arena.nbytes - off)], offset=off)
    ctx.sync()
    res = {}
    cases = []
    # enc16: data 2 GiB, parity 2 x (128 MiB + 4 KiB) after data_end + delta
    k, p, C, S = 16, 2, 128 * KiB, 1024
    pitch = S * C + 4 * KiB
    for d in DELTAS:
        assert k * S * C + d + p * pitch <= arena.nbytes
        par = arena.ptr + k * S * C + d
        cases.append((f"enc16_d{d // KiB}K", d, 2, (k + p) * C * S,
                      lambda par=par: ctx.encode(k, p, C, S, arena.ptr, k * C, par, pitch, C)))
    # dec8: [S][10][1 MiB] = 5 GiB at arena + delta
    k8, p8, C8, S8 = 8, 2, MiB, 512
    for d in DELTAS:
        assert d + S8 * (k8 + p8) * C8 <= arena.nbytes
        base = arena.ptr + d
        cases.append((f"dec8_d{d // KiB}K", d, 3, (k8 + 2) * C8 * S8,
                      lambda base=base: ctx.recover(k8, p8, C8, S8, base, (k8 + p8) * C8, [0, 1])))
    cfgs = [(name, d, cap, alg, fn) for name, d, c, alg, fn in cases for cap in (255, c)]
    ts = {(n, cap): [] for n, _, cap, _, _ in cfgs}
    for rnd in range(10):
        for n, d, cap, alg, fn in cfgs:
            ctx.set_wg_per_cu(cap)
            ctx.record(a)
            fn()
            ctx.record(b)
            ms = ctx.elapsed_ms(a, b)
            if rnd >= 3:
                ts[(n, cap)].append(ms)
        print("round", rnd, flush=True)
    ctx.set_wg_per_cu(0)
    for n, d, cap, alg, fn in cfgs:
        v = sorted(ts[(n, cap)])
        ms = v[len(v) // 2]
        res.setdefault(n, {"delta": d})[f"cap{cap}_GBps"] = round(alg / ms / 1e6, 1)
    res["_arena_ptr_mod_1GiB"] = arena.ptr % (1 << 30)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "placement_sweep.json"), "w"), indent=1)
    for n in res:
        if not n.startswith("_"):
            print(n, res[n])
    ctx.close()


if __name__ == "__main__":
    main()
