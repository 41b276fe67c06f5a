"""What makes EC_16P2 128 KiB x 1024 encode slower after other shapes ran
in the same process (profiles/r03/tuner_check/): blocks of back-to-back
launches, uncapped and at 2 blocks per CU, (1) on fresh buffers A in a fresh
process, (2) after an EC_8P2 1 MiB x 512 decode phase (its 5 GiB image
allocated, filled, recovered 30 times, freed) on the same buffers A, (3) on
newly allocated buffers B, (4) on A again.  Separates GPU/HBM state from
where the buffers landed.  usage: python tools/state_check.py ->
gpurun_out/state_check.json.  Bench infrastructure."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402
import bench  # noqa: E402

K, P, C, S = 16, 2, 128 << 10, 1024


def bufs(ctx, seed):
    data = ctx.alloc(S * K * C)
    bench.fill_device(ctx, data, S * K * C, seed)
    pitch = S * C + bench.PARITY_ROW_PAD
    par = ctx.alloc(P * pitch)
    return data, par, pitch


def measure(ctx, b, rounds=3):
    data, par, pitch = b

    def enc():
        ctx.encode(K, P, C, S, data.ptr, K * C, par.ptr, pitch, C)

    out = {"uncapped": [], "cap2": []}
    for r in range(rounds):
        for n, w in ((("uncapped", 255), ("cap2", 2)) if r % 2 == 0 else (("cap2", 2), ("uncapped", 255))):
            ctx.set_wg_per_cu(w)
            out[n].append(round(bench.time_kernel(ctx, enc, 15, warm=5), 4))
    ctx.set_wg_per_cu(0)
    return out


def decode_phase(ctx):
    k, p, C8, S8 = 8, 2, 1 << 20, 512
    st = (k + p) * C8
    img = ctx.alloc(S8 * st)
    bench.fill_device(ctx, img, S8 * st, 7)
    ctx.encode(k, p, C8, S8, img.ptr, st, img.ptr + k * C8, C8, st)
    for _ in range(30):
        ctx.recover(k, p, C8, S8, img.ptr, st, [0, 1])
    ctx.sync()
    img.free()


def main():
    ctx = ecg.Context(0)
    ctx.set_autotune(0)
    res = {}
    a = bufs(ctx, 7)
    res["1_fresh_A"] = measure(ctx, a)
    print(res, flush=True)
    decode_phase(ctx)
    res["2_after_decode_A"] = measure(ctx, a)
    print(res, flush=True)
    b = bufs(ctx, 7)
    res["3_after_decode_new_B"] = measure(ctx, b)
    print(res, flush=True)
    res["4_A_again"] = measure(ctx, a)
    print(res, flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "state_check.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
