"""Launch tuner vs explicit geometries, EC_16P2 128 KiB x 1024 and EC_8P2
1 MiB x 512 encode in the client layout (bench.py's detail rows): blocks of
B back-to-back launches -- uncapped (wg_per_cu 255), capped (2 / 3), and the
autotuned default -- in rotated order, R rounds; per block the median, plus
the tuner's own arm medians.  Launches within a block have events at every
boundary and no host wait between them (bench.time_interleaved).
usage: python tools/tuner_check.py -> gpurun_out/tuner_check.json.
Bench infrastructure."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402
import bench  # noqa: E402


def main():
    ctx = ecg.Context(0)
    res = {}
    churn = int(os.environ.get("CHURN_GIB", "0"))
    if churn:
        # allocation state as bench.py's detail rows leave it: a large image
        # allocated, filled, used and freed before the measured buffers exist
        big = ctx.alloc(churn << 30)
        bench.fill_device(ctx, big, churn << 30, 3)
        ctx.sync()
        big.free()
        res["churn_gib"] = churn
    shapes = (("EC_16P2_128KiB_x1024", 16, 2, 128 << 10, 1024, 2), ("EC_8P2_1MiB_x512", 8, 2, 1 << 20, 512, 3))
    for name, k, p, C, S, cap in shapes[:int(os.environ.get("NSHAPES", "2"))]:
        data = ctx.alloc(S * k * C)
        bench.fill_device(ctx, data, S * k * C, 7)
        pitch = S * C + bench.PARITY_ROW_PAD
        par = ctx.alloc(p * pitch)

        def enc(k=k, p=p, C=C, S=S, data=data, par=par, pitch=pitch):
            ctx.encode(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C)

        cfgs = [("uncapped", 255), (f"cap{cap}", cap), ("auto", 0)]
        rows = {n: [] for n, _ in cfgs}
        ctx.set_autotune(2)
        for rnd in range(6):
            order = cfgs[rnd % 3:] + cfgs[:rnd % 3]
            for n, w in order:
                ctx.set_wg_per_cu(w)
                rows[n].append(round(bench.time_kernel(ctx, enc, 15, warm=10), 4))
        ctx.set_wg_per_cu(0)
        st = ctx.tune_state(k, p, C, S, k * C, C)
        res[name] = {"block_medians_ms": rows,
                     "median_ms": {n: sorted(v)[len(v) // 2] for n, v in rows.items()},
                     "tuner": None if st is None else {"cap": st[0], "uncapped_ms": round(st[1], 4),
                                                       "capped_ms": round(st[2], 4)}}
        print(name, json.dumps(res[name]), flush=True)
        data.free()
        par.free()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", f"tuner_check_churn{churn}.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
