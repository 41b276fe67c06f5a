"""Fused product+checksum: time vs checksum chunk size (4 KiB = one column
per workgroup, like ecg_mm_kernel; larger = the workgroup walks the chunk's
columns in sequence) -> gpurun_out/tune8.json."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg


def main():
    ctx = ecg.Context(0)
    a, b = ctx.event(), ctx.event()

    def timed(fn, reps=9):
        ts = []
        for _ in range(reps):
            ctx.record(a); fn(); ctx.record(b)
            ts.append(ctx.elapsed_ms(a, b))
        ts.sort()
        return ts[len(ts) // 2]

    k, p, C, S = 8, 2, 1 << 20, 256
    data = ctx.alloc(S * k * C); data.fill(0x5A)
    pitch = S * C + 4096
    par = ctx.alloc(p * pitch)
    out = ctx.alloc(p * S * (C // 4096) * 8)
    res = {"encode_ms": timed(lambda: ctx.encode(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C))}
    for cs in (4096, 8192, 16384, 32768, 131072, 1 << 20):
        nch = C // cs
        for cpb in (1, 2, 4, 8):
            gx = max(1, (nch + cpb - 1) // cpb)
            ctx.set_launch(gx, 0, 0)
            res[f"fused_crc32_cs{cs >> 10}K_cpb{cpb}_ms"] = timed(
                lambda: ctx.encode_csum(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C, 2, cs, 1, out.ptr))
        ctx.set_launch(0, 0, 0)
    res = {kk: round(v, 4) for kk, v in res.items()}
    print(json.dumps(res, indent=0))
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "tune8.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
