"""Main offset-based product kernel vs the pointer-table kernel on the same
layouts (the pointer kernel keeps cell bases in SGPRs: 64 vs 116 VGPRs at
EC_8P2) -> gpurun_out/tune9.json."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
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

    res = {}
    for k, p, C, S in ((4, 2, 1 << 20, 1024), (8, 2, 1 << 20, 512), (16, 2, 128 << 10, 1024),
                       (2, 1, 128 << 10, 1024)):
        data = ctx.alloc(S * k * C); data.fill(0x5A)
        pitch = S * C + 4096
        par = ctx.alloc(p * pitch)
        en = ecg.cauchy1(k, p)
        enc = timed(lambda: [ctx.encode(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C) for _ in range(5)]) / 5
        import ctypes as ct
        cells = []
        for s in range(S):
            cells += [data.ptr + s * k * C + j * C for j in range(k)]
            cells += [par.ptr + r * pitch + s * C for r in range(p)]
        arr = (ct.c_void_p * len(cells))(*cells)
        co = np.ascontiguousarray(en[k:]).reshape(-1)
        L = ecg.lib()

        def ptr_calls(n=5):
            for _ in range(n):
                L.ecg_matmul_ptrs(ctx.h, k, p, co.ctypes.data_as(ecg.u8p), C, S, arr, None)
        alg = (k + p) * C * S
        row = {"offset_kernel_ms": round(enc, 4), "offset_GBps": round(alg / enc / 1e6, 1)}
        nchunk = C // 4096
        for gx in (nchunk, 64, 32, 16, 8, 4, 2):
            if gx > nchunk:
                continue
            ctx.set_launch(gx, 0, 0)
            ptr_calls(2)
            ptr = timed(ptr_calls) / 5
            row[f"ptr_gx{gx}_GBps"] = round(alg / ptr / 1e6, 1)
        ctx.set_launch(0, 0, 0)
        row["ptr_kernel"] = ecg.last_kernel()
        res[f"{k}p{p}_{C >> 10}K"] = row
        data.free(); par.free()
    print(json.dumps(res, indent=0))
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "tune9.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
