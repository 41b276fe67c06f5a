"""Degraded-read byte movement on device-resident data: EC_8P2, 1 MiB cells
(e_len = 1 Mi records of 1 byte), a whole-object fetch of S stripes with
cells d0,d1 lost.  Times ecg_recover on the stripe-list buffer and the
fill-back of the 2*S recovered cells into the user's sgl
(ecg_obj_ec_recov_fill_back, one ecg_copy_segs_kernel launch), with the
sgl's iovs 16-byte aligned and at odd byte offsets, and the copy kernel
against the box's streaming copy rate.  Per-case rate = 10 back-to-back
calls, wall clock (the host walk of one call overlaps the previous call's
copy); the copy kernel's own duration comes from rocprofv3 (gpu_run.sh
fillback_prof: 12 dispatches per case, in case order).  -> gpurun_out/bench_fillback.json.
Bench infrastructure (no oracle)."""
import ctypes as ct
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402


def main():
    ctx = ecg.Context(0)
    L = ecg.lib()
    a, b = ctx.event(), ctx.event()

    def timed(fn, reps=7):
        fn()
        ctx.sync()
        ts = []
        for _ in range(reps):
            ctx.record(a)
            fn()
            ctx.record(b)
            ts.append(ctx.elapsed_ms(a, b))
        ts.sort()
        return ts[len(ts) // 2]

    k, p, C, S = 8, 2, 1 << 20, 128
    srn = k * C
    stripes = ctx.alloc(S * (k + p) * C)
    stripes.fill(0x3C)
    res = {"shape": f"EC_8P2, 1 MiB cells, {S} stripes, cells d0,d1 lost, user sgl = whole object"}
    res["recover_ms"] = round(timed(lambda: ctx.recover(k, p, C, S, stripes.ptr, (k + p) * C, [0, 1])), 4)

    iod = (ecg.Recx * 1)(ecg.Recx(0, S * srn))
    rec = (ecg.RecxEp * S)(*[ecg.RecxEp(ecg.Recx(s * srn, 2 * C), 1, 1, 2) for s in range(S)])
    stl = (ecg.RecxEp * 1)(ecg.RecxEp(ecg.Recx(0, S * srn), 1, 1, 2))
    moved = 2 * C * S
    for iov_kib, skew in ((4096, 0), (4096, 5), (1024, 0), (1024, 11), (65536, 3), (64, 0), (64, 9)):
        n_iov = S * srn // (iov_kib << 10)
        user = ctx.alloc(S * srn + n_iov * 64)
        iovs = (ecg.Iov * n_iov)(*[ecg.Iov(user.ptr + i * ((iov_kib << 10) + 64) + skew, iov_kib << 10, 0)
                                   for i in range(n_iov)])
        sgl = ecg.Sgl(n_iov, 0, iovs)

        def fb():
            rc = L.ecg_obj_ec_recov_fill_back(ctx.h, 1, 0, iod, 1, ct.byref(sgl), rec, S, stl, 1, stripes.ptr,
                                              (k + p) * C, srn, None)
            assert rc == 0, L.ecg_strerror()

        fb()
        fb()
        ctx.sync()
        t0 = time.perf_counter()
        for _ in range(10):
            fb()
        ctx.sync()
        ms = (time.perf_counter() - t0) / 10 * 1e3
        res[f"fill_back_iov{iov_kib}KiB_skew{skew}"] = {
            "n_iov": n_iov, "copied_bytes": moved, "pipelined_ms_per_call": round(ms, 4),
            "alg_GBps_pipelined": round(2 * moved / ms / 1e6, 1), "kernel": L.ecg_last_kernel().decode()}
        user.free()
    ctx.set_launch(0, 0, 0)
    x, y = ctx.alloc(1 << 30), ctx.alloc(1 << 30)
    cp = timed(lambda: ctx.copy_kernel(y.ptr, x.ptr, 1 << 30, 0))
    res["stream_copy_1GiB_GBps"] = round(2 * (1 << 30) / cp / 1e6, 1)
    x.free(); y.free(); stripes.free()
    print(json.dumps(res, indent=0))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "bench_fillback.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
