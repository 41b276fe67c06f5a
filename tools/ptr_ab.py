"""Pointer-table product (ecg_matmul_ptrs: ISA-L's data[] / coding[] batched
over stripes, the client's in-place sgl encode) against the offset kernel
(ecg_encode) on the same client layout -- data [S][k][C], parity rows
[p][S][C] -- uncapped and at the candidate blocks-per-CU cap.  The pointer
table is built once; each timed call uploads it (part of the path) and
launches.  Median of 30 back-to-back calls after 40; tuner off.  Env:
PTR_SHUFFLE, PTR_GX_DIVS, PTR_DATA_OFF, PTR_TAG, ECG_TEST_LIB (below).
-> gpurun_out/ptr_ab.json.  Bench infrastructure."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("ECG_AUTOTUNE", "0")
from daos_amd import ecg  # noqa: E402

MiB = 1 << 20
# PTR_GX_DIVS: the pointer-table grid's x dimension = columns / d, so each
# block walks d columns of its stripe (the stripe's table row loaded once)
GX_DIVS = [int(d) for d in os.environ.get("PTR_GX_DIVS", "1").split(",")]
# PTR_SHUFFLE=1: the table lists the stripes in a shuffled order -- the same
# cells, no longer an affine table, so the pointer-table kernel runs
SHUFFLE = os.environ.get("PTR_SHUFFLE") == "1"
# PTR_DATA_OFF: the data cells start this many bytes into their buffer (user
# sgl cells in place at any byte); PTR_TAG: output file suffix
DATA_OFF = int(os.environ.get("PTR_DATA_OFF", "0"))
TAG = os.environ.get("PTR_TAG", "")
if os.environ.get("ECG_TEST_LIB"):
    ecg.LIB_PATH = os.path.abspath(os.environ["ECG_TEST_LIB"])


def timed(ctx, fn, iters=30, warm=40):
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
    lib = ecg.lib()
    res = {}
    for k, p, Cb, S in ((4, 2, MiB, 1024), (8, 2, MiB, 512), (16, 2, 128 << 10, 1024), (2, 1, 128 << 10, 1024)):
        coef = np.ascontiguousarray(ecg.cauchy1(k, p)[k:])
        cptr = coef.ctypes.data_as(C.POINTER(C.c_ubyte))
        data = ctx.alloc(S * k * Cb + 64)
        data.fill(0x3C)
        pitch = S * Cb + 4096
        par = ctx.alloc(p * pitch)
        cells = []
        order = np.random.default_rng(S).permutation(S) if SHUFFLE else range(S)
        for s in order:
            cells += [data.ptr + DATA_OFF + (int(s) * k + j) * Cb for j in range(k)]
            cells += [par.ptr + r * pitch + int(s) * Cb for r in range(p)]
        arr = (C.c_void_p * len(cells))(*cells)
        h = ctx.h

        def ptr_call():
            ecg._chk(lib.ecg_matmul_ptrs(h, k, p, cptr, Cb, S, arr, None), "matmul_ptrs")

        def off_call():
            ctx.encode(k, p, Cb, S, data.ptr + DATA_OFF, k * Cb, par.ptr, pitch, Cb)

        alg = (k + p) * Cb * S
        nchunk = Cb // 4096
        for cap in ((0, 2) if k >= 8 else (0,)):
            for name, fn, divs in (("offset", off_call, (1,)), ("ptr", ptr_call, GX_DIVS)):
                for dv in divs:
                    ctx.set_wg_per_cu(cap)
                    ctx.set_launch(nchunk // dv if dv > 1 else 0, 0, 0)
                    ms = timed(ctx, fn)
                    tag = f"EC_{k}P{p}_{Cb >> 10}K_x{S}_{name}_cap{cap}" + (f"_cols{dv}" if dv > 1 else "")
                    res[tag] = {"ms": round(ms, 4), "alg_GBps": round(alg / ms / 1e6, 1),
                                "kernel": ecg.last_kernel()}
                    print(tag, res[tag], flush=True)
        ctx.set_wg_per_cu(0)
        ctx.set_launch(0, 0, 0)
        data.free()
        par.free()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"ptr_ab{TAG}.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
