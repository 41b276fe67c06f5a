"""Latency of one small synchronous batch (EC_8P2, S stripes of C-byte cells,
device-resident): the strided encode, a pointer-table launch on an affine
table (runs the strided kernel, no table upload) and on a shuffled table
(table H2D + pointer-table kernel), each call followed by a stream sync.
Median of 200 after 20.  -> one JSON line per (C, S).  Bench infrastructure."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("ECG_AUTOTUNE", "0")
from daos_amd import ecg  # noqa: E402

if os.environ.get("ECG_TEST_LIB"):
    ecg.LIB_PATH = os.path.abspath(os.environ["ECG_TEST_LIB"])


def med_us(fn, ctx, n=200, warm=20):
    for _ in range(warm):
        fn()
        ctx.sync()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ctx.sync()
        ts.append(time.perf_counter() - t0)
    return round(sorted(ts)[n // 2] * 1e6, 1)


def main():
    ctx = ecg.Context(0)
    lib = ecg.lib()
    k, p = 8, 2
    coef = np.ascontiguousarray(ecg.cauchy1(k, p)[k:])
    cptr = coef.ctypes.data_as(C.POINTER(C.c_ubyte))
    for Cb, S in ((32768, 1), (32768, 16), (131072, 16), (131072, 64)):
        buf = ctx.alloc(S * (k + p) * Cb)
        buf.fill(0x3C)

        def cells(order):
            out = []
            for s in order:
                base = buf.ptr + int(s) * (k + p) * Cb
                out += [base + j * Cb for j in range(k + p)]
            return (C.c_void_p * len(out))(*out)

        aff = cells(range(S))
        shuf = cells(np.random.default_rng(S).permutation(S) if S > 1 else [0])
        # S == 1: make the table non-affine by swapping two data cells
        if S == 1:
            shuf[0], shuf[1] = shuf[1], shuf[0]
        h = ctx.h
        res = {"k": k, "p": p, "cell_bytes": Cb, "stripes": S}
        res["strided_us"] = med_us(lambda: ctx.matmul(coef, Cb, S, buf.ptr, [j * Cb for j in range(k)],
                                                      (k + p) * Cb, buf.ptr + k * Cb, [r * Cb for r in range(p)],
                                                      (k + p) * Cb, 0), ctx)
        res["ptrs_affine_us"] = med_us(lambda: ecg._chk(lib.ecg_matmul_ptrs(h, k, p, cptr, Cb, S, aff, None), "p"), ctx)
        res["ptrs_table_us"] = med_us(lambda: ecg._chk(lib.ecg_matmul_ptrs(h, k, p, cptr, Cb, S, shuf, None), "p"), ctx)
        res["table_kernel"] = ecg.last_kernel()
        print(json.dumps(res), flush=True)
        buf.free()
    ctx.close()


if __name__ == "__main__":
    main()
