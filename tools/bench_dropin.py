"""Latency of the synchronous ISA-L drop-in (ec_encode_data, one EC_8P2
stripe per call, through ctypes with the pointer arrays built once, as
the C tool does) by cell size.  At the default crossover host cells run the product
CPU path; with ECG_DROPIN_CROSSOVER=0 they take the GPU staging, once per
staging mode (env ECG_ZERO_COPY_MAX: 0 = always DMA copies, large = kernel on
the pinned staging in place); DROPIN_DEVICE=1: device cells.  Appends one JSON
line (with the kernel each size ran) to gpurun_out/bench_dropin.jsonl.  The
same without ctypes, and the crossover: tools/dropin_bench.c.  Bench infrastructure (no oracle)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from daos_amd import ecg  # noqa: E402


def main():
    k, p = 8, 2
    tbls = ecg.isal_init_tables(ecg.cauchy1(k, p)[k:])
    rng = np.random.default_rng(5)
    device = os.environ.get("DROPIN_DEVICE") == "1"
    res = {"zero_copy_max": os.environ.get("ECG_ZERO_COPY_MAX", "default"), "cells": "device" if device else "host",
           "crossover": os.environ.get("ECG_DROPIN_CROSSOVER", "default")}
    ctx = ecg.Context(0) if device else None
    L = ecg.lib()
    for C in (4096, 16384, 32768, 65536, 131072, 262144, 1 << 20):
        if device:
            buf = ctx.alloc((k + p) * C)
            buf.fill(0x5A)
            dp = (ecg.u8p * k)(*[ecg.C.cast(ecg.C.c_void_p(buf.ptr + j * C), ecg.u8p) for j in range(k)])
            cp = (ecg.u8p * p)(*[ecg.C.cast(ecg.C.c_void_p(buf.ptr + (k + r) * C), ecg.u8p) for r in range(p)])
            tp = tbls.ctypes.data_as(ecg.u8p)

            def call():
                L.ec_encode_data(C, k, p, tp, dp, cp)
        else:
            cells = [rng.integers(0, 256, C, dtype=np.uint8) for _ in range(k)]
            coding = [np.zeros(C, dtype=np.uint8) for _ in range(p)]
            dp = (ecg.u8p * k)(*[c.ctypes.data_as(ecg.u8p) for c in cells])
            cp = (ecg.u8p * p)(*[c.ctypes.data_as(ecg.u8p) for c in coding])
            tp = tbls.ctypes.data_as(ecg.u8p)

            def call():
                L.ec_encode_data(C, k, p, tp, dp, cp)
        for _ in range(5):
            call()
        it = 200 if C <= 65536 else 40
        t0 = time.perf_counter()
        for _ in range(it):
            call()
        us = (time.perf_counter() - t0) / it * 1e6
        res[f"{C >> 10}KiB_us"] = round(us, 1)
        res[f"{C >> 10}KiB_kernel"] = ecg.last_kernel()
        res[f"{C >> 10}KiB_GiBps"] = round(k * C / (us / 1e6) / (1 << 30), 2)
        if device:
            buf.free()
    print(json.dumps(res), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "bench_dropin.jsonl"), "a") as f:
        f.write(json.dumps(res) + "\n")


if __name__ == "__main__":
    main()
