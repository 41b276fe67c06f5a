"""Soak of the synchronous drop-in under concurrency: T threads, each issuing
random ec_encode_data / ec_encode_data_update / xor_gen calls on host cells
(CPU path, or GPU staging in the crossover-0 phase) and on device cells
(HIP kernels on the context's drop-in stream pool), every output checked
against the scalar oracle.  Two phases: default crossover, then 0.  Prints
one JSON line per phase (calls, mismatches, routes seen, seconds).  Test /
bench infrastructure (the oracle is the checker)."""
import ctypes as C
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402
from oracle import ref  # noqa: E402


def worker(ctx, tid, calls, out):
    rng = np.random.default_rng(1000 + tid)
    L = ecg.lib()
    bad, routes = 0, {}
    for i in range(calls):
        op = ("encode", "update", "xor")[int(rng.integers(0, 3))]
        k = 1 if op == "update" else int(rng.choice([2, 3, 4, 8, 16, 24] + ([70] if op == "xor" else [])))
        rows = 1 if op == "xor" else int(rng.integers(1, 9))
        n = int(rng.choice([1, 33, 4096, 4099, 32768, 65536 + 7]))
        device = bool(rng.integers(0, 2))
        coef = np.ones((1, k), np.uint8) if op == "xor" else rng.integers(0, 256, (rows, k), dtype=np.uint8)
        src = rng.integers(0, 256, (k, n), dtype=np.uint8)
        dst0 = rng.integers(0, 256, (rows, n), dtype=np.uint8)
        want = ref.encode_data(coef, src)
        if op == "update":
            want ^= dst0
        stride = n + 32
        soff = [j * stride + int(rng.integers(0, 16)) for j in range(k)]
        doff = [r * stride + int(rng.integers(0, 16)) for r in range(rows)]
        if device:
            sb, db = ctx.alloc(k * stride), ctx.alloc(rows * stride)
            for j in range(k):
                sb.upload(src[j], offset=soff[j])
            for r in range(rows):
                db.upload(dst0[r], offset=doff[r])
            sp, dp = [sb.ptr + o for o in soff], [db.ptr + o for o in doff]
        else:
            hs, hd = np.zeros(k * stride, np.uint8), np.zeros(rows * stride, np.uint8)
            for j in range(k):
                hs[soff[j]: soff[j] + n] = src[j]
            for r in range(rows):
                hd[doff[r]: doff[r] + n] = dst0[r]
            sp, dp = [hs.ctypes.data + o for o in soff], [hd.ctypes.data + o for o in doff]
        if op == "xor":
            v = (C.c_void_p * (k + 1))(*(sp + dp))
            L.xor_gen(k + 1, n, v)
        else:
            tb = ecg.isal_init_tables(coef)
            spp = (ecg.u8p * k)(*[C.cast(C.c_void_p(x), ecg.u8p) for x in sp])
            dpp = (ecg.u8p * rows)(*[C.cast(C.c_void_p(x), ecg.u8p) for x in dp])
            if op == "encode":
                L.ec_encode_data(n, k, rows, tb.ctypes.data_as(ecg.u8p), spp, dpp)
            else:
                L.ec_encode_data_update(n, k, rows, 0, tb.ctypes.data_as(ecg.u8p), spp[0], dpp)
        kern = ecg.last_kernel().split("<")[0]
        routes[kern] = routes.get(kern, 0) + 1
        if device:
            raw = db.download()
            got = np.stack([raw[o: o + n] for o in doff])
            sb.free()
            db.free()
        else:
            got = np.stack([hd[o: o + n] for o in doff])
        bad += int(not np.array_equal(got, want))
    out[tid] = (bad, routes)


def phase(ctx, crossover, threads=16, calls=1000):
    if crossover is not None:
        ecg.set_dropin_crossover(crossover)
    out = {}
    t0 = time.perf_counter()
    th = [threading.Thread(target=worker, args=(ctx, t, calls, out)) for t in range(threads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    routes = {}
    for _, r in out.values():
        for kk, v in r.items():
            routes[kk] = routes.get(kk, 0) + v
    res = {"crossover": "default" if crossover is None else crossover, "threads": threads,
           "calls": threads * calls, "mismatches": sum(b for b, _ in out.values()), "routes": routes,
           "seconds": round(time.perf_counter() - t0, 1)}
    print(json.dumps(res), flush=True)
    return res


def main():
    ctx = ecg.Context(0)
    a = phase(ctx, None)
    b = phase(ctx, 0)
    ctx.close()
    sys.exit(1 if a["mismatches"] or b["mismatches"] else 0)


if __name__ == "__main__":
    main()
