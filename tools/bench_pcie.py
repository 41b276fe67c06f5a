"""PCIe-inclusive (host-resident) rates -- recorded in DESIGN.md §7; never the
bench.py `value`.

  * raw pinned hipMemcpyAsync H2D / D2H (1 GiB)
  * ecg_encode_host / ecg_recover_host on EC_8P2 1 MiB x 512 stripes in
    pinned memory (3-slot H2D || kernel || D2H pipeline), chunk sweep
  * BASELINE config 5, "rebuild stream": alternating encode and 2-erasure
    recovery batches, host<->device copies included
  * the synchronous one-stripe ISA-L drop-in (ec_encode_data, 1 MiB cells),
    i.e. what an unbatched DAOS caller sees
Writes gpurun_out/pcie.json.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from daos_amd import ecg  # noqa: E402
from tools.datagen import stripe_bytes  # noqa: E402

GIB = float(1 << 30)


def main():
    ctx = ecg.Context(0)
    out = {}
    # raw pinned copies
    n = 1 << 30
    h = ctx.host_alloc(n)
    d = ctx.alloc(n)
    h.array[:] = 7
    for kind, name in ((0, "h2d"), (1, "d2h")):
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            if kind == 0:
                ecg._chk(ecg.lib().ecg_memcpy(ctx.h, d.ptr, h.ptr, n, 0, None), "h2d")
            else:
                ecg._chk(ecg.lib().ecg_memcpy(ctx.h, h.ptr, d.ptr, n, 1, None), "d2h")
            ctx.sync()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        out[f"pinned_{name}_GBps"] = round(n / ts[len(ts) // 2] / 1e9, 2)
    h.free()
    d.free()
    print("raw", out, flush=True)

    k, p, Cb, S = 8, 2, 1 << 20, 512
    data = ctx.host_alloc(S * k * Cb)
    par = ctx.host_alloc(S * p * Cb)
    stripes = ctx.host_alloc(S * (k + p) * Cb)
    blk = stripe_bytes(256 << 20, 9)
    a = data.array
    for off in range(0, a.size, blk.size):
        m = min(blk.size, a.size - off)
        a[off:off + m] = blk[:m]
    ctx.encode_host(k, p, Cb, S, data.array, par.array, chunk=64)
    img = stripes.array.reshape(S, k + p, Cb)
    src = data.array.reshape(S, k, Cb)
    img[:, :k] = src
    img[:, k:] = par.array.reshape(p, S, Cb).transpose(1, 0, 2)

    user = k * Cb * S
    for chunk in (8, 16, 32, 64, 128):
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            ctx.encode_host(k, p, Cb, S, data.array, par.array, chunk=chunk)
            ts.append(time.perf_counter() - t0)
        ts.sort()
        out[f"encode_host_8P2_chunk{chunk}_GiBps"] = round(user / ts[1] / GIB, 2)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            ctx.recover_host(k, p, Cb, S, stripes.array, [0, 1], chunk=chunk)
            ts.append(time.perf_counter() - t0)
        ts.sort()
        out[f"recover_host_8P2_d0d1_chunk{chunk}_GiBps"] = round(user / ts[1] / GIB, 2)
        print(chunk, out[f"encode_host_8P2_chunk{chunk}_GiBps"], out[f"recover_host_8P2_d0d1_chunk{chunk}_GiBps"],
              flush=True)
    # recovered bytes must equal the original data cells
    chk = np.array_equal(stripes.array.reshape(S, k + p, Cb)[:, :k], src)
    out["recover_host_bytes_ok"] = bool(chk)

    # config 5: rebuild stream, alternating batches of 64 stripes
    t0 = time.perf_counter()
    done = 0
    for i in range(0, S, 64):
        if (i // 64) % 2 == 0:
            ctx.encode_host(k, p, Cb, 64, data.array[i * k * Cb:(i + 64) * k * Cb], par.array[: 64 * p * Cb],
                            chunk=16)
        else:
            ctx.recover_host(k, p, Cb, 64, stripes.array[i * (k + p) * Cb:(i + 64) * (k + p) * Cb], [0, 1],
                             chunk=16)
        done += 64
    dt = time.perf_counter() - t0
    out["rebuild_stream_8P2_mixed_GiBps"] = round(done * k * Cb / dt / GIB, 2)

    # one-stripe synchronous ISA-L drop-in path
    tbls = ecg.isal_init_tables(ecg.cauchy1(k, p)[k:])
    cells = [np.frombuffer(blk[j * Cb:(j + 1) * Cb].tobytes(), dtype=np.uint8).copy() for j in range(k)]
    coding = [np.zeros(Cb, dtype=np.uint8) for _ in range(p)]
    ecg.isal_encode_data(tbls, k, p, cells, coding)
    t0 = time.perf_counter()
    it = 50
    for _ in range(it):
        ecg.isal_encode_data(tbls, k, p, cells, coding)
    dt = time.perf_counter() - t0
    out["isal_ec_encode_data_1stripe_8P2_1MiB_us"] = round(dt / it * 1e6, 1)
    out["isal_ec_encode_data_1stripe_8P2_1MiB_GiBps"] = round(it * k * Cb / dt / GIB, 2)
    small = [c[:4096].copy() for c in cells]
    scod = [np.zeros(4096, dtype=np.uint8) for _ in range(p)]
    t0 = time.perf_counter()
    for _ in range(200):
        ecg.isal_encode_data(tbls, k, p, small, scod)
    out["isal_ec_encode_data_1stripe_8P2_4KiB_us"] = round((time.perf_counter() - t0) / 200 * 1e6, 1)
    for b in (data, par, stripes):
        b.free()
    print(json.dumps(out), flush=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "pcie.json"), "w"), indent=1)
    ctx.close()


if __name__ == "__main__":
    main()
