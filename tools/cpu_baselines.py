"""CPU baseline rows of BASELINE.md §3 on the GPU box's host: the oracle's
ISA-L-equivalent restatement (scalar ec_encode_data_base and the SIMD
nibble-table / GFNI variant, OpenMP over stripes) on bounded samples of each
BASELINE config, 1 core and the box's CPU share (16).  Reported baseline,
not the optimisation target.  -> gpurun_out/cpu_baselines.json.

Test/bench infrastructure: imports oracle/ (allowed for cpu_baseline legs).
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import ref  # noqa: E402
from tools.datagen import stripe_bytes  # noqa: E402

GIB = float(1 << 30)
BUDGET_S = float(os.environ.get("CPU_BASELINE_SECONDS", "3"))


def rate(fn, user_bytes):
    fn()                                    # warm (page faults, OpenMP pool)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < BUDGET_S:
        fn()
        n += 1
    dt = time.perf_counter() - t0
    return round(n * user_bytes / dt / GIB, 3), round(dt, 2), n


def main():
    cores = max(1, min(16, len(os.sched_getaffinity(0))))
    variant = {0: "scalar", 1: "avx2-vpshufb", 2: "gfni-avx512"}[ref.simd_variant()]
    out = {"cpu_model": "", "cores_used_max": cores, "simd_variant": variant, "budget_s": BUDGET_S}
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                out["cpu_model"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    rows = {}
    # (name, k, p, C, sample stripes, op)
    for name, k, p, C, S, op in (("EC_2P1_128KiB_encode", 2, 1, 128 << 10, 256, "enc"),
                                 ("EC_4P2_1MiB_encode", 4, 2, 1 << 20, 32, "enc"),
                                 ("EC_8P2_1MiB_decode_d0d1", 8, 2, 1 << 20, 16, "dec"),
                                 ("EC_16P2_128KiB_encode", 16, 2, 128 << 10, 64, "enc")):
        data = stripe_bytes(S * k * C, 3)
        par = np.empty(p * S * C, dtype=np.uint8)
        stripes = None
        if op == "dec":
            stripes = np.zeros(S * (k + p) * C, dtype=np.uint8)
            sv = stripes.reshape(S, k + p, C)
            sv[:, :k] = data.reshape(S, k, C)
            sv[:, k:] = ref.encode_batch(k, p, C, S, data, nthreads=cores, simd=True).reshape(p, S, C) \
                .transpose(1, 0, 2)
            rc, de, dec, el, gt, _ = ref.recov_codec(k, p, [0, 1])
            assert rc == 0
        for simd in (False, True):
            for nt in (1, cores):
                if not simd and nt != 1:
                    continue
                if op == "enc":
                    fn = (lambda k=k, p=p, C=C, S=S, nt=nt, simd=simd:
                          ref.encode_batch(k, p, C, S, data, nthreads=nt, simd=simd, out=par))
                else:
                    fn = (lambda k=k, C=C, S=S, nt=nt, simd=simd, gt=gt, dec=dec, el=el, p=p:
                          ref.recov_batch(k, 2, gt, dec, el, C, (k + p) * C, S, stripes, nthreads=nt, simd=simd))
                v, dt, n = rate(fn, k * C * S)
                rows[f"{name}_{'simd' if simd else 'scalar'}_{nt}c"] = {
                    "GiBps_user": v, "cores": nt, "variant": variant if simd else "scalar",
                    "sample": f"{S} stripes x {n} reps in {dt} s"}
                print(name, simd, nt, v, flush=True)
    out["rows"] = rows
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "cpu_baselines.json"), "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
