"""Soak of the batching queue (ecg_queue_*) under concurrency: rounds of
seeded random one-stripe requests -- encodes and in-place recoveries on host
or device cells (device stripes at random byte offsets of one allocation),
one-cell updates on host or device cells, EC classes 2+1 .. 16+3, cells of
1 byte .. 96 KiB -- posted from T threads to one queue, then a flush and every
output compared with the oracle.  Each round draws its host-cell route
(computed on the completion threads below the drop-in crossover, or staged
over PCIe at crossover 0), max_batch and max_wait_us; a last phase runs the
CPU executor (no context).  Prints one JSON line per phase: requests,
mismatches, failed callbacks, batches, seconds.  Test / bench infrastructure
(the oracle is the checker).
usage: python tools/queue_soak.py [rounds] [threads]"""
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

CLASSES = [(2, 1), (4, 2), (8, 2), (8, 3), (16, 2), (16, 3)]
SIZES = [1, 31, 4096, 4100, 12288, 40000, 98304]


def make_jobs(rng, n, device_ok):
    jobs = []
    for case in range(n):
        k, p = CLASSES[int(rng.integers(0, len(CLASSES)))]
        cb = int(rng.choice(SIZES))
        op = ("encode", "recover", "update")[case % 3]
        device = device_ok and bool(rng.integers(0, 2))
        data = rng.integers(0, 256, (k, cb), dtype=np.uint8)
        par = ref.encode_data(ref.cauchy1(k, p)[k:], data)
        job = {"op": op, "k": k, "p": p, "C": cb, "device": device, "data": data, "par": par}
        if op == "recover":
            nerr = int(rng.integers(1, p + 1))
            job["err"] = sorted(int(x) for x in rng.choice(k + p, nerr, replace=False))
        if op == "update":
            job["vec_i"] = int(rng.integers(0, k))
            job["new"] = rng.integers(0, 256, cb, dtype=np.uint8)
        jobs.append(job)
    return jobs


def layout(rng, jobs):
    """Each job's [k+p][C] stripe image (+ the update's new cell) at a random
    byte offset of its own slot in one image."""
    slots = [(j["k"] + j["p"] + 1) * j["C"] + 64 for j in jobs]
    base = np.cumsum([0] + slots[:-1])
    img = np.zeros(int(sum(slots)), dtype=np.uint8)
    for j, b in zip(jobs, base):
        j["off"] = int(b) + int(rng.integers(0, 16))
        stripe = np.concatenate([j["data"], j["par"]])
        if j["op"] == "recover":
            stripe = stripe.copy()
            stripe[j["err"]] = 0xA5
        elif j["op"] == "encode":
            stripe = np.concatenate([j["data"], np.zeros_like(j["par"])])
        j["host"] = stripe.copy()
        img[j["off"]: j["off"] + stripe.size] = stripe.reshape(-1)
        if j["op"] == "update":
            n0 = j["off"] + stripe.size
            img[n0: n0 + j["C"]] = j["new"]
    return img


def submit(q, i, j, dev):
    k, p, cb = j["k"], j["p"], j["C"]
    if j["device"]:
        a = dev.ptr + j["off"]
        if j["op"] == "encode":
            q.encode_ptrs(i, k, p, cb, [a + c * cb for c in range(k)], [a + (k + r) * cb for r in range(p)])
        elif j["op"] == "recover":
            q.recover_ptr(i, k, p, cb, a, j["err"])
        else:
            q.update_ptrs(i, k, p, cb, j["vec_i"], a + j["vec_i"] * cb, a + (k + p) * cb,
                          [a + (k + r) * cb for r in range(p)])
        return
    h = j["host"]
    if j["op"] == "encode":
        q.encode(i, k, p, [h[c] for c in range(k)], [h[k + r] for r in range(p)])
    elif j["op"] == "recover":
        q.recover(i, k, p, h, j["err"])
    else:
        q.update(i, k, p, j["vec_i"], h[j["vec_i"]], j["new"], [h[k + r] for r in range(p)])


def check(jobs, got):
    bad = 0
    for j in jobs:
        k, p, cb = j["k"], j["p"], j["C"]
        out = got[j["off"]: j["off"] + (k + p) * cb].reshape(k + p, cb) if j["device"] else j["host"]
        if j["op"] == "update":
            d2 = j["data"].copy()
            d2[j["vec_i"]] = j["new"]
            want = ref.encode_data(ref.cauchy1(k, p)[k:], d2)
            bad += not np.array_equal(out[k:], want)
        else:
            bad += not (np.array_equal(out[:k], j["data"]) and np.array_equal(out[k:], j["par"]))
    return bad


def one_round(ctx, rng, nthreads, njobs, cpu_queue=False):
    jobs = make_jobs(rng, njobs, device_ok=not cpu_queue)
    img = layout(rng, jobs)
    dev = None if cpu_queue else ctx.to_device(img)
    q = ecg.Queue(None if cpu_queue else ctx, max_batch=int(rng.choice([4, 16, 64, 256])),
                  max_wait_us=int(rng.choice([20, 200, 2000])))
    try:
        def worker(t):
            for i in range(t, len(jobs), nthreads):
                submit(q, i, jobs[i], dev)

        th = [threading.Thread(target=worker, args=(t,)) for t in range(nthreads)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        q.flush()
        failed = sum(1 for rc in q.done.values() if rc != 0) + (len(jobs) - len(q.done))
        got = dev.download() if dev is not None else None
        bad = check(jobs, got)
        _, nbatch = q.stats()
        return len(jobs), bad, failed, nbatch
    finally:
        q.close()
        if dev is not None:
            dev.free()


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    nthreads = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    ctx = ecg.Context(0)
    rng = np.random.default_rng(0x50A4)
    old = ecg.dropin_crossover()
    for phase in ("device queue", "cpu executor"):
        t0 = time.time()
        tot = {"requests": 0, "mismatches": 0, "failed": 0, "batches": 0, "routes": {"cpu": 0, "staged": 0}}
        for r in range(rounds if phase == "device queue" else max(4, rounds // 4)):
            route = "cpu"
            if phase == "device queue":
                route = "cpu" if rng.integers(0, 2) else "staged"
                ecg.set_dropin_crossover((1 << 64) - 1 if route == "cpu" else 0)
            n, bad, failed, nb = one_round(ctx, rng, nthreads, int(rng.integers(48, 160)),
                                           cpu_queue=phase == "cpu executor")
            tot["requests"] += n
            tot["mismatches"] += bad
            tot["failed"] += failed
            tot["batches"] += nb
            tot["routes"][route] += 1
        ecg.set_dropin_crossover(old)
        tot.update({"phase": phase, "threads": nthreads, "seconds": round(time.time() - t0, 1)})
        print(json.dumps(tot), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
