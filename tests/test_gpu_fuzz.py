"""Seeded random layouts through ecg_matmul, byte for byte against the oracle.

The product picks its kernel per launch from the operands (ecg_kernels.hip
ecg_k_launch_matmul: dwordx4 / dword / funnel-shift lanes, outputs at any
byte stored as misaligned dwords, the partial last 4 KiB column of a cell
dword by dword; k > 16 split into accumulating launches).  The fixed cases in
test_gpu_align.py pin each choice; these cases draw the layout at random --
base offsets, cell pitches, stripe strides, cell order, in-place recovery-style
layouts where sources and outputs share one buffer, accumulate or overwrite --
so combinations nobody wrote down still meet the oracle (the reference's
ec_encode_data takes arbitrary pointers per cell, ref:src/object/cli_ec.c:540,
2641).  Bytes outside the output cells must be untouched, and the kernel that
ran must be the one `predict` (a restatement of the launch rules) names.
"""
import numpy as np
import pytest

N_CASES = 96
CELLS = [1, 3, 4, 17, 255, 1000, 1024, 4095, 4096, 4097, 6000, 8192, 12288 + 20, 20000 + 3]
CELLS16 = [16, 1024, 4096, 8192, 12288 + 16]


def gran(bits):
    return 16 if bits % 16 == 0 else 8 if bits % 8 == 0 else 4 if bits % 4 == 0 else 1


def predict(sbase, soff, sstride, dbase, doff, dstride, acc=False):
    """The lanes one launch runs (ecg_mm_dev.h align_granule, and
    ecg_k_launch_matmul's g2 for k = 8 with rows 1-3 and no accumulate whose
    sources are off a 16-byte boundary); bases are byte offsets from a
    256-byte-aligned allocation, soff / doff the launch's cells.
    Destinations at any byte take the lanes' stores as misaligned dwords."""
    sb = sbase | sstride
    for o in soff:
        sb |= o
    db = dbase | dstride
    for o in doff:
        db |= o
    gs, gd = gran(sb), gran(db)
    if gs < 16 and len(soff) == 8 and 1 <= len(doff) <= 3 and not acc:
        return "g2"
    return "g1" if gs < 4 else "g16" if gs == gd == 16 else "g4"


def draw(rng, mode):
    """mode 0: everything 16-byte aligned; 1: dword-aligned; 2: outputs all
    equally off a dword boundary; 3: sources at any byte; 4: anything."""
    k = int(rng.choice([1, 2, 3, 4, 5, 8, 12, 16, 17, 24]))
    rows = int(rng.integers(1, 7))
    S = int(rng.integers(1, 5))
    inplace = bool(rng.integers(0, 2)) and mode != 3
    acc = bool(rng.integers(0, 2))
    unit = 16 if mode == 0 else 4 if mode in (1, 2, 3) else int(rng.choice([1, 4, 16]))
    C = int(rng.choice(CELLS16 if mode == 0 else CELLS))
    if mode in (1, 2) and C % 4:
        C += 4 - C % 4                      # the output stripe stride of the separate layout is C
    pitch = -(-(C + unit * int(rng.integers(0, 3))) // unit) * unit if unit > 1 else C + int(rng.integers(0, 5))
    pad = unit * int(rng.integers(0, 5))
    if mode == 4:
        sbase, dbase = int(rng.integers(0, 20)), int(rng.integers(0, 20))
    else:
        sbase, dbase = unit * int(rng.integers(0, 3)), unit * int(rng.integers(0, 3))
        if mode == 2:
            dbase += int(rng.integers(1, 4))
            sbase = dbase if inplace else sbase
        if mode == 3:
            sbase += int(rng.integers(1, 4))
    return k, rows, C, S, inplace, acc, pitch, pad, sbase, dbase


def run_case(ctx, oracle, ecglib, seed):
    rng = np.random.default_rng(1000 + seed)
    k, rows, C, S, inplace, acc, pitch, pad, sbase, dbase = draw(rng, seed % 5)
    coef = rng.integers(0, 256, (rows, k), dtype=np.uint8)
    if inplace:
        # one [S][k + rows][pitch] image: a random choice of cells are the sources,
        # the rest the outputs (a degraded read's survivors and erased cells)
        order = rng.permutation(k + rows)
        stride = (k + rows) * pitch + pad
        src_off = [int(c) * pitch for c in order[:k]]
        dst_off = [int(c) * pitch for c in order[k:]]
        img = rng.integers(0, 256, sbase + S * stride + 64, dtype=np.uint8)
        bufs = (ctx.to_device(img),)
        src_stride = dst_stride = stride
        dbase = sbase
        before = img
    else:
        # separate source [S][k][pitch] and output rows [rows][S][C] (+ row padding), cells in random order
        src_stride = k * pitch + pad
        img = rng.integers(0, 256, sbase + S * src_stride + 64, dtype=np.uint8)
        src_off = [int(c) * pitch for c in rng.permutation(k)]
        drow = S * C + pad
        dst_off = [int(r) * drow for r in rng.permutation(rows)]
        dst_stride = C
        before = rng.integers(0, 256, dbase + rows * drow + 64, dtype=np.uint8)
        bufs = (ctx.to_device(img), ctx.to_device(before))
    last = src_off[(k - 1) // 16 * 16:]           # k > 16: the last launch takes the last <= 16 cells
    want = predict(sbase, last, src_stride, dbase, dst_off, dst_stride, acc or k > 16)
    try:
        ctx.matmul(coef, C, S, bufs[0].ptr + sbase, src_off, src_stride, bufs[-1].ptr + dbase, dst_off,
                   dst_stride, 1 if acc else 0)
        ctx.sync()
        kern = ecglib.last_kernel()
        after = bufs[-1].download()
    finally:
        for b in bufs:
            b.free()
    expect = before.copy()
    for s in range(S):
        cells = np.stack([img[sbase + s * src_stride + o: sbase + s * src_stride + o + C] for o in src_off])
        prod = oracle.encode_data(coef, cells)
        for r, o in enumerate(dst_off):
            at = dbase + s * dst_stride + o
            expect[at: at + C] = (expect[at: at + C] ^ prod[r]) if acc else prod[r]
    what = (f"seed {seed}: k={k} rows={rows} C={C} S={S} inplace={inplace} acc={acc} pitch={pitch} pad={pad} "
            f"bases={sbase},{dbase} kernel={kern} predicted={want}")
    bad = np.flatnonzero(after != expect)
    assert bad.size == 0, f"{what}: {bad.size} bytes differ, first at {bad[0]}"
    got = kern.rsplit(",", 1)[-1].rstrip(">") if ",g" in kern else "g16"
    assert got == want, what
    return got


def test_predict_covers_every_class():
    """The draw reaches every lane-access class (host-only check of the draw)."""
    seen = {}
    for seed in range(N_CASES):
        rng = np.random.default_rng(1000 + seed)
        k, rows, C, S, inplace, acc, pitch, pad, sbase, dbase = draw(rng, seed % 5)
        rng.integers(0, 256, (rows, k), dtype=np.uint8)
        if inplace:
            order = rng.permutation(k + rows)
            stride = (k + rows) * pitch + pad
            cls = predict(sbase, [int(c) * pitch for c in order[:k]][(k - 1) // 16 * 16:], stride, sbase,
                          [int(c) * pitch for c in order[k:]], stride, acc or k > 16)
        else:
            rng.integers(0, 256, sbase + S * (k * pitch + pad) + 64, dtype=np.uint8)
            soff = [int(c) * pitch for c in rng.permutation(k)]
            cls = predict(sbase, soff[(k - 1) // 16 * 16:], k * pitch + pad, dbase,
                          [int(r) * (S * C + pad) for r in rng.permutation(rows)], C, acc or k > 16)
        seen[cls] = seen.get(cls, 0) + 1
    assert {"g1", "g2", "g4", "g16"} <= set(seen), seen
    # and outputs off a dword boundary (the byte kernel's case before round 4)
    assert sum(1 for s in range(N_CASES) if s % 5 == 2) >= 10
    assert predict(0, [0], 4096, 1, [0, 8193], 4096) == "g4"
    assert predict(3, [0], 4096, 1, [0], 4096) == "g1"


@pytest.mark.gpu
def test_random_layouts(ctx, oracle, ecglib):
    kernels = {}
    for seed in range(N_CASES):
        got = run_case(ctx, oracle, ecglib, seed)
        kernels[got] = kernels.get(got, 0) + 1
    print("kernels:", kernels)
    assert {"g1", "g2", "g4", "g16"} <= set(kernels), kernels


def table_affine(offs, S, k, rows):
    """ecg_ptrs.c table_affine: every cell at a fixed offset from a per-stripe
    base (one stride for the inputs, one for the outputs)."""
    n = k + rows
    if S == 1:
        return True
    bs, bd = offs[n] - offs[0], offs[n + k] - offs[k]
    return all(offs[s * n + j] == offs[j] + s * (bs if j < k else bd) for s in range(S) for j in range(n))


def ptr_predict(ins, outs, C, k=0, rows=0):
    """ecg_ptrs.c ptr_granule + ecg_k_launch_matmul_ptrs (addresses as offsets
    from a 256-byte-aligned allocation)."""
    ib = 0
    for a in ins:
        ib |= a
    ob = 0
    for a in outs:
        ob |= a
    if ib & 15 and k == 8 and 1 <= rows <= 3:
        return "g2"
    if ib & 3:
        return "g1"
    return "g16" if ((ib | ob) & 15) == 0 and C % 16 == 0 else "g4"


@pytest.mark.gpu
def test_random_pointer_tables(ctx, oracle, ecglib):
    """The pointer-table product (ISA-L's data[] / coding[] per stripe,
    ref:src/object/cli_ec.c:476-546) over seeded random cells: every cell in
    its own slot of one buffer at a drawn skew (all 0, all dword multiples, or
    any byte, for inputs and outputs separately), slots shuffled, random
    k <= 16, rows <= 6, cell sizes and stripe counts."""
    seen = {}
    for seed in range(48):
        rng = np.random.default_rng(5000 + seed)
        k, rows = int(rng.integers(1, 17)), int(rng.integers(1, 7))
        C = int(rng.choice(CELLS16 if seed % 4 == 0 else CELLS))
        S = int(rng.integers(1, 5))
        n = S * (k + rows)
        slot = (C + 15) // 16 * 16 + 32
        unit_in, unit_out = (16, 16) if seed % 4 == 0 else (int(rng.choice([16, 4, 1])), int(rng.choice([16, 4, 1])))
        order = rng.permutation(n + 3)[:n]
        skews = [int(rng.integers(0, 16 // u)) * u if u > 1 else int(rng.integers(0, 16))
                 for u in [unit_in if i % (k + rows) < k else unit_out for i in range(n)]]
        host = rng.integers(0, 256, (n + 3) * slot, dtype=np.uint8)
        coef = rng.integers(0, 256, (rows, k), dtype=np.uint8)
        offs = [int(o) * slot + sk for o, sk in zip(order, skews)]
        want = ptr_predict([o for i, o in enumerate(offs) if i % (k + rows) < k],
                           [o for i, o in enumerate(offs) if i % (k + rows) >= k], C, k, rows)
        buf = ctx.to_device(host)
        try:
            ctx.matmul_ptrs(k, rows, coef, C, S, [buf.ptr + o for o in offs])
            ctx.sync()
            kern = ecglib.last_kernel()
            dev = buf.download()
        finally:
            buf.free()
        expect = host.copy()
        for s in range(S):
            base = s * (k + rows)
            cells = np.stack([host[offs[base + j]: offs[base + j] + C] for j in range(k)])
            prod = oracle.encode_data(coef, cells)
            for r in range(rows):
                o = offs[base + k + r]
                expect[o: o + C] = prod[r]
        affine = table_affine(offs, S, k, rows)
        what = (f"seed {seed}: k={k} rows={rows} C={C} S={S} units={unit_in},{unit_out} affine={affine} "
                f"kernel={kern} want={want}")
        bad = np.flatnonzero(dev != expect)
        assert bad.size == 0, f"{what}: {bad.size} bytes differ, first at {bad[0]}"
        got = kern.rsplit(",", 1)[-1].rstrip(">") if ",g" in kern else "g16"
        if affine:      # the offset kernel, its lanes by its own rule
            n = k + rows
            bs, bd = (offs[n] - offs[0], offs[n + k] - offs[k]) if S > 1 else (0, 0)
            want = predict(offs[0], [offs[j] - offs[0] for j in range(k)], bs, offs[k],
                           [offs[k + r] - offs[k] for r in range(rows)], bd)
            what += f" -> offset kernel {want}"
            assert kern.startswith("ecg_mm_kernel<"), what
        else:
            assert kern.startswith("ecg_mm_ptr_kernel<"), what
        assert got == want, what
        seen[got] = seen.get(got, 0) + 1
    print("kernels:", seen)
    assert {"g1", "g4", "g16"} <= set(seen), seen


@pytest.mark.gpu
def test_random_dropin_calls(ctx, oracle, ecglib):
    """Seeded random ISA-L-convention calls through the drop-in's router
    (ecg_dropin.c): ec_encode_data / ec_encode_data_update / xor_gen with k up
    to 70 sources and up to 10 output rows, lengths from 1 byte to 70 KiB,
    cells at random byte offsets -- on host cells at a random crossover (so the
    CPU path and the GPU staging both run) and on device cells (the HIP
    kernels in place).  Every output equals the oracle's; the route taken is
    the one the placement and the crossover name."""
    import ctypes as C

    L = ecglib.lib()
    rng = np.random.default_rng(0xD80)
    old = ecglib.dropin_crossover()
    routes = set()
    try:
        for case in range(96):
            op = ("encode", "update", "xor")[case % 3]
            k = int(rng.choice([1, 2, 3, 4, 8, 16, 17, 33, 64, 70])) if op != "update" else 1
            if op == "encode":
                k = min(k, 64)
            rows = 1 if op == "xor" else int(rng.integers(1, 11))
            n = int(rng.choice([1, 15, 64, 100, 4096, 4097, 33333, 70000]))
            device = bool(rng.integers(0, 2))
            cross = [0, n * (k + rows), (1 << 64) - 1][int(rng.integers(0, 3))]
            ecglib.set_dropin_crossover(cross)
            coef = rng.integers(0, 256, (rows, k), dtype=np.uint8) if op != "xor" else np.ones((1, k), np.uint8)
            src = rng.integers(0, 256, (k, n), dtype=np.uint8)
            dst0 = rng.integers(0, 256, (rows, n), dtype=np.uint8)
            want = oracle.encode_data(coef, src)
            if op == "update":
                want = want ^ dst0
            soff = [int(rng.integers(0, 16)) + j * (n + 32) for j in range(k)]
            doff = [int(rng.integers(0, 16)) + r * (n + 32) for r in range(rows)]
            if device:
                sb, db = ctx.alloc(k * (n + 32)), ctx.alloc(rows * (n + 32))
                for j in range(k):
                    sb.upload(src[j], offset=soff[j])
                for r in range(rows):
                    db.upload(dst0[r], offset=doff[r])
                sp = [sb.ptr + o for o in soff]
                dp = [db.ptr + o for o in doff]
            else:
                hs = np.zeros(k * (n + 32), np.uint8)
                hd = np.zeros(rows * (n + 32), np.uint8)
                for j in range(k):
                    hs[soff[j]: soff[j] + n] = src[j]
                for r in range(rows):
                    hd[doff[r]: doff[r] + n] = dst0[r]
                sp = [hs.ctypes.data + o for o in soff]
                dp = [hd.ctypes.data + o for o in doff]
            if op == "xor":
                v = (C.c_void_p * (k + 1))(*(sp + dp))
                assert L.xor_gen(k + 1, n, v) == (0 if k >= 2 else 1)
                if k < 2:
                    want = dst0
            else:
                tb = ecglib.isal_init_tables(coef)
                spp = (ecglib.u8p * k)(*[C.cast(C.c_void_p(x), ecglib.u8p) for x in sp])
                dpp = (ecglib.u8p * rows)(*[C.cast(C.c_void_p(x), ecglib.u8p) for x in dp])
                if op == "encode":
                    L.ec_encode_data(n, k, rows, tb.ctypes.data_as(ecglib.u8p), spp, dpp)
                else:
                    L.ec_encode_data_update(n, k, rows, 0, tb.ctypes.data_as(ecglib.u8p), spp[0], dpp)
            if op != "xor" or k >= 2:
                kern = ecglib.last_kernel()
                gpu = device or n * (k + rows) >= cross
                assert kern.startswith("ecg_mm") if gpu else kern.startswith("cpu:"), (case, op, device, cross, kern)
                routes.add((device, gpu))
            if device:
                raw = db.download()
                got = np.stack([raw[o: o + n] for o in doff])
                sb.free()
                db.free()
            else:
                got = np.stack([hd[o: o + n] for o in doff])
            assert np.array_equal(got, want), (case, op, k, rows, n, device, cross)
    finally:
        ecglib.set_dropin_crossover(old)
    assert routes >= {(True, True), (False, True), (False, False)}, routes


@pytest.mark.gpu
def test_random_queue_requests(ctx, oracle, ecglib, route):
    """Seeded random one-stripe requests posted to one ecg_queue from 6
    threads at once: encodes and recoveries on host or device cells (device
    stripes at random byte offsets in one shared allocation, so the queue's
    device slots batch them into pointer-table launches) and host-cell delta
    updates, EC classes 2+1 .. 16+3, cell sizes 1 byte .. 40 KiB.  After one
    flush every request's callback reported 0 and every output equals the
    oracle's."""
    import threading

    rng = np.random.default_rng(0xB47)
    classes = [(2, 1), (4, 2), (8, 2), (8, 3), (16, 2), (16, 3)]
    sizes = [1, 31, 4096, 4100, 12288, 40000]
    jobs = []
    for case in range(144):
        k, p = classes[int(rng.integers(0, len(classes)))]
        Cb = int(rng.choice(sizes))
        op = ("encode", "recover", "update")[case % 3]
        device = op != "update" and bool(rng.integers(0, 2))
        data = rng.integers(0, 256, (k, Cb), dtype=np.uint8)
        par = oracle.encode_data(oracle.cauchy1(k, p)[k:], data)
        job = {"op": op, "k": k, "p": p, "C": Cb, "device": device, "data": data, "par": par}
        if op == "recover":
            nerr = int(rng.integers(1, p + 1))
            job["err"] = sorted(int(x) for x in rng.choice(k + p, nerr, replace=False))
        if op == "update":
            job["vec_i"] = int(rng.integers(0, k))
            job["new"] = rng.integers(0, 256, Cb, dtype=np.uint8)
        jobs.append(job)
    # device stripes: each [k+p][C] image at a random byte offset of its own slot in one allocation
    slots = [(k + p) * Cb + 64 for j in jobs for k, p, Cb in [(j["k"], j["p"], j["C"])]]
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
        j["host"] = stripe.copy()            # host-cell requests work on their own arrays
        img[j["off"]: j["off"] + stripe.size] = stripe.reshape(-1)
    dev = ctx.to_device(img)
    q = ecglib.Queue(ctx, max_batch=32, max_wait_us=200)
    try:
        def worker(t):
            for i in range(t, len(jobs), 6):
                j = jobs[i]
                k, p, Cb = j["k"], j["p"], j["C"]
                if j["op"] == "update":
                    h = j["host"]
                    q.update(i, k, p, j["vec_i"], h[j["vec_i"]], j["new"], [h[k + r] for r in range(p)])
                elif j["device"]:
                    a = dev.ptr + j["off"]
                    if j["op"] == "encode":
                        q.encode_ptrs(i, k, p, Cb, [a + c * Cb for c in range(k)],
                                      [a + (k + r) * Cb for r in range(p)])
                    else:
                        q.recover_ptr(i, k, p, Cb, a, j["err"])
                elif j["op"] == "encode":
                    h = j["host"]
                    q.encode(i, k, p, [h[c] for c in range(k)], [h[k + r] for r in range(p)])
                else:
                    q.recover(i, k, p, j["host"], j["err"])

        th = [threading.Thread(target=worker, args=(t,)) for t in range(6)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        q.flush()
        assert len(q.done) == len(jobs) and all(rc == 0 for rc in q.done.values()), q.done
        got = dev.download()
        for i, j in enumerate(jobs):
            k, p, Cb = j["k"], j["p"], j["C"]
            if j["op"] == "update":
                d2 = j["data"].copy()
                d2[j["vec_i"]] = j["new"]
                want = oracle.encode_data(oracle.cauchy1(k, p)[k:], d2)
                assert np.array_equal(j["host"][k:], want), (i, j["op"])
                continue
            out = got[j["off"]: j["off"] + (k + p) * Cb].reshape(k + p, Cb) if j["device"] else j["host"]
            assert np.array_equal(out[:k], j["data"]), (i, j["op"], j["device"])
            assert np.array_equal(out[k:], j["par"]), (i, j["op"], j["device"], k, p, Cb)
        nreq, nbatch = q.stats()
        assert nreq == len(jobs) and nbatch <= nreq
    finally:
        q.close()
        dev.free()
