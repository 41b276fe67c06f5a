"""Per-request delta parity updates on device cells (include/ecg.h
ecg_update_ptrs) and the batching queue's device-cell aggregation updates
(ecg_queue_update on HBM cells), against the oracle.

What the reference does per updated data cell of a stripe
(agg_update_parity, ref:src/object/srv_ec_aggregate.c:1062-1105):
xor_gen(old, new -> diff) then ec_encode_data_update(vec_i) into the stripe's
p parity cells.  XOR commutes, so any set of such requests applied in any
order gives one parity: the oracle applies them one by one
(oracle.encode_data_update = ISA-L ec_encode_data_update_base restated), and
the queue test also checks whole stripes against oracle.agg_update_parity.
"""
import ctypes as C
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def rand(shape, seed):
    return np.random.default_rng(seed).integers(0, 256, shape, dtype=np.uint8)


def _expected(oracle, k, p, parity0, reqs, olds, news):
    """parity0 [S][p][C]; reqs = [(stripe, vec_i)]; old/new cells per request."""
    en = oracle.cauchy1(k, p)[k:]
    want = parity0.copy()
    for i, (s, v) in enumerate(reqs):
        want[s] = oracle.encode_data_update(en, v, olds[i] ^ news[i], want[s])
    return want


@pytest.mark.parametrize("k,p,C_,align", [
    (2, 1, 65536, 16), (4, 2, 65536 + 4096 * 3, 16), (8, 2, 131072, 16), (8, 3, 4096 * 5 + 48, 16),
    (16, 2, 65536, 16), (4, 5, 32768, 16), (8, 8, 8192 + 16, 16),
    (8, 2, 12288 + 4, 4), (4, 2, 4096 * 3 + 8, 1), (8, 2, 4096 + 3, 1), (2, 1, 999, 1),
])
def test_update_ptrs_matches_oracle(ctx, oracle, ecglib, k, p, C_, align):
    """Random requests over S stripes, several per stripe (some stripes more
    than ECG_UPD_MU = 8, so a parity set spans ordered launches); cells at
    offsets of the given alignment; the byte kernel for C % 4 != 0."""
    S, nreq = 24, 96
    rng = np.random.default_rng(k * 1000 + p * 10 + C_ + align)
    stripe_of = np.concatenate([np.zeros(12, dtype=int), rng.integers(0, S, nreq - 12)])   # stripe 0: 12 updates
    vec = rng.integers(0, k, nreq)
    par0 = rand((S, p, C_), 7)
    olds = rand((nreq, C_), 8)
    news = rand((nreq, C_), 9)
    slot = (C_ + 64 + 15) & ~15
    off = 0 if align == 16 else (4 if align == 4 else 3)
    # one device image: parity cells [S][p], then old and new cells, each at slot*i + off
    npar = S * p
    img = np.zeros((npar + 2 * nreq) * slot + 64, dtype=np.uint8)

    def put(i, a):
        img[i * slot + off: i * slot + off + C_] = a

    for s in range(S):
        for r in range(p):
            put(s * p + r, par0[s, r])
    for i in range(nreq):
        put(npar + i, olds[i])
        put(npar + nreq + i, news[i])
    d = ctx.to_device(img)
    try:
        def addr(i):
            return d.ptr + i * slot + off
        reqs = [(int(vec[i]), addr(npar + i), addr(npar + nreq + i),
                 [addr(int(stripe_of[i]) * p + r) for r in range(p)]) for i in range(nreq)]
        before = ctx.stats()
        ctx.update_ptrs(k, p, C_, reqs)
        ctx.sync()
        kname = ecglib.last_kernel()
        after = ctx.stats()
        got = d.download()
        want = _expected(oracle, k, p, par0, list(zip(stripe_of, vec)), olds, news)
        for s in range(S):
            for r in range(p):
                i = s * p + r
                assert np.array_equal(got[i * slot + off: i * slot + off + C_], want[s, r]), (s, r, kname)
        assert after["update_cells"] - before["update_cells"] == nreq
        # 12 requests on stripe 0 -> 2 items of it -> at least 2 ordered launches
        assert after["launches"] - before["launches"] >= 2
        if C_ % 4:
            assert kname == "ecg_upd_ptr_byte_kernel", kname
        elif align == 16 and C_ % 16 == 0:
            assert kname.startswith("ecg_upd_ptr_kernel<") and kname.endswith(",g16>"), kname
        else:
            assert kname.endswith(",g4>"), kname
        # the untouched old/new cells are unchanged
        for i in range(nreq):
            assert np.array_equal(got[(npar + i) * slot + off:(npar + i) * slot + off + C_], olds[i])
    finally:
        d.free()


def test_update_ptrs_overlapping_parity_sets(ctx, oracle, ecglib):
    """Requests whose parity cells are different pointers into overlapping
    bytes (a cell at x and another at x + C/2): they may not run in one
    launch; the result equals applying the requests one by one to the shared
    buffer."""
    k, p, C_ = 4, 2, 16384
    half = C_ // 2
    nreq = 10
    rng = np.random.default_rng(77)
    buf0 = rand(10 * C_, 78)                      # the shared parity buffer
    olds = rand((nreq, C_), 79)
    news = rand((nreq, C_), 80)
    vec = rng.integers(0, k, nreq)
    # request i's parity cells: rows at (i * half) and (i * half + 3 C) -- request i and i+1 overlap by half a cell
    pofs = [(i * half, i * half + 3 * C_ + (half if i % 2 else 0)) for i in range(nreq)]
    assert all(b + C_ <= len(buf0) for _, b in pofs)
    img = np.concatenate([buf0, olds.reshape(-1), news.reshape(-1)])
    d = ctx.to_device(img)
    try:
        obase = d.ptr + len(buf0)
        nbase = obase + nreq * C_
        reqs = [(int(vec[i]), obase + i * C_, nbase + i * C_, [d.ptr + pofs[i][0], d.ptr + pofs[i][1]])
                for i in range(nreq)]
        ctx.update_ptrs(k, p, C_, reqs)
        ctx.sync()
        got = d.download(len(buf0))
        en = oracle.cauchy1(k, p)[k:]
        want = buf0.copy()
        for i in range(nreq):
            par = np.stack([want[pofs[i][r]: pofs[i][r] + C_] for r in range(p)])
            par = oracle.encode_data_update(en, int(vec[i]), olds[i] ^ news[i], par)
            for r in range(p):
                want[pofs[i][r]: pofs[i][r] + C_] = par[r]
        assert np.array_equal(got, want)
    finally:
        d.free()


def test_update_ptrs_errors(ctx, ecglib):
    """One request's own parity cells overlapping, vec_i >= k, k > 16, a
    NULL cell and an old / new cell overlapping any parity cell of the call
    are refused (-DER_INVAL) before any launch."""
    L = ecglib.lib()
    C_ = 4096
    d = ctx.alloc(8 * C_)
    try:
        def call(k, p, vec_i, cells):
            arr = (C.c_void_p * len(cells))(*cells)
            v = np.array([vec_i], dtype=np.uint8)
            return L.ecg_update_ptrs(ctx.h, k, p, C_, 1, arr, v.ctypes.data_as(ecglib.u8p), None)

        assert call(4, 2, 0, [d.ptr, d.ptr + C_, d.ptr + 2 * C_, d.ptr + 2 * C_ + 100]) == -ecglib.DER_INVAL
        assert "overlap" in L.ecg_strerror().decode()
        assert call(4, 2, 4, [d.ptr, d.ptr + C_, d.ptr + 2 * C_, d.ptr + 3 * C_]) == -ecglib.DER_INVAL
        assert call(17, 2, 0, [d.ptr, d.ptr + C_, d.ptr + 2 * C_, d.ptr + 3 * C_]) == -ecglib.DER_INVAL
        assert call(4, 2, 0, [d.ptr, None, d.ptr + 2 * C_, d.ptr + 3 * C_]) == -ecglib.DER_INVAL
        assert L.ecg_update_ptrs(ctx.h, 4, 2, C_, 0, None, None, None) == 0     # nothing to do
        # an old / new cell overlapping a parity cell of the call: its own, or another request's
        assert call(4, 2, 0, [d.ptr + 2 * C_ + 8, d.ptr + C_, d.ptr + 2 * C_, d.ptr + 4 * C_]) == -ecglib.DER_INVAL
        assert "old cell overlaps a parity cell" in L.ecg_strerror().decode()
        cells = [d.ptr, d.ptr + C_, d.ptr + 2 * C_, d.ptr + 3 * C_,
                 d.ptr + 4 * C_, d.ptr + 3 * C_ + C_ - 1, d.ptr + 6 * C_, d.ptr + 7 * C_]
        arr = (C.c_void_p * 8)(*cells)
        v = np.zeros(2, dtype=np.uint8)
        assert L.ecg_update_ptrs(ctx.h, 4, 2, C_, 2, arr, v.ctypes.data_as(ecglib.u8p), None) == -ecglib.DER_INVAL
        assert "request 1: the new cell overlaps" in L.ecg_strerror().decode()
        cells[5] = d.ptr + 4 * C_ + C_                  # adjacent, not overlapping
        arr = (C.c_void_p * 8)(*cells)
        assert L.ecg_update_ptrs(ctx.h, 4, 2, C_, 2, arr, v.ctypes.data_as(ecglib.u8p), None) == 0
        ctx.sync()
    finally:
        d.free()


def test_queue_device_updates_input_is_parity(ctx, oracle, ecglib):
    """A queued batch the direct call refuses (request 1 reads, as its old
    cell, the parity request 0 rewrites; request 3 names its own parity as
    its new cell): the queue runs the batch's requests one by one in order,
    each with its own result -- request 3 fails alone (-DER_INVAL), the
    others give what applying them one after another gives."""
    k, p, C_ = 4, 2, 8192
    img0 = rand(16 * C_, 31)
    d = ctx.to_device(img0)
    q = ecglib.Queue(ctx, max_batch=8, max_wait_us=200000)     # the 4 requests wait for one batch
    cell = lambda i: d.ptr + i * C_                             # noqa: E731
    reqs = [(1, 8, 9, [0, 1]),          # (vec_i, old, new, parity) as cell indices
            (2, 0, 10, [2, 3]),         # old = request 0's parity 0
            (0, 11, 12, [4, 5]),
            (3, 13, 6, [6, 7])]         # new = its own parity 0: refused
    try:
        for i, (v, o, n, par) in enumerate(reqs):
            q.update_ptrs(i, k, p, C_, v, cell(o), cell(n), [cell(r) for r in par])
        q.flush()
        assert q.done[3] == -ecglib.DER_INVAL and all(q.done[i] == 0 for i in range(3)), q.done
        got = d.download().reshape(16, C_)
        en = oracle.cauchy1(k, p)[k:]
        want = img0.reshape(16, C_).copy()
        for v, o, n, par in reqs[:3]:
            upd = oracle.encode_data_update(en, v, want[o] ^ want[n], np.stack([want[r] for r in par]))
            for j, r in enumerate(par):
                want[r] = upd[j]
        assert np.array_equal(got, want)
    finally:
        q.close()
        d.free()


def test_queue_device_updates_16_threads(ctx, oracle, ecglib):
    """16 threads post per-cell aggregation
    updates (agg_update_parity's xor_gen + ec_encode_data_update per updated
    cell, ref:src/object/srv_ec_aggregate.c:1086-1102) of overlapping stripes
    on DEVICE cells -- every stripe's updated cells posted by different
    threads, so one stripe's requests land in one batch, in different
    batches and in different ordered launches.  Final parity of every stripe
    equals oracle.agg_update_parity over its updated cells."""
    k, p, C_ = 8, 2, 65536
    S, T = 64, 16
    rng = np.random.default_rng(2606)
    par0 = rand((S, p, C_), 11)
    upd = []                                   # (stripe, cell)
    for s in range(S):
        ncell = int(rng.integers(1, 5))       # DAOS updates when fewer than half the cells changed
        for c in rng.choice(k, ncell, replace=False):
            upd.append((s, int(c)))
    rng.shuffle(upd)
    n = len(upd)
    olds = rand((n, C_), 12)
    news = rand((n, C_), 13)
    img = np.concatenate([par0.reshape(-1), olds.reshape(-1), news.reshape(-1)])
    d = ctx.to_device(img)
    q = ecglib.Queue(ctx, max_batch=64, max_wait_us=200)
    h2d0 = ctx.stats()["h2d_bytes"]
    try:
        obase = d.ptr + par0.nbytes
        nbase = obase + olds.nbytes

        def worker(t):
            for i in range(t, n, T):
                s, c = upd[i]
                q.update_ptrs(i, k, p, C_, c, obase + i * C_, nbase + i * C_,
                              [d.ptr + (s * p + r) * C_ for r in range(p)])

        th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        q.flush()
        nr, nb = q.stats()
        assert nr == n and len(q.done) == n and all(rc == 0 for rc in q.done.values()), q.done
        got = d.download(par0.nbytes).reshape(S, p, C_)
        for s in range(S):
            mine = sorted((c, i) for i, (ss, c) in enumerate(upd) if ss == s)
            bit_map = bytearray(2)
            for c, _ in mine:
                bit_map[c // 8] |= 1 << (c % 8)
            o = np.stack([olds[i] for _, i in mine])
            w = np.stack([news[i] for _, i in mine])
            want = oracle.agg_update_parity(k, p, C_, 1, bytes(bit_map), o, w, [(0, k * C_)], par0[s])
            assert np.array_equal(got[s], want), s
        # device cells in place: no request crossed PCIe
        assert ctx.stats()["h2d_bytes"] == h2d0
        assert 1 <= nb <= n
    finally:
        q.close()
        d.free()


def test_queue_device_updates_same_cell_chain(ctx, oracle, ecglib):
    """The same data cell of one stripe updated again and again (old -> v1 ->
    v2 -> ... -> new) from several threads at once: the deltas telescope, so
    the final parity is the encode of the final data."""
    k, p, C_ = 4, 2, 32768
    steps = 24
    vals = rand((steps + 1, C_), 21)           # successive contents of data cell 2
    data = rand((k, C_), 22)
    data[2] = vals[0]
    en = oracle.cauchy1(k, p)
    par0 = oracle.encode_data(en[k:], data)
    img = np.concatenate([par0.reshape(-1), vals.reshape(-1)])
    d = ctx.to_device(img)
    q = ecglib.Queue(ctx, max_batch=8, max_wait_us=100)
    try:
        vbase = d.ptr + par0.nbytes

        def worker(t):
            for i in range(t, steps, 4):
                q.update_ptrs(i, k, p, C_, 2, vbase + i * C_, vbase + (i + 1) * C_,
                              [d.ptr + r * C_ for r in range(p)])

        th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        q.flush()
        assert all(rc == 0 for rc in q.done.values()) and len(q.done) == steps
        data[2] = vals[steps]
        got = d.download(par0.nbytes).reshape(p, C_)
        assert np.array_equal(got, oracle.encode_data(en[k:], data))
    finally:
        q.close()
        d.free()


@pytest.mark.parametrize("seed", range(6))
def test_update_ptrs_random_overlaps(ctx, oracle, ecglib, seed):
    """Seeded random batches whose parity cells land at random offsets of one
    small buffer -- identical sets, partial overlaps and disjoint cells mixed,
    so the fold, the ordered launches and the greedy colouring all run --
    against the oracle applying the requests one by one."""
    rng = np.random.default_rng(4242 + seed)
    k = int(rng.choice([2, 4, 8, 16]))
    p = int(rng.integers(1, 4))
    C_ = int(rng.choice([4096, 8192 + 16, 12288 + 4, 3000]))
    span = C_ * int(rng.integers(3 * p, 6 * p))          # small: overlaps are common
    nreq = int(rng.integers(5, 60))
    base_sets = []                                        # a few parity sets reused verbatim
    for _ in range(int(rng.integers(1, 5))):
        base_sets.append(sorted(int(x) for x in rng.choice(span // C_ - 1, p, replace=False) * C_))
    reqs_off = []
    for _ in range(nreq):
        if rng.random() < 0.5:
            offs = list(base_sets[int(rng.integers(0, len(base_sets)))])
        else:                                             # rows at random byte offsets, disjoint among themselves
            while True:
                offs = sorted(int(x) for x in rng.integers(0, span - C_, p))
                if all(offs[i + 1] - offs[i] >= C_ for i in range(p - 1)):
                    break
            if C_ % 4 == 0 and rng.random() < 0.7:
                offs = [o & ~3 for o in offs]
                if not all(offs[i + 1] - offs[i] >= C_ for i in range(p - 1)):
                    offs = list(base_sets[0])
        reqs_off.append(offs)
    vec = rng.integers(0, k, nreq)
    buf0 = rand(span, 5000 + seed)
    olds = rand((nreq, C_), 5100 + seed)
    news = rand((nreq, C_), 5200 + seed)
    img = np.concatenate([buf0, olds.reshape(-1), news.reshape(-1)])
    d = ctx.to_device(img)
    try:
        ob, nb = d.ptr + span, d.ptr + span + nreq * C_
        ctx.update_ptrs(k, p, C_, [(int(vec[i]), ob + i * C_, nb + i * C_, [d.ptr + o for o in reqs_off[i]])
                                   for i in range(nreq)])
        ctx.sync()
        got = d.download(span)
        en = oracle.cauchy1(k, p)[k:]
        want = buf0.copy()
        for i in range(nreq):
            par = np.stack([want[o:o + C_] for o in reqs_off[i]])
            par = oracle.encode_data_update(en, int(vec[i]), olds[i] ^ news[i], par)
            for r, o in enumerate(reqs_off[i]):
                want[o:o + C_] = par[r]
        assert np.array_equal(got, want), (k, p, C_, nreq, ecglib.last_kernel())
    finally:
        d.free()


def test_queue_device_updates_multi_context_same_device(ctx, oracle, ecglib):
    """A queue over an ecg_multi_t that lists one device twice: its slots
    alternate between two contexts of the same GPU, so update batches of one
    stripe land on both.  They must still run one after another (one update
    stream per DEVICE, not per context) -- 8 threads updating the same 6
    stripes over and over, every stripe's final parity the oracle's."""
    k, p, C_ = 4, 2, 65536
    S, per_stripe, T = 6, 24, 8
    m = ecglib.Multi([0, 0])
    rng = np.random.default_rng(77)
    par0 = rand((S, p, C_), 31)
    n = S * per_stripe
    upd = [(i % S, int(rng.integers(0, k))) for i in range(n)]
    olds = rand((n, C_), 32)
    news = rand((n, C_), 33)
    img = np.concatenate([par0.reshape(-1), olds.reshape(-1), news.reshape(-1)])
    d = m.ctxs[0].to_device(img)
    q = ecglib.Queue(m, max_batch=16, max_wait_us=50)
    try:
        ob = d.ptr + par0.nbytes
        nb = ob + olds.nbytes

        def worker(t):
            for i in range(t, n, T):
                s, c = upd[i]
                q.update_ptrs(i, k, p, C_, c, ob + i * C_, nb + i * C_, [d.ptr + (s * p + r) * C_ for r in range(p)])

        th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        q.flush()
        assert len(q.done) == n and all(rc == 0 for rc in q.done.values())
        got = d.download(par0.nbytes).reshape(S, p, C_)
        en = oracle.cauchy1(k, p)[k:]
        for s in range(S):
            want = par0[s]
            for i, (ss, c) in enumerate(upd):
                if ss == s:
                    want = oracle.encode_data_update(en, c, olds[i] ^ news[i], want)
            assert np.array_equal(got[s], want), s
    finally:
        q.close()
        d.free()
        m.close()


def test_update_ptrs_large_overlapping_batch(ctx, oracle, ecglib):
    """1500 requests whose parity cells sit at random byte offsets of a
    buffer 40 cells long: nearly every item meets several others, so the
    launches come from the conflict-graph colouring (one sweep over the
    sorted parity intervals) -- every parity byte's read-modify-writes in
    separate launches, the result the requests applied one by one."""
    rng = np.random.default_rng(1500)
    k, p, C_, nreq = 8, 2, 512, 1500
    span = C_ * 40
    offs = []
    for _ in range(nreq):
        while True:
            o = sorted(int(x) for x in rng.integers(0, span - C_, p))
            if o[1] - o[0] >= C_:
                break
        offs.append(o)
    vec = rng.integers(0, k, nreq)
    buf0 = rand(span, 77)
    olds = rand((nreq, C_), 78)
    news = rand((nreq, C_), 79)
    d = ctx.to_device(np.concatenate([buf0, olds.reshape(-1), news.reshape(-1)]))
    try:
        ob, nb = d.ptr + span, d.ptr + span + nreq * C_
        before = ctx.stats()["launches"]
        ctx.update_ptrs(k, p, C_, [(int(vec[i]), ob + i * C_, nb + i * C_, [d.ptr + o for o in offs[i]])
                                   for i in range(nreq)])
        ctx.sync()
        launches = ctx.stats()["launches"] - before
        got = d.download(span)
        en = oracle.cauchy1(k, p)[k:]
        want = buf0.copy()
        for i in range(nreq):
            par = oracle.encode_data_update(en, int(vec[i]), olds[i] ^ news[i],
                                            np.stack([want[o:o + C_] for o in offs[i]]))
            for r, o in enumerate(offs[i]):
                want[o:o + C_] = par[r]
        assert np.array_equal(got, want)
        assert 2 <= launches < nreq, launches
    finally:
        d.free()
