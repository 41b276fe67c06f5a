"""GPU parity of the pointer-table product (ecg_matmul_ptrs) and of the
client's scatter-gather encode (ecg_obj_ec_recx_encode, restating
obj_ec_recx_encode / obj_ec_stripe_encode, ref:src/object/cli_ec.c:476-546,
593-663) against the CPU oracle.  Bit-exact."""
import ctypes as ct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ptr_granule(in_skews, out_skews, C, k=0, rows=0):
    """ecg_ptrs.c ptr_granule + ecg_k_launch_matmul_ptrs: 1 funnel-shifted
    inputs, 4 dword lanes, 16 dwordx4 lanes, 2 (k = 8, rows 1-3, an input off
    16 bytes) funnel-shifted 16-byte lanes (outputs at any byte: misaligned
    stores)."""
    ib = 0
    for x in in_skews:
        ib |= x
    ob = 0
    for x in out_skews:
        ob |= x
    if ib & 15 and k == 8 and 1 <= rows <= 3:
        return 2
    if ib & 3:
        return 1
    return 16 if ((ib | ob) & 15) == 0 and C % 16 == 0 else 4


@pytest.mark.parametrize("k,rows,C,S,iskew,oskew", [
    (8, 2, 65536, 12, 0, 0), (4, 3, 4096 * 3 + 48, 7, 0, 0), (16, 2, 8192, 5, 0, 0),
    (6, 5, 1000, 9, 3, 3),                      # outputs off a dword: misaligned dword stores
    (2, 1, 4097, 4, 3, 3),
    (8, 2, 65536 + 4096 + 20, 6, 0, 0),         # cell size not a multiple of 16: dword lanes
    (8, 2, 65536, 6, 8, 4),                     # 8- / 4-byte aligned cells: dword lanes
    (8, 2, 65536 + 1000, 6, "rand", 0),         # inputs at random byte offsets: funnel-shifted dwords
    (16, 3, 12288 + 5, 4, "rand", 8),
    (4, 2, 4096, 9, 1, 0), (5, 3, 5000, 4, "rand", 4),
])
def test_matmul_ptrs(oracle, ecglib, ctx, k, rows, C, S, iskew, oskew):
    """Cells scattered at random (disjoint, shuffled) offsets of one buffer,
    inputs and outputs at the given byte skews within their slots ("rand":
    each input cell at its own random skew, as in-place sgl cells are)."""
    rng = np.random.default_rng(k * 100 + rows + C)
    slot = (C + 15) // 16 * 16 + 32
    nslots = S * (k + rows) + 8
    buf = ctx.alloc(nslots * slot)
    order = rng.permutation(nslots)[: S * (k + rows)]
    host = rng.integers(0, 256, nslots * slot, dtype=np.uint8)
    skews = []
    for s in range(S):
        for j in range(k + rows):
            if j < k:
                skews.append(int(rng.integers(0, 16)) if iskew == "rand" else iskew)
            else:
                skews.append(oskew)
    try:
        buf.upload(host)
        addrs = [buf.ptr + int(o) * slot + sk for o, sk in zip(order, skews)]
        coef = rng.integers(0, 256, (rows, k), dtype=np.uint8)
        ctx.matmul_ptrs(k, rows, coef, C, S, addrs)
        ctx.sync()
        kern = ecglib.last_kernel()
        g = _ptr_granule([a for i, a in enumerate(addrs) if i % (k + rows) < k],
                         [a for i, a in enumerate(addrs) if i % (k + rows) >= k], C, k, rows)
        if g == 16:
            assert kern.startswith("ecg_mm_ptr_kernel<") and ",g" not in kern, kern
        else:
            assert kern.startswith("ecg_mm_ptr_kernel<") and kern.endswith(f",g{g}>"), kern
        dev = buf.download()
        for s in range(S):
            cells = np.stack([host[int(order[s * (k + rows) + j]) * slot + skews[s * (k + rows) + j]:][:C]
                              for j in range(k)])
            want = oracle.encode_data(coef, cells)
            for r in range(rows):
                i = s * (k + rows) + k + r
                o = int(order[i]) * slot + skews[i]
                assert np.array_equal(dev[o:o + C], want[r]), (s, r)
            # bytes around the outputs untouched
            for r in range(rows):
                i = s * (k + rows) + k + r
                o = int(order[i]) * slot
                assert np.array_equal(dev[o:o + skews[i]], host[o:o + skews[i]])
                assert np.array_equal(dev[o + skews[i] + C:o + slot], host[o + skews[i] + C:o + slot])
    finally:
        buf.free()


@pytest.mark.parametrize("rows", [1, 2, 3])
def test_matmul_ptrs_g2_generic_variant(oracle, ecglib, ctx, rows):
    """k = 8 with a source off a 16-byte boundary picks the g2
    lanes, which exist only as k = 8 shapes; with ecg_set_launch variant 1 (the
    runtime-shaped kernels) no g2 entry matches, and the launch must fall back
    to the funnel-shifted dword lanes (g1, runtime-shaped) instead of failing
    with hipErrorInvalidDeviceFunction."""
    k, C, S = 8, 65536 + 64, 5
    rng = np.random.default_rng(880 + rows)
    slot = C + 64
    buf = ctx.alloc(S * (k + rows) * slot + 64)
    host = rng.integers(0, 256, S * (k + rows) * slot + 64, dtype=np.uint8)
    # shuffled slots: not an affine table, so the pointer-table kernel runs
    order = rng.permutation(S * (k + rows))
    offs = [int(order[s * (k + rows) + j]) * slot + (1 if j == 0 else 0)
            for s in range(S) for j in range(k + rows)]        # source 0 of every stripe at +1
    addrs = [buf.ptr + o for o in offs]
    coef = rng.integers(0, 256, (rows, k), dtype=np.uint8)
    try:
        buf.upload(host)
        ctx.set_launch(0, 0, 1)
        try:
            ctx.matmul_ptrs(k, rows, coef, C, S, addrs)
            ctx.sync()
        finally:
            ctx.set_launch(0, 0, 0)
        kern = ecglib.last_kernel()
        assert kern == "ecg_mm_ptr_kernel<0,0,g1>", kern
        dev = buf.download()
        for s in range(S):
            cells = np.stack([host[offs[s * (k + rows) + j]:][:C] for j in range(k)])
            want = oracle.encode_data(coef, cells)
            for r in range(rows):
                o = offs[s * (k + rows) + k + r]
                assert np.array_equal(dev[o:o + C], want[r]), (s, r)
    finally:
        buf.free()


def _oc(k, p):
    redun = {(2, 1): 32, (2, 2): 33, (4, 1): 34, (4, 2): 35, (8, 1): 36, (8, 2): 37, (16, 1): 38, (16, 2): 39,
             (4, 3): 40, (8, 3): 41, (16, 3): 42}[(k, p)]
    return (redun << 24) | 1


def _split_sgl(rng, total, C, n_iov, zero_iovs):
    """Random split of [0, total) into iov lengths (some cutting cells, some empty)."""
    cuts = sorted(set(int(x) for x in rng.integers(1, total, n_iov - 1)))
    lens = np.diff([0] + cuts + [total]).tolist()
    for _ in range(zero_iovs):
        lens.insert(int(rng.integers(0, len(lens))), 0)
    return lens


@pytest.mark.parametrize("k,p,C,recx_plan,n_iov,zeros,shift", [
    (4, 2, 8192, [(0, 3), (131072, 2)], 1, 0, 0),             # one iov: every cell in place
    (8, 2, 4096, [(0, 4), (4096 * 8 * 6, 3)], 7, 2, 0),        # cells cut across iovs, empty iovs
    (2, 1, 1000, [(0, 5), (30000, 4), (60000, 1)], 23, 3, 0),  # cell size not a multiple of 16
    (16, 2, 16384, [(16384 * 16, 3)], 5, 1, 0),                # leading gap
    (4, 3, 4096, [(0, 2), (32768, 2)], 64, 0, 0),               # many small iovs
    (8, 2, 65536, [(0, 6)], 1, 0, 3),                           # one iov at an odd address: cells in place, unaligned
    (8, 2, 65536 + 12, [(0, 3), (8 * 65548 * 5, 2)], 4, 1, 5),  # odd iovs, cells cut and in place
])
def test_recx_encode_sgl(oracle, ecglib, ctx, k, p, C, recx_plan, n_iov, zeros, shift):
    L = ecglib.lib()
    rng = np.random.default_rng(n_iov * 31 + k)
    stripe = k * C
    total = max(off + n * stripe for off, n in recx_plan)
    stream = rng.integers(0, 256, total, dtype=np.uint8)
    lens = _split_sgl(rng, total, C, n_iov, zeros)
    buf = ctx.alloc(total + 64 * len(lens) + 64)
    nstripes = sum(n for _, n in recx_plan)
    pbufs = [ctx.alloc(nstripes * C) for _ in range(p)]
    try:
        # iovs placed with gaps between them in device memory (the first at byte `shift`)
        iovs, pos, dev_off = [], 0, shift
        for ln in lens:
            buf.upload(stream[pos:pos + ln], offset=dev_off) if ln else None
            iovs.append(ecglib.Iov(buf.ptr + dev_off, ln))
            pos += ln
            dev_off += ln + 16 * int(rng.integers(1, 4))
        iov_arr = (ecglib.Iov * len(iovs))(*iovs)
        rx = (ecglib.EcRecx * len(recx_plan))(*[ecglib.EcRecx(off, n, 0) for off, n in recx_plan])
        pb = (ct.c_void_p * p)(*[b.ptr for b in pbufs])
        rc = L.ecg_obj_ec_recx_encode(ctx.h, _oc(k, p), C, iov_arr, len(iovs), rx, len(recx_plan), pb, None)
        assert rc == 0, ecglib.lib().ecg_strerror()
        ctx.sync()
        kern = ecglib.last_kernel()
        if n_iov == 1 and len(recx_plan) == 1:
            # one iov, one recx: every cell in place at base + (s*k + j)*C, parity at pbuf + s*C --
            # an affine table, which runs the offset kernel (no pointer table)
            assert kern.startswith(f"ecg_mm_kernel<{k},{p},"), kern
        else:
            assert kern.startswith("ecg_mm_ptr_kernel<"), kern
        if shift % 4:       # in-place cells at odd addresses, parity aligned: funnel-shifted inputs
            # (k = 8 on 16-byte lanes, g2, in both the offset and the pointer-table kernel)
            g = 2 if k == 8 else 1
            assert kern.endswith(f",g{g}>"), kern
        en = oracle.cauchy1(k, p)
        n = 0
        got = [b.download() for b in pbufs]
        for off, cnt in recx_plan:
            for j in range(cnt):
                cells = stream[off + j * stripe: off + (j + 1) * stripe].reshape(k, C)
                want = oracle.encode_data(en[k:], cells)
                for m in range(p):
                    assert np.array_equal(got[m][n * C:(n + 1) * C], want[m]), (off, j, m)
                n += 1
    finally:
        buf.free()
        for b in pbufs:
            b.free()


def test_recx_encode_rec2big(ecglib, ctx):
    L = ecglib.lib()
    C, k, p = 4096, 4, 2
    buf = ctx.alloc(3 * C * k)
    pb_bufs = [ctx.alloc(4 * C) for _ in range(p)]
    try:
        iov = (ecglib.Iov * 2)(ecglib.Iov(buf.ptr, 2 * C * k), ecglib.Iov(buf.ptr + 2 * C * k, C * k - 100))
        rx = (ecglib.EcRecx * 1)(ecglib.EcRecx(0, 3, 0))
        pb = (ct.c_void_p * p)(*[b.ptr for b in pb_bufs])
        assert L.ecg_obj_ec_recx_encode(ctx.h, _oc(k, p), C, iov, 2, rx, 1, pb, None) == -2013
        rx2 = (ecglib.EcRecx * 2)(ecglib.EcRecx(C * k, 1, 0), ecglib.EcRecx(0, 1, 0))
        assert L.ecg_obj_ec_recx_encode(ctx.h, _oc(k, p), C, iov, 2, rx2, 2, pb, None) == -1003
    finally:
        buf.free()
        for b in pb_bufs:
            b.free()


@pytest.mark.parametrize("k,p,C,S,moved", [(8, 2, 65536, 6, False), (4, 2, 4096 * 3 + 40, 5, False),
                                           (16, 3, 8192, 3, False), (8, 2, 65536, 6, True)])
def test_matmul_ptrs_affine_table(ctx, oracle, ecglib, k, p, C, S, moved):
    """A pointer table of the client's contiguous layout -- data cell j of
    stripe s at base + (s*k + j)*C, parity of stripe s at pbuf[m] + s*C
    (ref:src/object/cli_ec.c:510-536, 638-640) -- runs the offset kernel
    (no table upload); one cell moved elsewhere keeps the pointer-table
    kernel.  Same bytes either way."""
    rng = np.random.default_rng(k * 7 + C + S + moved)
    data = rng.integers(0, 256, (S, k, C), dtype=np.uint8)
    d = ctx.to_device(data)
    spare = ctx.alloc(C + 64)
    spare.upload(data[S - 1, 1])
    par = ctx.alloc(p * (S * C + 4096))
    try:
        cells = []
        for s in range(S):
            cells += [d.ptr + (s * k + j) * C for j in range(k)]
            cells += [par.ptr + r * (S * C + 4096) + s * C for r in range(p)]
        if moved:
            cells[(S - 1) * (k + p) + 1] = spare.ptr
        coef = oracle.cauchy1(k, p)[k:]
        ctx.matmul_ptrs(k, p, coef, C, S, cells)
        ctx.sync()
        kern = ecglib.last_kernel()
        assert kern.startswith("ecg_mm_ptr_kernel<" if moved else f"ecg_mm_kernel<{k},{p},"), kern
        raw = par.download()
        for r in range(p):
            got = raw[r * (S * C + 4096): r * (S * C + 4096) + S * C].reshape(S, C)
            for s in range(S):
                assert np.array_equal(got[s], oracle.encode_data(coef, data[s])[r]), (r, s)
    finally:
        d.free()
        spare.free()
        par.free()
