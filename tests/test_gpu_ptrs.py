"""GPU parity of the pointer-table product (ecg_matmul_ptrs) and of the
client's scatter-gather encode (ecg_obj_ec_recx_encode, restating
obj_ec_recx_encode / obj_ec_stripe_encode, ref:src/object/cli_ec.c:476-546,
593-663) against the CPU oracle.  Bit-exact."""
import ctypes as ct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("k,rows,C,S,aligned", [(8, 2, 65536, 12, True), (4, 3, 4096 * 3 + 48, 7, True),
                                                 (16, 2, 8192, 5, True), (6, 5, 1000, 9, False),
                                                 (2, 1, 4097, 4, False)])
def test_matmul_ptrs(oracle, ecglib, ctx, k, rows, C, S, aligned):
    """Cells scattered at random (disjoint, shuffled) offsets of one buffer."""
    rng = np.random.default_rng(k * 100 + rows)
    slot = (C + 15) // 16 * 16 + (0 if aligned else 16)
    nslots = S * (k + rows) + 8
    buf = ctx.alloc(nslots * slot)
    order = rng.permutation(nslots)[: S * (k + rows)]
    skew = 0 if aligned else 3
    host = rng.integers(0, 256, nslots * slot, dtype=np.uint8)
    try:
        buf.upload(host)
        addrs = [buf.ptr + int(o) * slot + skew for o in order]
        coef = rng.integers(0, 256, (rows, k), dtype=np.uint8)
        ctx.matmul_ptrs(k, rows, coef, C, S, addrs)
        ctx.sync()
        kern = ecglib.last_kernel()
        assert ("ptr_byte" in kern) == (not aligned or C % 16 != 0), kern
        dev = buf.download()
        for s in range(S):
            cells = np.stack([host[int(order[s * (k + rows) + j]) * slot + skew:][:C] for j in range(k)])
            want = oracle.encode_data(coef, cells)
            for r in range(rows):
                o = int(order[s * (k + rows) + k + r]) * slot + skew
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


@pytest.mark.parametrize("k,p,C,recx_plan,n_iov,zeros", [
    (4, 2, 8192, [(0, 3), (131072, 2)], 1, 0),             # one iov: every cell in place
    (8, 2, 4096, [(0, 4), (4096 * 8 * 6, 3)], 7, 2),        # cells cut across iovs, empty iovs
    (2, 1, 1000, [(0, 5), (30000, 4), (60000, 1)], 23, 3),  # unaligned cells
    (16, 2, 16384, [(16384 * 16, 3)], 5, 1),                # leading gap
    (4, 3, 4096, [(0, 2), (32768, 2)], 64, 0),               # many small iovs
])
def test_recx_encode_sgl(oracle, ecglib, ctx, k, p, C, recx_plan, n_iov, zeros):
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
        # iovs placed with gaps between them in device memory
        iovs, pos, dev_off = [], 0, 0
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
