"""Rebuild of a parity shard (ecg_migrate_update_parity, restating
migrate_update_parity, ref:src/object/srv_obj_migrate.c:1096-1181).

CPU: the library's plan sizing against the restated walk (oracle/migrate_py.py)
over aligned / unaligned / short ranges, encode and replicate-only.
GPU: every piece -- recx, bytes (parity cells = this shard's row of the
Cauchy1 encode of the full stripe, replicated records = the fetched bytes) and
chunk checksums -- against the oracle, bit-exact; the fused checksum path
(cells on chunk boundaries) and the grouped one (iod_size 3: records per chunk
does not divide the parity index) both run."""
import ctypes as ct

import numpy as np
import pytest

from oracle import migrate_py


def _oc(k, p):
    redun = {(2, 1): 32, (2, 2): 33, (4, 1): 34, (4, 2): 35, (8, 1): 36, (8, 2): 37, (16, 1): 38, (16, 2): 39,
             (4, 3): 40, (8, 3): 41, (16, 3): 42}[(k, p)]
    return (redun << 24) | 1


RANGES = [  # k, p, e_len, iod_size, offset (records), size (records), encode
    (4, 2, 1024, 1, 0, 4096 * 3, True),             # whole stripes
    (4, 2, 1024, 1, 1000, 4096 * 3 + 77, True),     # partial head and tail
    (8, 2, 512, 8, 4096, 300, True),                # shorter than a stripe: replicate only
    (2, 1, 4096, 3, 5, 8192 * 2, True),             # iod_size 3
    (16, 2, 256, 4, 0, 4096 * 2 + 256, True),
    (4, 2, 1024, 1, 512, 3000, False),              # replicate by cells
    (4, 2, 32768, 1, 0, 131072 * 2, True),          # cells on 32 KiB chunk boundaries: fused checksums
    (8, 2, 8192, 4, 65536 - 100, 65536 * 3, True),  # 4-byte records, 8192 per chunk: fused, partial ends
]


@pytest.mark.parametrize("rng_args", RANGES)
def test_plan_size_matches_walk(ecglib, rng_args):
    k, p, e_len, isz, off, size, enc = rng_args
    L = ecglib.lib()
    n, npar, cb = ct.c_uint32(), ct.c_uint32(), ct.c_uint64()
    assert L.ecg_migrate_plan_size(_oc(k, p), e_len, isz, off, size, int(enc), 2, 32768, ct.byref(n),
                                   ct.byref(npar), ct.byref(cb)) == 0
    w = migrate_py.walk(k, e_len, off, size, enc)
    assert n.value == len(w) and npar.value == sum(1 for x in w if x[2])
    want_cb = sum(L.ecg_csum_chunk_count(32768, isz, ix, nr) * 4 for ix, nr, _, _ in w)
    assert cb.value == want_cb
    assert L.ecg_migrate_plan_size((1 << 24) | 1, e_len, isz, off, size, 1, 0, 0, ct.byref(n), None,
                                   None) == -ecglib.DER_INVAL               # not an EC class


@pytest.mark.gpu
@pytest.mark.parametrize("csum_type", [0, 2, 3])
@pytest.mark.parametrize("rng_args", RANGES)
def test_update_parity_matches_oracle(oracle, ecglib, ctx, rng_args, csum_type):
    k, p, e_len, isz, off, size, enc = rng_args
    L = ecglib.lib()
    shard = k + p - 1
    rng = np.random.default_rng(size + k)
    host = rng.integers(0, 256, size * isz, dtype=np.uint8)
    want = migrate_py.update_parity(oracle, k, p, e_len, isz, shard, host, off, size, enc, csum_type, 32768)
    n, npar, cb = ct.c_uint32(), ct.c_uint32(), ct.c_uint64()
    assert L.ecg_migrate_plan_size(_oc(k, p), e_len, isz, off, size, int(enc), csum_type, 32768, ct.byref(n),
                                   ct.byref(npar), ct.byref(cb)) == 0
    buf = ctx.to_device(host)
    par = ctx.alloc(max(1, npar.value * e_len * isz))
    cs = ctx.alloc(max(8, cb.value))
    pieces = (ecglib.MigratePiece * max(1, n.value))()
    got_n = ct.c_uint32()
    try:
        rc = L.ecg_migrate_update_parity(ctx.h, _oc(k, p), e_len, isz, shard, buf.ptr, off, size, int(enc),
                                         csum_type, 32768, par.ptr, cs.ptr, pieces, n.value, ct.byref(got_n), None)
        assert rc == 0, L.ecg_strerror()
        ctx.sync()
        assert got_n.value == len(want)
        pbytes, cbytes = par.download(), cs.download()
        cl = {2: 4, 3: 8}.get(csum_type, 0)
        for pc, w in zip(pieces[:got_n.value], want):
            assert (pc.recx.rx_idx, pc.recx.rx_nr) == w["recx"]
            assert bool(pc.parity) == w["parity"]
            src = pbytes if pc.parity else host
            assert np.array_equal(src[pc.buf_off:pc.buf_off + pc.buf_len], w["bytes"]), w["recx"]
            if csum_type:
                dt = np.uint32 if cl == 4 else np.uint64
                got = cbytes[pc.csum_off:pc.csum_off + pc.nr_csums * cl].view(dt)
                assert np.array_equal(got, w["csums"]), w["recx"]
    finally:
        buf.free()
        par.free()
        cs.free()


@pytest.mark.gpu
def test_update_parity_errors(ecglib, ctx):
    L = ecglib.lib()
    buf = ctx.alloc(4096 * 4)
    pieces = (ecglib.MigratePiece * 1)()
    n = ct.c_uint32()
    try:
        # a data shard is not rebuilt through parity (ref :1129 asserts shard >= k)
        assert L.ecg_migrate_update_parity(ctx.h, _oc(4, 2), 1024, 1, 2, buf.ptr, 0, 4096, 1, 0, 0, buf.ptr, None,
                                           pieces, 1, ct.byref(n), None) == -ecglib.DER_INVAL
        # two pieces (stripe + tail) do not fit a capacity of one
        assert L.ecg_migrate_update_parity(ctx.h, _oc(4, 2), 1024, 1, 4, buf.ptr, 0, 4097, 1, 0, 0, buf.ptr, None,
                                           pieces, 1, ct.byref(n), None) == -ecglib.DER_REC2BIG
    finally:
        buf.free()


@pytest.mark.gpu
def test_update_parity_fused_when_aligned(ecglib, ctx):
    """Whole stripes with cells on chunk boundaries: the kept parity row and
    its checksums come from one fused launch (k data cells in, 1 cell out)."""
    L = ecglib.lib()
    k, p, e_len = 4, 2, 32768
    buf = ctx.alloc(k * e_len * 4)
    par = ctx.alloc(4 * e_len)
    cs = ctx.alloc(4 * 4)
    pieces = (ecglib.MigratePiece * 4)()
    n = ct.c_uint32()
    try:
        buf.fill(0x21)
        assert L.ecg_migrate_update_parity(ctx.h, _oc(k, p), e_len, 1, 4, buf.ptr, 0, 4 * k * e_len, 1, 2, 32768,
                                           par.ptr, cs.ptr, pieces, 4, ct.byref(n), None) == 0
        ctx.sync()
        assert n.value == 4 and all(pc.parity for pc in pieces)
        assert ecglib.last_kernel() == "ecg_mm_csum_kernel<4,1,crc32>", ecglib.last_kernel()
    finally:
        buf.free()
        par.free()
        cs.free()
