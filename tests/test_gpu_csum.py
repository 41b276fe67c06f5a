"""GPU parity of the chunked checksums (include/ecg_csum.h) against the CPU
oracle (oracle/csum_ref.c, pinned in tests/test_csum_oracle.py).

Bit-exact: every checksum of every chunk must equal the oracle's.  Covers the
DAOS hash types (crc16 / crc32 / crc64 / adler32), the csummer's chunk
geometry (unaligned record index, records larger than the chunk, partial first
and last chunks, single record), the 16-byte-aligned and byte-granular kernel
paths, batched extents, and the rebuild pattern it exists for: parity cells
regenerated on the device, then checksummed without leaving HBM
(ref:src/object/srv_obj_migrate.c:1096-1181).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TYPES = (1, 2, 3, 7)
DT = {2: np.uint16, 4: np.uint32, 8: np.uint64}


def _dev_csum(ecglib, ctx, htype, cs, rb, idx, nr, host, ext_stride=0, n_ext=1, offset=0):
    """Upload host bytes at device offset `offset`, checksum on the device, return [n_ext][n]."""
    L = ecglib.lib()
    n = L.ecg_csum_chunk_count(cs, rb, idx, nr)
    cl = L.ecg_csum_len(htype)
    buf = ecglib.DeviceBuffer(ctx, offset + max(1, host.nbytes))
    out = ecglib.DeviceBuffer(ctx, max(8, n_ext * n * cl))
    try:
        buf.upload(host, offset=offset)
        out.fill(0xA5)
        ctx.csum_extents(htype, cs, rb, idx, nr, buf.ptr + offset, ext_stride, n_ext, out.ptr)
        ctx.sync()
        assert "crc" in L.ecg_last_kernel().decode() or "adler" in L.ecg_last_kernel().decode()
        return out.download(n_ext * n * cl).view(DT[cl]).reshape(n_ext, n)
    finally:
        buf.free()
        out.free()


GEOMS = [
    # (chunksize, rec_size, rx_idx, rx_nr)
    (32768, 1, 0, 1 << 20),            # DAOS default chunk over a 1 MiB cell
    (16384, 1, 0, 5 << 16),            # ftest cksum_size 16 KiB
    (32768, 1, 100, 200000),           # unaligned index: partial first + last chunk
    (4096, 8, 3, 10000),               # 8-byte records
    (32768, 6, 7, 30001),              # record size not dividing the chunk (rec chunk 32766)
    (4096, 65536, 5, 9),               # records larger than the chunk: one chunk per record
    (1024, 1, 0, 1),                   # single record
    (64, 1, 0, 1000),                  # tiny chunks (4 pieces) + tails
    (1 << 20, 1, 0, (1 << 20) + 15),   # one big chunk + 15-byte tail chunk
    (24, 1, 0, 1000),                  # chunk not a multiple of 16: byte path
]


@pytest.mark.parametrize("htype", TYPES)
@pytest.mark.parametrize("geom", GEOMS)
def test_csum_parity(oracle, ecglib, ctx, htype, geom):
    cs, rb, idx, nr = geom
    rng = np.random.default_rng(hash((htype,) + geom) & 0xFFFFFFFF)
    host = rng.integers(0, 256, rb * nr, dtype=np.uint8)
    got = _dev_csum(ecglib, ctx, htype, cs, rb, idx, nr, host)
    want = oracle.csum_extents(htype, cs, rb, idx, nr, host)
    assert got.shape == want.shape
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]


SHAPE_GEOMS = GEOMS + [(1 << 20, 1, 0, 3 << 20), ((1 << 20) + 4096, 1, 5, 2 << 20),
                       (65536, 16, 0, 70001), (2048, 1, 0, 100000),
                       (4096, 1, 0, 4096 * 7 + 16 * 5), (8192, 8, 0, 3001),
                       # step counts that are not multiples of the 4-piece Horner
                       # step (zero prefix) in every shape
                       ((1 << 20) + 5120 + 48, 1, 3, 3 << 20), (1040, 1, 0, 1040 * 9 + 7),
                       (5 * 4096 + 1024, 1, 0, 7 * (5 * 4096 + 1024) - 16)]


def _shape(cs, rb, nch, n_ext):
    """The kernel shape ecg_csum_extents picks (ecg_csum.c): a workgroup per
    chunk for fewer than 4096 chunks of >= 16 steps, a 16-lane group per
    chunk of <= 8 steps, else a wave per chunk."""
    rcs = cs - cs % rb if rb <= cs else rb
    steps = (rcs // 16 + 63) // 64
    if n_ext * nch < 4096 and steps >= 16:
        return "split"
    return "group" if steps <= 8 else "wave"


@pytest.mark.parametrize("many", [False, True])
@pytest.mark.parametrize("htype", (1, 2, 3, 7))
@pytest.mark.parametrize("geom", SHAPE_GEOMS)
def test_crc_kernel_shapes(oracle, ecglib, ctx, many, htype, geom):
    """Every kernel shape the geometry selects: a workgroup per chunk (few
    long chunks -- CRC: the waves' slice CRCs shifted and combined; adler32:
    the threads' position-weighted sums added; chunks shorter than the
    workgroup's slices leave waves idle), a 16-lane group per short chunk
    (4 chunks per wave, the wave's last groups idle past the final chunk),
    and a wave per chunk.  `many` repeats the extent (stride 0) until there
    are >= 4096 chunks, which turns the workgroup shape into the wave shape."""
    cs, rb, idx, nr = geom
    L = ecglib.lib()
    rng = np.random.default_rng((hash(geom) + htype) & 0xFFFFFFFF)
    host = rng.integers(0, 256, rb * nr, dtype=np.uint8)
    nch = L.ecg_csum_chunk_count(cs, rb, idx, nr)
    n_ext = -(-4096 // nch) if many else 1
    got = _dev_csum(ecglib, ctx, htype, cs, rb, idx, nr, host, ext_stride=0, n_ext=n_ext)
    kern = L.ecg_last_kernel().decode()
    if "bytes" not in kern:
        want_shape = _shape(cs, rb, nch, n_ext)
        assert ("split" in kern) == (want_shape == "split"), kern
        assert ("group" in kern) == (want_shape == "group" and htype != 7), kern
    want = oracle.csum_extents(htype, cs, rb, idx, nr, host)
    assert np.array_equal(got, np.tile(want, (n_ext, 1)))


@pytest.mark.parametrize("htype", TYPES)
@pytest.mark.parametrize("offset", [1, 3, 8, 15])
def test_csum_unaligned_base(oracle, ecglib, ctx, htype, offset):
    """Extents starting off a 16-byte boundary take the byte-granular kernel."""
    rng = np.random.default_rng(offset)
    host = rng.integers(0, 256, 100000, dtype=np.uint8)
    got = _dev_csum(ecglib, ctx, htype, 4096, 1, 0, host.size, host, offset=offset)
    assert "bytes" in ecglib.lib().ecg_last_kernel().decode()
    assert np.array_equal(got, oracle.csum_extents(htype, 4096, 1, 0, host.size, host))


@pytest.mark.parametrize("htype", TYPES)
def test_csum_batched_extents(oracle, ecglib, ctx, htype):
    """64 cells of 256 KiB + 4 KiB pitch, one launch."""
    C, pitch, n = 256 << 10, (256 << 10) + 4096, 64
    rng = np.random.default_rng(htype + 100)
    host = rng.integers(0, 256, pitch * n, dtype=np.uint8)
    got = _dev_csum(ecglib, ctx, htype, 32768, 1, 0, C, host, ext_stride=pitch, n_ext=n)
    want = oracle.csum_extents(htype, 32768, 1, 0, C, host, ext_stride=pitch, n_ext=n)
    assert np.array_equal(got, want)


def test_csum_special_data(oracle, ecglib, ctx):
    """All-zero and all-0xFF chunks (crc64's inverted register must still fold in)."""
    for fill in (0x00, 0xFF):
        host = np.full(300000, fill, dtype=np.uint8)
        for htype in TYPES:
            got = _dev_csum(ecglib, ctx, htype, 32768, 1, 0, host.size, host)
            assert np.array_equal(got, oracle.csum_extents(htype, 32768, 1, 0, host.size, host)), (fill, htype)


def test_csum_errors(ecglib, ctx):
    L = ecglib.lib()
    buf = ecglib.DeviceBuffer(ctx, 4096)
    try:
        assert L.ecg_csum_extents(ctx.h, 5, 4096, 1, 0, 4096, buf.ptr, 0, 1, buf.ptr, None) == -2037
        assert L.ecg_csum_extents(ctx.h, 2, 0, 1, 0, 4096, buf.ptr, 0, 1, buf.ptr, None) == -1003
        assert L.ecg_csum_extents(ctx.h, 2, 4096, 0, 0, 4096, buf.ptr, 0, 1, buf.ptr, None) == -1003
        assert L.ecg_csum_extents(ctx.h, 2, 4096, 1, 0, 0, buf.ptr, 0, 1, buf.ptr, None) == 0
    finally:
        buf.free()


@pytest.mark.parametrize("htype", (1, 2, 3))
def test_rebuild_parity_then_csum(oracle, ecglib, ctx, htype):
    """Rebuild pattern: encode EC_8P2 parity on the device, checksum the
    regenerated parity cells in place (32 KiB chunks), compare with the oracle
    encode + oracle checksums."""
    k, p, C, S = 8, 2, 1 << 20, 16
    rng = np.random.default_rng(7)
    data = rng.integers(0, 256, S * k * C, dtype=np.uint8)
    d = ecglib.DeviceBuffer(ctx, data.nbytes)
    par = ecglib.DeviceBuffer(ctx, p * S * C)
    cl = ecglib.lib().ecg_csum_len(htype)
    out = ecglib.DeviceBuffer(ctx, p * S * (C // 32768) * cl)
    try:
        d.upload(data)
        ctx.encode(k, p, C, S, d.ptr, k * C, par.ptr, S * C, C)
        # parity cells are [p][S][C]: p*S extents of C bytes at pitch C
        ctx.csum_extents(htype, 32768, 1, 0, C, par.ptr, C, p * S, out.ptr)
        ctx.sync()
        got = out.download().view(DT[cl]).reshape(p * S, -1)
        want_par = oracle.encode_batch(k, p, C, S, data, nthreads=8, simd=True)
        want = oracle.csum_extents(htype, 32768, 1, 0, C, want_par, ext_stride=C, n_ext=p * S)
        assert np.array_equal(got, want)
    finally:
        d.free()
        par.free()
        out.free()


# ---- fused product + checksum (ecg_encode_csum / ecg_recover_csum) ----------

def _want_cell_csums(oracle, htype, cs, rb, cells):
    """oracle checksums of each cell (rows of `cells`), as extents at index 0."""
    C = cells.shape[-1]
    flat = np.ascontiguousarray(cells.reshape(-1, C))
    return oracle.csum_extents(htype, cs, rb, 0, C // rb, flat.reshape(-1), ext_stride=C, n_ext=flat.shape[0])


FUSED = [
    # (k, p, C, S, chunksize, rec_size, htype)
    (2, 1, 1 << 20, 4, 32768, 1, 2),
    (4, 2, 1 << 20, 6, 32768, 1, 2),
    (8, 2, 1 << 20, 4, 32768, 1, 2),
    (8, 2, 1 << 20, 4, 32768, 1, 1),
    (8, 2, 1 << 20, 4, 32768, 1, 3),
    (16, 2, 128 << 10, 8, 16384, 1, 2),
    (8, 3, 256 << 10, 5, 4096, 1, 3),
    (4, 1, 65536 + 48, 3, 32768, 1, 2),       # ragged last chunk (not a 4 KiB multiple)
    (4, 2, 100000, 3, 8192, 8, 1),            # 8-byte records, ragged
    (16, 3, 40960, 3, 12288, 4096, 3),        # records of 4 KiB, 3 per chunk
]


@pytest.mark.parametrize("case", FUSED)
def test_encode_csum_fused(oracle, ecglib, ctx, case):
    k, p, C, S, cs, rb, htype = case
    L = ecglib.lib()
    nch = L.ecg_csum_chunk_count(cs, rb, 0, C // rb)
    cl = L.ecg_csum_len(htype)
    rng = np.random.default_rng(sum(case))
    data = rng.integers(0, 256, S * k * C, dtype=np.uint8)
    d = ctx.to_device(data)
    par = ctx.alloc(p * S * C)
    out = ctx.alloc(p * S * nch * cl)
    try:
        ctx.encode_csum(k, p, C, S, d.ptr, k * C, par.ptr, S * C, C, htype, cs, rb, out.ptr)
        ctx.sync()
        assert "ecg_mm_csum" in L.ecg_last_kernel().decode(), L.ecg_last_kernel()
        got_par = par.download().reshape(p, S, C)
        want_par = oracle.encode_batch(k, p, C, S, data, nthreads=8, simd=True).reshape(p, S, C)
        assert np.array_equal(got_par, want_par)
        got = out.download().view(DT[cl]).reshape(p, S, nch)
        want = _want_cell_csums(oracle, htype, cs, rb, want_par).reshape(p, S, nch)
        assert np.array_equal(got, want), np.argwhere(got != want)[:5]
    finally:
        d.free(); par.free(); out.free()


ITEM_CASES = [
    # (k, p, C, S, chunksize, htype): chunks cut into work items of `cols` columns, ragged last chunks
    (8, 2, 3 * 65536 + 4096 * 3 + 48, 3, 65536, 2),      # last chunk 3 columns + 48 B
    (4, 1, (1 << 20) + 48, 2, 1 << 20, 1),                 # 256-column chunks, last chunk 48 B
    (8, 3, 5 * 32768, 2, 32768, 3),
    (16, 2, 131072 + 16, 2, 40960, 2),                     # 10-column chunks
]


@pytest.mark.parametrize("cols", [1, 2, 3, 5, 0])
@pytest.mark.parametrize("case", ITEM_CASES)
def test_encode_csum_fused_items(oracle, ecglib, ctx, case, cols):
    """Every split of a chunk into work items (ecg_set_fused_cols; 0 = the
    default) yields the same checksums: per-item multipliers, the last
    chunk's own rows (zero padding removed), xorout once per chunk."""
    k, p, C, S, cs, htype = case
    L = ecglib.lib()
    nch = L.ecg_csum_chunk_count(cs, 1, 0, C)
    cl = L.ecg_csum_len(htype)
    rng = np.random.default_rng(sum(case) + cols)
    data = rng.integers(0, 256, S * k * C, dtype=np.uint8)
    d = ctx.to_device(data)
    par = ctx.alloc(p * S * C)
    out = ctx.alloc(p * S * nch * cl)
    assert L.ecg_set_fused_cols(ctx.h, cols) == 0
    try:
        ctx.encode_csum(k, p, C, S, d.ptr, k * C, par.ptr, S * C, C, htype, cs, 1, out.ptr)
        ctx.sync()
        assert "ecg_mm_csum" in L.ecg_last_kernel().decode(), L.ecg_last_kernel()
        want_par = oracle.encode_batch(k, p, C, S, data, nthreads=8, simd=True).reshape(p, S, C)
        assert np.array_equal(par.download().reshape(p, S, C), want_par)
        got = out.download().view(DT[cl]).reshape(p, S, nch)
        want = _want_cell_csums(oracle, htype, cs, 1, want_par).reshape(p, S, nch)
        assert np.array_equal(got, want), np.argwhere(got != want)[:5]
    finally:
        L.ecg_set_fused_cols(ctx.h, 0)
        d.free(); par.free(); out.free()


@pytest.mark.parametrize("errs", [[3, 9], [9, 3], [8, 9], [0], [0, 1], [5]])
@pytest.mark.parametrize("htype", (2, 3))
def test_recover_csum_fused(oracle, ecglib, ctx, errs, htype):
    k, p, C, S, cs = 8, 2, 256 << 10, 6, 32768
    L = ecglib.lib()
    nch = C // cs
    cl = L.ecg_csum_len(htype)
    rng = np.random.default_rng(len(errs) * 10 + htype)
    data = rng.integers(0, 256, (S, k, C), dtype=np.uint8)
    en = oracle.cauchy1(k, p)
    stripes = np.zeros((S, k + p, C), dtype=np.uint8)
    for s in range(S):
        stripes[s, :k] = data[s]
        stripes[s, k:] = oracle.encode_data(en[k:], data[s])
    broken = stripes.copy()
    broken[:, errs] = 0
    d = ctx.to_device(broken)
    out = ctx.alloc(len(errs) * S * nch * cl)
    try:
        ctx.recover_csum(k, p, C, S, d.ptr, (k + p) * C, errs, htype, cs, 1, out.ptr)
        ctx.sync()
        got_st = d.download().reshape(S, k + p, C)
        assert np.array_equal(got_st, stripes)
        got = out.download().view(DT[cl]).reshape(len(errs), S, nch)
        for i, e in enumerate(errs):
            want = _want_cell_csums(oracle, htype, cs, 1, stripes[:, e])
            assert np.array_equal(got[i], want), (e, i)
    finally:
        d.free(); out.free()


@pytest.mark.parametrize("variant", ["adler32", "chunk_not_4k", "unaligned", "k_over_16"])
def test_encode_csum_fallback(oracle, ecglib, ctx, variant):
    """Shapes the fused kernel does not take run product + checksum launches."""
    k, p, C, S, cs, rb, htype, off = 4, 2, 1 << 18, 3, 32768, 1, 2, 0
    if variant == "adler32":
        htype = 7
    elif variant == "chunk_not_4k":
        cs = 6000
    elif variant == "unaligned":
        off = 4
    else:
        k = 20
    L = ecglib.lib()
    nch = L.ecg_csum_chunk_count(cs, rb, 0, C // rb)
    cl = L.ecg_csum_len(htype)
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, S * k * C, dtype=np.uint8)
    d = ctx.alloc(data.nbytes + 64)
    d.upload(data, offset=off)
    par = ctx.alloc(p * S * C + 64)
    out = ctx.alloc(p * S * nch * cl)
    try:
        ctx.encode_csum(k, p, C, S, d.ptr + off, k * C, par.ptr + off, S * C, C, htype, cs, rb, out.ptr)
        ctx.sync()
        assert "ecg_mm_csum_kernel" not in L.ecg_last_kernel().decode()
        want_par = oracle.encode_batch(k, p, C, S, data, nthreads=8, simd=True).reshape(p, S, C)
        assert np.array_equal(par.download(p * S * C, offset=off).reshape(p, S, C), want_par)
        got = out.download().view(DT[cl]).reshape(p, S, nch)
        assert np.array_equal(got, _want_cell_csums(oracle, htype, cs, rb, want_par).reshape(p, S, nch))
    finally:
        d.free(); par.free(); out.free()


def test_encode_csum_errors(ecglib, ctx):
    L = ecglib.lib()
    b = ctx.alloc(1 << 16)
    try:
        assert L.ecg_encode_csum(ctx.h, 4, 2, 4096, 1, b.ptr, 4 * 4096, b.ptr, 4096, 4096, 4, 4096, 1, b.ptr,
                                 None) == -2037
        assert L.ecg_encode_csum(ctx.h, 4, 2, 4097, 1, b.ptr, 4 * 4097, b.ptr, 4097, 4097, 2, 4096, 2, b.ptr,
                                 None) == -1003          # cell not a multiple of the record size
    finally:
        b.free()


def test_encode_csum_misaligned_csums(oracle, ecglib, ctx):
    """A checksum array that is only 2-byte aligned takes the two-pass path."""
    k, p, C, S, cs = 4, 2, 1 << 18, 2, 32768
    nch = C // cs
    rng = np.random.default_rng(9)
    data = rng.integers(0, 256, S * k * C, dtype=np.uint8)
    d = ctx.to_device(data)
    par = ctx.alloc(p * S * C)
    out = ctx.alloc(p * S * nch * 2 + 16)
    try:
        ctx.encode_csum(k, p, C, S, d.ptr, k * C, par.ptr, S * C, C, 1, cs, 1, out.ptr + 2)
        ctx.sync()
        want_par = oracle.encode_batch(k, p, C, S, data, nthreads=8, simd=True).reshape(p, S, C)
        got = out.download(p * S * nch * 2, offset=2).view(np.uint16).reshape(p, S, nch)
        assert np.array_equal(got, _want_cell_csums(oracle, 1, cs, 1, want_par).reshape(p, S, nch))
    finally:
        d.free(); par.free(); out.free()


DEFAULT_KINDS = [  # (k, p, htype): each fused instantiation's table kind (ecg_fused_kernels.hip CS_TB)
    (8, 2, 2), (8, 2, 3), (8, 2, 1), (4, 2, 2), (4, 2, 3), (8, 1, 2), (8, 1, 3), (16, 2, 2), (16, 2, 3),
    (8, 3, 2), (8, 3, 3), (4, 1, 2), (16, 1, 2), (2, 2, 3),
]


@pytest.mark.parametrize("cols", [0, 3, 8])        # the default split of a chunk into work items / others
@pytest.mark.parametrize("case", DEFAULT_KINDS)
def test_encode_csum_fused_kinds(oracle, ecglib, ctx, case, cols):
    """Every fused instantiation with its table kind (the byte tables for
    crc64 and for crc32 at EC_8P2, the 5-bit tables elsewhere) gives the
    oracle's parity and chunk checksums -- ragged last chunk and 16-byte tail
    of the cell included, items of the default and of other column counts."""
    k, p, htype = case
    C, S, cs = 3 * 32768 + 4096 + 16, 3, 32768
    L = ecglib.lib()
    nch = L.ecg_csum_chunk_count(cs, 1, 0, C)
    cl = L.ecg_csum_len(htype)
    rng = np.random.default_rng(k * 10 + p + htype + cols)
    data = rng.integers(0, 256, S * k * C, dtype=np.uint8)
    d = ctx.to_device(data)
    par = ctx.alloc(p * S * C)
    out = ctx.alloc(p * S * nch * cl)
    try:
        assert L.ecg_set_fused_cols(ctx.h, cols) == 0
        ctx.encode_csum(k, p, C, S, d.ptr, k * C, par.ptr, S * C, C, htype, cs, 1, out.ptr)
        ctx.sync()
        assert L.ecg_last_kernel().decode().startswith(f"ecg_mm_csum_kernel<{k},{p},"), L.ecg_last_kernel()
        want_par = oracle.encode_batch(k, p, C, S, data, nthreads=8, simd=True).reshape(p, S, C)
        assert np.array_equal(par.download().reshape(p, S, C), want_par)
        got = out.download().view(DT[cl]).reshape(p, S, nch)
        want = _want_cell_csums(oracle, htype, cs, 1, want_par).reshape(p, S, nch)
        assert np.array_equal(got, want), np.argwhere(got != want)[:5]
    finally:
        L.ecg_set_fused_cols(ctx.h, 0)
        d.free(); par.free(); out.free()
