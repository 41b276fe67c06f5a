"""Second, independent restatement of the DAOS chunked checksums (pure Python,
table-driven, small inputs only).  TEST INFRASTRUCTURE ONLY.

oracle/csum_ref.c restates the hashes bit by bit; this file builds the usual
256-entry byte tables from the polynomials and walks the chunk ranges with its
own arithmetic (floor/ceil over record indexes, ref:src/common/checksum.c:
1457-1565), so the two share no code.  Hash semantics: see csum_ref.c header.
"""
from __future__ import annotations

import zlib


def _tbl_refl(poly: int, width: int):
    t = []
    for v in range(256):
        c = v
        for _ in range(8):
            c = (c >> 1) ^ poly if c & 1 else c >> 1
        t.append(c)
    return t


def _tbl_msb(poly: int, width: int):
    top, mask = 1 << (width - 1), (1 << width) - 1
    t = []
    for v in range(256):
        c = v << (width - 8)
        for _ in range(8):
            c = ((c << 1) ^ poly) & mask if c & top else (c << 1) & mask
        t.append(c)
    return t


_T16 = _tbl_msb(0x8BB7, 16)
_T32 = _tbl_refl(0x82F63B78, 32)
_T64 = _tbl_refl(0xC96C5795D7870F42, 64)


def crc16_t10dif(seed: int, data: bytes) -> int:
    c = seed
    for b in data:
        c = ((c << 8) & 0xFFFF) ^ _T16[((c >> 8) ^ b) & 0xFF]
    return c


def crc32_iscsi(data: bytes, seed: int) -> int:
    c = seed
    for b in data:
        c = (c >> 8) ^ _T32[(c ^ b) & 0xFF]
    return c


def crc64_ecma_refl(seed: int, data: bytes) -> int:
    c = ~seed & (2**64 - 1)
    for b in data:
        c = (c >> 8) ^ _T64[(c ^ b) & 0xFF]
    return ~c & (2**64 - 1)


def adler32(seed: int, data: bytes) -> int:
    return zlib.adler32(data, seed)     # zlib's adler32(data, value) has the same seed semantics


HASH = {1: lambda d: crc16_t10dif(0, d), 2: lambda d: crc32_iscsi(d, 0),
        3: lambda d: crc64_ecma_refl(0, d), 7: lambda d: adler32(0, d)}


def chunk_ranges(chunksize: int, rec_size: int, rx_idx: int, rx_nr: int):
    """[(first_record, n_records)] of every checksum chunk of one extent."""
    if rx_nr == 0:
        return []
    rcs = rec_size if rec_size > chunksize else (chunksize // rec_size) * rec_size
    per = rcs // rec_size
    lo, hi = rx_idx, rx_idx + rx_nr - 1
    out = []
    start = (lo // per) * per
    while start <= hi:
        a, b = max(start, lo), min(start + per - 1, hi)
        out.append((a, b - a + 1))
        start += per
    return out


def csum_extent(htype: int, chunksize: int, rec_size: int, rx_idx: int, rx_nr: int, buf: bytes):
    return [HASH[htype](bytes(buf[(a - rx_idx) * rec_size:(a - rx_idx + n) * rec_size]))
            for a, n in chunk_ranges(chunksize, rec_size, rx_idx, rx_nr)]
