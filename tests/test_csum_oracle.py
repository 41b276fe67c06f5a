"""CPU checks of the checksum oracle, no GPU.

Pins the bitwise C restatement (oracle/csum_ref.c) with the catalogue check
values, an independent table-driven Python restatement (oracle/csum_py.py),
zlib's adler32, and the reference's own chunk-geometry test cases
(ref:src/common/tests/checksum_tests.c:1272-1420), and checks the product's
host-side chunk math (ecg_csum_chunk_count / ecg_csum_record_chunksize, no
device call) against them.
"""
import json
import os
import zlib

import numpy as np
import pytest

from oracle import csum_py

GOLD = os.path.join(os.path.dirname(__file__), "golden")
TYPES = (1, 2, 3, 7)


def test_check_values(oracle):
    kat = json.load(open(os.path.join(GOLD, "kat.json")))["csum_check"]
    d = kat["input"].encode()
    assert oracle.crc16_t10dif(0, d) == int(kat["crc16_t10dif_seed0"], 16)
    assert oracle.crc32_iscsi(d, 0xFFFFFFFF) ^ 0xFFFFFFFF == int(kat["crc32_iscsi_seed_ffffffff_xor_ffffffff"], 16)
    assert oracle.crc64_ecma_refl(0, d) == int(kat["crc64_ecma_refl_seed0"], 16)
    assert oracle.adler32(1, d) == int(kat["adler32_seed1"], 16)
    assert csum_py.crc16_t10dif(0, d) == int(kat["crc16_t10dif_seed0"], 16)
    assert csum_py.crc32_iscsi(d, 0xFFFFFFFF) ^ 0xFFFFFFFF == int(kat["crc32_iscsi_seed_ffffffff_xor_ffffffff"], 16)
    assert csum_py.crc64_ecma_refl(0, d) == int(kat["crc64_ecma_refl_seed0"], 16)


def test_restatements_agree(oracle):
    rng = np.random.default_rng(11)
    for n in list(range(0, 40)) + [255, 256, 1000, 4099]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for seed in (0, 1, 0xBEEF, 0xFFFFFFFF):
            assert oracle.crc16_t10dif(seed & 0xFFFF, d) == csum_py.crc16_t10dif(seed & 0xFFFF, d)
            assert oracle.crc32_iscsi(d, seed) == csum_py.crc32_iscsi(d, seed)
            assert oracle.crc64_ecma_refl(seed, d) == csum_py.crc64_ecma_refl(seed, d)
            if (seed & 0xFFFF) < 65521 and (seed >> 16) < 65521:     # valid adler states only
                assert oracle.adler32(seed, d) == zlib.adler32(d, seed)


# (chunksize, rec_size, rx_idx, rx_nr) -> count, from test_recx_calc_chunks and
# test_csum_chunk_count (hi = rx_idx + rx_nr - 1), ref checksum_tests.c:1273-1306
CHUNK_COUNTS = [
    ((4, 1, 0, 0), 0), ((4, 1, 0, 1), 1), ((4, 2, 0, 1), 1), ((4, 1, 1, 16), 5),
    ((1, 1, 0, 1), 1), ((2, 1, 0, 2), 1), ((2, 1, 1, 2), 2), ((2, 1, 1, 3), 2), ((2, 1, 1, 5), 3),
    ((4, 1, 0, 11), 3),        # test_daos_checksummer_with_multiple_chunks: "11/4=3"
]

# (chunk index, expected first record, expected records, cs, rb, rx_idx, rx_nr),
# daos_recx_get_chunk_tests, ref checksum_tests.c:1356-1405
CHUNK_RANGES = [
    (0, 0, 2, 2, 1, 0, 10), (1, 2, 2, 2, 1, 0, 10), (2, 4, 2, 2, 1, 0, 10), (4, 8, 2, 2, 1, 0, 10),
    (0, 1, 1, 2, 1, 1, 2), (1, 2, 1, 2, 1, 1, 2), (0, 3, 5, 8, 1, 3, 5), (0, 3, 4, 8, 1, 3, 4),
    (0, 2, 6, 8, 1, 2, 50), (1, 8, 8, 8, 1, 2, 50), (5, 40, 8, 8, 1, 2, 50), (6, 48, 4, 8, 1, 2, 50),
    (1, 2, 2, 8, 4, 0, 10), (1, 2, 1, 2, 1, 0, 3), (0, 4, 4, 4, 1, 4, 4), (0, 16, 16, 16, 1, 16, 16),
    (0, 2**64 - 1, 1, 32 * 1024, 6, 2**64 - 1, 1),
]


@pytest.mark.parametrize("args,want", CHUNK_COUNTS)
def test_chunk_count(oracle, ecglib, args, want):
    cs, rb, idx, nr = args
    assert oracle.csum_chunk_count(cs, rb, idx, nr) == want
    assert len(csum_py.chunk_ranges(cs, rb, idx, nr)) == want
    assert ecglib.lib().ecg_csum_chunk_count(cs, rb, idx, nr) == want


def test_chunk_ranges():
    for ci, lo, nr, cs, rb, idx, rnr in CHUNK_RANGES:
        assert csum_py.chunk_ranges(cs, rb, idx, rnr)[ci] == (lo, nr)


def test_record_chunksize(oracle, ecglib):
    for cs, rb in [(32768, 1), (32768, 6), (32768, 65536), (16384, 4096), (10, 4), (4, 4)]:
        want = rb if rb > cs else cs // rb * rb
        assert oracle.csum_record_chunksize(cs, rb) == want
        assert ecglib.lib().ecg_csum_record_chunksize(cs, rb) == want


@pytest.mark.parametrize("htype", TYPES)
def test_extent_chunking_agrees(oracle, htype):
    """C oracle (calc_csum_recx_with_no_map restatement) == Python restatement
    over ragged geometries, including unaligned starts and records > chunk."""
    rng = np.random.default_rng(htype)
    for cs, rb, idx, nr in [(4, 1, 1, 16), (8, 1, 2, 50), (8, 4, 0, 10), (32, 6, 7, 40), (16, 64, 3, 5),
                            (1024, 1, 1000, 3000), (4096, 8, 511, 1025), (10, 4, 5, 33)]:
        buf = rng.integers(0, 256, rb * nr, dtype=np.uint8)
        got = oracle.csum_extents(htype, cs, rb, idx, nr, buf)[0].tolist()
        assert got == csum_py.csum_extent(htype, cs, rb, idx, nr, buf.tobytes()), (cs, rb, idx, nr)


def test_unsupported_type(ecglib):
    assert ecglib.lib().ecg_csum_len(4) == -2037      # SHA1: -DER_NOTSUPPORTED
    assert [ecglib.lib().ecg_csum_len(t) for t in TYPES] == [2, 4, 8, 4]
