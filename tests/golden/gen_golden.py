"""Generate tests/golden/fixtures.npz (committed; re-run only to regenerate).

Inputs reuse the data patterns and sizes of the reference's own EC tests:
  make_buffer (runs of 1000 bytes of start + i % 25)  ref:src/tests/suite/daos_rebuild_common.c:661-674
  sizes DATA_SIZE 4 MiB+347, 933, 311, 8569, 37      ref:src/tests/suite/daos_rebuild_common.c:654-658
  cell j filled with byte j, or 0x80 (overwrite)      ref:src/tests/suite/daos_aggregate_ec.c:90-109
  TEST_EC_CELL_SZ = 32 KiB                            ref:src/tests/suite/daos_aggregate_ec.c:32
Expected outputs come from the CPU oracle (oracle/ec_ref.c), cross-checked
here against the independent numpy restatement (oracle/gf_np.py) before
anything is written.  The reference itself cannot run here (ISA-L is not in
the image, DAOS needs its SCons build), so these fixtures pin the oracle and
the GPU path to each other and to the KATs in kat.json -- "parity unpinned"
by any reference-produced bytes.
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)

from oracle import gf_np, ref  # noqa: E402


def make_buffer(start: int, total: int) -> np.ndarray:
    out = np.empty(total, dtype=np.uint8)
    i = 0
    pos = 0
    while pos < total:
        n = min(1000, total - pos)
        out[pos:pos + n] = (start + i % 25) & 0xFF
        i += 1
        pos += n
    return out


def cells_from(buf: np.ndarray, k: int, C: int) -> np.ndarray:
    """Split a user buffer into k cells of C bytes (zero padded), one stripe."""
    out = np.zeros((k, C), dtype=np.uint8)
    flat = out.reshape(-1)
    n = min(buf.size, flat.size)
    flat[:n] = buf[:n]
    return out


CASES = [
    # name, k, p, C, input builder
    ("agg_fill_j_2p1_32k", 2, 1, 32768, lambda k, C: np.repeat(np.arange(k, dtype=np.uint8)[:, None], C, 1)),
    ("agg_fill_80_4p2_32k", 4, 2, 32768, lambda k, C: np.full((k, C), 0x80, dtype=np.uint8)),
    ("agg_fill_j_8p2_32k", 8, 2, 32768, lambda k, C: np.repeat(np.arange(k, dtype=np.uint8)[:, None], C, 1)),
    ("mkbuf_a_933_4p2", 4, 2, 256, lambda k, C: cells_from(make_buffer(ord("a"), 933), k, C)),
    ("mkbuf_b_8569_8p3", 8, 3, 1072, lambda k, C: cells_from(make_buffer(ord("b"), 8569), k, C)),
    ("mkbuf_b_37_2p2", 2, 2, 24, lambda k, C: cells_from(make_buffer(ord("b"), 37), k, C)),
    ("iod3_311x3_4p1", 4, 1, 311 * 3, lambda k, C: cells_from(make_buffer(ord("c"), 4 * 311 * 3), k, C)),
    ("mkbuf_16p3_4k", 16, 3, 4096, lambda k, C: cells_from(make_buffer(ord("d"), 16 * 4096), k, C)),
    ("rand_16p2_4097", 16, 2, 4097, lambda k, C: np.random.default_rng(7).integers(0, 256, (k, C), dtype=np.uint8)),
    ("rand_8p1_1000", 8, 1, 1000, lambda k, C: np.random.default_rng(8).integers(0, 256, (k, C), dtype=np.uint8)),
    ("rand_4p3_4096", 4, 3, 4096, lambda k, C: np.random.default_rng(9).integers(0, 256, (k, C), dtype=np.uint8)),
    ("rand_16p1_333", 16, 1, 333, lambda k, C: np.random.default_rng(10).integers(0, 256, (k, C), dtype=np.uint8)),
]


def main() -> None:
    out = {}
    for name, k, p, C, mk in CASES:
        data = mk(k, C)
        en = ref.cauchy1(k, p)
        assert np.array_equal(en, gf_np.cauchy1(k, p))
        par = ref.encode_data(en[k:], data)
        assert np.array_equal(par, gf_np.matmul_cells(en[k:], data)), name
        out[f"{name}/data"] = data
        out[f"{name}/parity"] = par
        out[f"{name}/kp"] = np.array([k, p], dtype=np.int32)
    path = os.path.join(os.path.dirname(__file__), "fixtures.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {len(CASES)} cases, {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
