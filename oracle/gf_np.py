"""Second, independent CPU restatement of the EC codec math (numpy).

TEST INFRASTRUCTURE ONLY -- imported by tests/ and bench.py's cpu_baseline leg,
never by the product (daos_amd/).

It shares no code with oracle/ec_ref.c: the field is built here by carry-less
multiplication + reduction (not log/exp walking), encode uses a full 256x256
product table, and matrix inversion is a separate Gauss-Jordan.  The two
oracles must agree byte for byte (tests/test_oracle.py); parity of both is
"unpinned" by reference fixtures (none exist for this path -- see
oracle/ec_ref.h), and pinned to the KATs of SURVEY.md App. A.5.

Reference behaviour restated:
  gf_gen_cauchy1_matrix      ref:src/object/obj_class.c:614 (ISA-L, external)
  ec_encode_data             ref:src/object/cli_ec.c:540,571,2641
  obj_ec_recov_codec_init    ref:src/object/cli_ec.c:2152-2250
"""
from __future__ import annotations

import numpy as np

POLY = 0x11D


def _clmul_reduce(a: int, b: int) -> int:
    r = 0
    for i in range(8):
        if (b >> i) & 1:
            r ^= a << i
    for bit in range(15, 7, -1):
        if (r >> bit) & 1:
            r ^= POLY << (bit - 8)
    return r


MUL = np.array([[_clmul_reduce(a, b) for b in range(256)] for a in range(256)], dtype=np.uint8)
INV = np.zeros(256, dtype=np.uint8)
for _a in range(1, 256):
    INV[_a] = int(np.nonzero(MUL[_a] == 1)[0][0])


def gf_mul(a: int, b: int) -> int:
    return int(MUL[a, b])


def gf_inv(a: int) -> int:
    return int(INV[a])


def cauchy1(k: int, p: int) -> np.ndarray:
    """(k+p) x k: identity, then 1/(i ^ j) for parity rows i in [k, k+p)."""
    m = np.zeros((k + p, k), dtype=np.uint8)
    m[:k, :k] = np.eye(k, dtype=np.uint8)
    for i in range(k, k + p):
        for j in range(k):
            m[i, j] = INV[i ^ j]
    return m


def matmul_cells(coef: np.ndarray, cells: np.ndarray) -> np.ndarray:
    """coef [rows, k] (uint8) x cells [k, n] (uint8) -> [rows, n] over GF(2^8)."""
    rows, k = coef.shape
    out = np.zeros((rows, cells.shape[1]), dtype=np.uint8)
    for r in range(rows):
        acc = np.zeros(cells.shape[1], dtype=np.uint8)
        for j in range(k):
            acc ^= MUL[int(coef[r, j])][cells[j]]
        out[r] = acc
    return out


def invert(mat: np.ndarray) -> np.ndarray | None:
    n = mat.shape[0]
    a = mat.copy()
    out = np.eye(n, dtype=np.uint8)
    for c in range(n):
        piv = next((r for r in range(c, n) if a[r, c]), None)
        if piv is None:
            return None
        if piv != c:
            a[[c, piv]] = a[[piv, c]]
            out[[c, piv]] = out[[piv, c]]
        s = int(INV[int(a[c, c])])
        a[c] = MUL[s][a[c]]
        out[c] = MUL[s][out[c]]
        for r in range(n):
            if r != c and a[r, c]:
                f = int(a[r, c])
                a[r] ^= MUL[f][a[c]]
                out[r] ^= MUL[f][out[c]]
    return out


def recov_matrix(k: int, p: int, err_list: list[int]):
    """DAOS decode-matrix build (ref:src/object/cli_ec.c:2152-2250).

    Returns (rows [nerrs, k], dec_idx [k], reused_encode) with rows in err_list
    order, following the reference's data-errors-first indexing.
    """
    if len(err_list) > p:
        raise ValueError("DER_DATA_LOSS")
    enc = cauchy1(k, p)
    data_nerrs = sum(1 for e in err_list if e < k)
    if data_nerrs == 0 and len(err_list) == p:
        return enc[k:].copy(), None, True
    alive = [i for i in range(k + p) if i not in set(err_list)][:k]
    inv = invert(enc[alive])
    rows = np.zeros((len(err_list), k), dtype=np.uint8)
    for i in range(data_nerrs):
        rows[i] = inv[err_list[i]]
    for e in range(data_nerrs, len(err_list)):
        # enc[e] * inv : sum_j enc[e][j] * inv[j][i]
        rows[e] = matmul_cells(enc[err_list[e]][None, :], inv)[0]
    return rows, np.array(alive, dtype=np.uint32), False
