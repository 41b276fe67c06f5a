"""CPU oracle checks (no GPU): pin the oracle before trusting it.

1. KATs of SURVEY.md App. A.5 (tests/golden/kat.json, hand-entered).
2. Two independent restatements agree: oracle/ec_ref.c (log/exp tables) vs
   oracle/gf_np.py (carry-less multiply + product table).
3. The committed fixtures (reference data patterns) reproduce.
4. The SIMD CPU baseline (AVX2 / GFNI) is byte-identical to the scalar oracle.
5. The DAOS recovery logic restores data for every erasure set <= p.
"""
import itertools
import json
import os

import numpy as np
import pytest

from oracle import gf_np

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CLASSES = [(2, 1), (2, 2), (4, 1), (4, 2), (8, 1), (8, 2), (16, 1), (16, 2), (4, 3), (8, 3), (16, 3)]


def _hex_rows(rows):
    return [bytes.fromhex(r.replace(" ", "")) for r in rows]


def test_kat_field(oracle):
    kat = json.load(open(os.path.join(GOLD, "kat.json")))
    for a, want in kat["gf_inv"].items():
        assert oracle.gf_inv(int(a)) == int(want, 16)
        assert gf_np.gf_inv(int(a)) == int(want, 16)
    for a, b, want in kat["gf_mul"]:
        assert oracle.gf_mul(a, b) == int(want, 16)


def test_kat_cauchy_rows(oracle):
    kat = json.load(open(os.path.join(GOLD, "kat.json")))
    for kp, rows in kat["cauchy_parity_rows"].items():
        k, p = map(int, kp.split(","))
        m = oracle.cauchy1(k, p)
        assert [bytes(r) for r in m[k:]] == _hex_rows(rows)
        assert np.array_equal(m[:k], np.eye(k, dtype=np.uint8))


def test_kat_const_cells(oracle):
    kat = json.load(open(os.path.join(GOLD, "kat.json")))["const_cell_parity"]
    for kp, want in kat.items():
        if kp.startswith("_"):
            continue
        k, p = map(int, kp.split(","))
        cells = np.array([[j + 1] * 100 for j in range(k)], dtype=np.uint8)
        par = oracle.encode_data(oracle.cauchy1(k, p)[k:], cells)
        for r in range(p):
            assert set(par[r].tolist()) == {int(want[r], 16)}


def test_field_tables_agree(oracle):
    tbl = np.array([[oracle.gf_mul(a, b) for b in range(256)] for a in range(256)], dtype=np.uint8)
    assert np.array_equal(tbl, gf_np.MUL)
    inv = np.array([oracle.gf_inv(a) for a in range(256)], dtype=np.uint8)
    assert np.array_equal(inv, gf_np.INV)


@pytest.mark.parametrize("k,p", CLASSES)
def test_cauchy_and_encode_agree(oracle, k, p):
    en = oracle.cauchy1(k, p)
    assert np.array_equal(en, gf_np.cauchy1(k, p))
    rng = np.random.default_rng(k * 100 + p)
    for n in (1, 15, 16, 33, 257, 1000):
        cells = rng.integers(0, 256, (k, n), dtype=np.uint8)
        want = gf_np.matmul_cells(en[k:], cells)
        assert np.array_equal(oracle.encode_data(en[k:], cells), want)
        assert np.array_equal(oracle.encode_data(en[k:], cells, simd=True), want)


def test_init_tables_layout(oracle):
    coef = np.arange(256, dtype=np.uint8).reshape(16, 16)
    t = oracle.init_tables(coef).reshape(256, 32)
    for i, c in enumerate(range(256)):
        assert list(t[i, :16]) == [gf_np.gf_mul(c, n) for n in range(16)]
        assert list(t[i, 16:]) == [gf_np.gf_mul(c, n << 4) for n in range(16)]


def test_invert(oracle):
    rng = np.random.default_rng(3)
    for n in (1, 2, 5, 16):
        for _ in range(5):
            m = rng.integers(0, 256, (n, n), dtype=np.uint8)
            a = oracle.invert(m)
            b = gf_np.invert(m)
            assert (a is None) == (b is None)
            if a is not None:
                assert np.array_equal(a, b)
                assert np.array_equal(gf_np.matmul_cells(m, a), np.eye(n, dtype=np.uint8))
    assert oracle.invert(np.zeros((3, 3), dtype=np.uint8)) is None


def test_update_and_xor(oracle):
    rng = np.random.default_rng(5)
    k, p, n = 8, 3, 777
    en = oracle.cauchy1(k, p)
    data = rng.integers(0, 256, (k, n), dtype=np.uint8)
    par = oracle.encode_data(en[k:], data)
    new = rng.integers(0, 256, n, dtype=np.uint8)
    delta = np.zeros(n, dtype=np.uint8)
    assert oracle.xor_gen([data[3].copy(), new.copy(), delta]) == 0
    assert np.array_equal(delta, data[3] ^ new)
    upd = oracle.encode_data_update(en[k:], 3, delta, par)
    data[3] = new
    assert np.array_equal(upd, oracle.encode_data(en[k:], data))
    assert oracle.xor_gen([data[0].copy(), delta]) != 0  # < 2 sources


@pytest.mark.parametrize("k,p", CLASSES)
def test_recovery_all_patterns(oracle, k, p):
    rng = np.random.default_rng(k + 17 * p)
    n = 64
    en = oracle.cauchy1(k, p)
    data = rng.integers(0, 256, (k, n), dtype=np.uint8)
    stripe = np.concatenate([data, oracle.encode_data(en[k:], data)])
    pats = [c for e in range(1, p + 1) for c in itertools.combinations(range(k + p), e)]
    if len(pats) > 200:
        pats = [pats[i] for i in rng.choice(len(pats), 200, replace=False)]
    for pat in pats:
        rc, de, dec, el, gt, reused = oracle.recov_codec(k, p, list(pat))
        assert rc == 0
        if reused:      # all parity lost: plain re-encode (ref:src/object/cli_ec.c:2205-2210)
            out = oracle.encode_data(en[k:], stripe[:k])
        else:
            out = oracle.encode_data(de, stripe[dec])
        for i, e in enumerate(el):
            assert np.array_equal(out[i], stripe[e]), (pat, e)
        # numpy restatement builds the same rows
        rows, dec2, reused2 = gf_np.recov_matrix(k, p, list(pat))
        assert reused2 == reused
        if not reused:
            assert np.array_equal(rows, de)
            assert list(dec2) == list(dec)


def test_recovery_too_many(oracle):
    rc, *_ = oracle.recov_codec(4, 2, [0, 1, 2])
    assert rc == -2026


def test_reference_quirk_parity_first(oracle):
    """ref:src/object/cli_ec.c:2226-2243 indexes the inverse with the first
    er_data_nerrs entries of the insertion-ordered err_list.  With a parity
    cell listed first, that row index is >= k: the reference reads a row of
    its zero-filled (k+p) x k inverse buffer beyond the k x k that
    gf_invert_matrix wrote (:1963-1984, :2223), so the parity cell it writes
    is ALL ZERO BYTES, while the data cells listed later are still right
    (their rows come from enc[e] * inv == inv[e] for e < k)."""
    k, p = 4, 2
    rng = np.random.default_rng(1)
    en = oracle.cauchy1(k, p)
    data = rng.integers(0, 256, (k, 32), dtype=np.uint8)
    stripe = np.concatenate([data, oracle.encode_data(en[k:], data)])
    rc, de, dec, el, gt, reused = oracle.recov_codec(k, p, [5, 0])
    assert rc == 0 and not reused
    assert not de[0].any()                          # the misindexed decode row is zeros
    out = oracle.encode_data(de, stripe[dec])
    assert np.array_equal(out[1], stripe[0])        # data cell recovered
    assert not out[0].any()                         # the reference's parity cell: zeros
    assert stripe[5].any()                          # ... which is not the true parity
    # k=4, p=3: {4, 5, 0} and {4, 0, 1}: exactly the parity cells among the first
    # er_data_nerrs entries come out zero, every other cell is right
    en3 = oracle.cauchy1(4, 3)
    stripe3 = np.concatenate([data, oracle.encode_data(en3[4:], data)])
    for errs, zero in (([4, 5, 0], {0}), ([4, 0, 1], {0}), ([5, 6, 1], {0}), ([0, 4, 1], {1}), ([0, 1, 4], set())):
        rc, de, dec, el, gt, reused = oracle.recov_codec(4, 3, errs)
        assert rc == 0 and not reused
        out = oracle.encode_data(de, stripe3[dec])
        for i, e in enumerate(el):
            if i in zero:
                assert not out[i].any(), (errs, e)
            else:
                assert np.array_equal(out[i], stripe3[e]), (errs, e)


def test_fixtures_reproduce(oracle):
    fx = np.load(os.path.join(GOLD, "fixtures.npz"))
    names = sorted({n.split("/")[0] for n in fx.files})
    assert len(names) >= 10
    for name in names:
        k, p = fx[f"{name}/kp"]
        data = fx[f"{name}/data"]
        en = oracle.cauchy1(int(k), int(p))
        assert np.array_equal(oracle.encode_data(en[k:], data), fx[f"{name}/parity"]), name


def test_batch_helpers(oracle):
    k, p, C, S = 4, 2, 4096, 8
    rng = np.random.default_rng(2)
    data = rng.integers(0, 256, S * k * C, dtype=np.uint8)
    par = oracle.encode_batch(k, p, C, S, data, nthreads=2)
    par2 = oracle.encode_batch(k, p, C, S, data, nthreads=2, simd=True)
    assert np.array_equal(par, par2)
    d = data.reshape(S, k, C)
    en = oracle.cauchy1(k, p)
    for s in range(S):
        assert np.array_equal(par.reshape(p, S, C)[:, s], oracle.encode_data(en[k:], d[s]))


def test_singv_cell_bytes(oracle):
    # obj_ec_singv_cell_bytes: ceil(size / k) rounded up to 8 (ref:src/object/obj_ec.h:421-434)
    assert oracle.singv_cell_bytes(8569, 2) == 4288
    assert oracle.singv_cell_bytes(8569, 4) == 2144
    assert oracle.singv_cell_bytes(8569, 16) == 536
    assert oracle.singv_cell_bytes(4096, 4) == 1024


def test_agg_diff_preprocess_rules(oracle):
    """Restatement of ref:src/object/srv_ec_aggregate.c:1006-1058 on a cell of
    8 records x 4 bytes (cell index 1 = records 8..15)."""
    d = np.full(32, 0xFF, np.uint8)
    out = oracle.agg_diff_preprocess(d, 8, 4, 1, [(9, 2), (13, 1)]).reshape(8, 4)[:, 0]
    assert list(out) == [0, 255, 255, 0, 0, 255, 0, 0]
    # no extent touches the cell: nothing zeroed (hole_off stays 0)
    assert (oracle.agg_diff_preprocess(d, 8, 4, 1, [(0, 4)]) == 0xFF).all()
    # extent running past the cell end: no tail zeroing
    out = oracle.agg_diff_preprocess(d, 8, 4, 1, [(12, 10)]).reshape(8, 4)[:, 0]
    assert list(out) == [0, 0, 0, 0, 255, 255, 255, 255]
