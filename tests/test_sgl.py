"""Degraded-read byte movement without a GPU: the stripe list built by the
C library (ecg_obj_ec_stripe_list_init, obj_ec_stripe_list_init/_add,
ref:src/object/cli_ec.c:2252-2381) against the Python restatement, and the
fill-back restatement (oracle/sgl_py.py, obj_ec_recov_fill_back,
ref:src/object/cli_ec.c:2710-2812) against what a degraded read must
return: the object's bytes at the recovered records' places in the user's
scatter-gather list, nothing else touched."""
import ctypes as ct

import numpy as np
import pytest

from oracle import sgl_py
from tests.sgl_cases import expected_user_bytes, make_case, stripe_image


def c_stripe_list(ecglib, srn, items):
    arr = (ecglib.RecxEp * max(1, len(items)))(
        *[ecglib.RecxEp(ecglib.Recx(r["idx"], r["nr"]), r["ep"], 1, r["type"]) for r in items])
    out = (ecglib.RecxEp * max(1, len(items)))()
    n = ct.c_uint32()
    rc = ecglib.lib().ecg_obj_ec_stripe_list_init(srn, arr, len(items), out, len(items), ct.byref(n))
    assert rc == 0
    return [{"idx": out[i].re_recx.rx_idx, "nr": out[i].re_recx.rx_nr, "ep": out[i].re_ep,
             "type": out[i].re_type} for i in range(n.value)]


@pytest.mark.parametrize("seed", range(12))
def test_stripe_list_matches_oracle(ecglib, seed):
    rng = np.random.default_rng(seed)
    srn = int(rng.choice([8, 24, 64 * 3]))
    items = []
    for _ in range(int(rng.integers(1, 14))):
        idx = int(rng.integers(0, 20 * srn))
        items.append({"idx": idx, "nr": int(rng.integers(1, 3 * srn)), "ep": int(rng.integers(1, 4)),
                      "type": int(rng.choice([1, 2, 2, 2]))})
    want = sgl_py.stripe_list_init(srn, items)
    got = c_stripe_list(ecglib, srn, items)
    assert got == [{k: v for k, v in w.items()} for w in want]
    for s in got:                               # whole stripes, every shadow record covered
        assert s["idx"] % srn == 0 and s["nr"] % srn == 0
    for r in items:
        if r["type"] == 2:
            assert any(s["idx"] <= r["idx"] and r["idx"] + r["nr"] <= s["idx"] + s["nr"] for s in got)


def test_stripe_list_merge_rules(ecglib):
    """Adjacent entries merge only at equal epochs; overlapping ones merge
    and keep the higher epoch (ref:src/object/cli_ec.c:2264-2305)."""
    S = 8
    items = [{"idx": 0, "nr": 3, "ep": 1, "type": 2}, {"idx": 9, "nr": 2, "ep": 1, "type": 2},
             {"idx": 17, "nr": 1, "ep": 2, "type": 2}, {"idx": 5, "nr": 1, "ep": 3, "type": 2}]
    got = c_stripe_list(ecglib, S, items)
    assert got == [{"idx": 0, "nr": 16, "ep": 3, "type": 2}, {"idx": 16, "nr": 8, "ep": 2, "type": 2}]
    assert got == sgl_py.stripe_list_init(S, items)


def test_stripe_list_errors(ecglib):
    L = ecglib.lib()
    n = ct.c_uint32()
    arr = (ecglib.RecxEp * 2)(ecglib.RecxEp(ecglib.Recx(0, 1), 1, 1, 2), ecglib.RecxEp(ecglib.Recx(100, 1), 2, 1, 2))
    out = (ecglib.RecxEp * 1)()
    assert L.ecg_obj_ec_stripe_list_init(0, arr, 2, out, 1, ct.byref(n)) == -ecglib.DER_INVAL
    assert L.ecg_obj_ec_stripe_list_init(8, arr, 2, out, 1, ct.byref(n)) == -ecglib.DER_INVAL   # cap
    assert L.ecg_obj_ec_stripe_list_init(8, arr, 1, out, 1, ct.byref(n)) == 0 and n.value == 1


CASES = [  # seed, k, e_len, iod_size, nstripes, n_iod, n_iov, n_recov, zero_iovs, slack
    (1, 4, 64, 1, 6, 3, 5, 4, 0, 0),
    (2, 2, 100, 3, 8, 4, 9, 6, 2, 17),       # iod_size 3 (ref daos_rebuild_common.c IOD3_DATA_SIZE)
    (3, 8, 32, 8, 5, 2, 1, 3, 0, 0),         # one iov
    (4, 16, 16, 5, 4, 5, 31, 7, 3, 1),
    (5, 4, 1024, 1, 3, 1, 4, 2, 0, 0),
]


@pytest.mark.parametrize("case_args", CASES)
def test_fill_back_oracle_semantics(case_args):
    """The restated fill-back puts exactly the recovered records' bytes at
    their user-sgl offsets, and keeps the reference's iov_len / sg_nr_out
    bookkeeping within capacity."""
    case = make_case(*case_args)
    stripes = sgl_py.stripe_list_init(case["srn"], case["recov"])
    p = 2
    img = stripe_image(case, stripes, p)
    sgl = sgl_py.Sgl([np.full(n, 0xEE, np.uint8) for n in case["lens"]])
    C = case["e_len"] * case["iod_size"]
    sgl_py.recov_fill_back(case["iod_size"], case["iod"], sgl, case["recov"], stripes, img, (case["k"] + p) * C,
                           case["srn"])
    got = np.concatenate(sgl.bufs) if sgl.bufs else np.zeros(0, np.uint8)
    assert np.array_equal(got, expected_user_bytes(case))
    assert all(0 <= ln <= len(b) for ln, b in zip(sgl.iov_len, sgl.bufs))
    assert 0 < sgl.nr_out <= len(sgl.bufs)


def test_fill_back_oracle_singv():
    sgl = sgl_py.Sgl([np.zeros(5, np.uint8), np.zeros(0, np.uint8), np.zeros(40, np.uint8)])
    img = np.arange(64, dtype=np.uint8)
    sgl_py.recov_fill_back(37, [], sgl, [], [], img, 64, 8, singv=True)   # 37-byte value (ref :657)
    assert np.array_equal(np.concatenate(sgl.bufs)[:37], img[:37])
    assert sgl.iov_len == [5, 0, 32] and sgl.nr_out == 3


def test_struct_layouts_match_daos(ecglib):
    """ecg_iov_t / ecg_recx_ep_t / ecg_sgl_t are field-for-field d_iov_t,
    struct daos_recx_ep and d_sg_list_t (ref:src/include/gurt/types.h:93-132,
    ref:src/include/daos/object.h:714-719), so DAOS glue casts pointers."""
    assert ct.sizeof(ecglib.Iov) == 24 and ecglib.Iov.iov_len.offset == 16
    assert ct.sizeof(ecglib.Recx) == 16
    assert ct.sizeof(ecglib.RecxEp) == 32 and ecglib.RecxEp.re_ep.offset == 16
    assert ecglib.RecxEp.re_rec_size.offset == 24 and ecglib.RecxEp.re_type.offset == 28
    assert ct.sizeof(ecglib.Sgl) == 16 and ecglib.Sgl.sg_iovs.offset == 8
