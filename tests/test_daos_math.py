"""Stripe / index math of the DAOS codec surface (ref:src/object/obj_ec.h:271-350),
host-only: the exported functions against the macros restated here, and the
round-trip property the reference relies on (daos idx -> (target, VOS idx) ->
daos idx) for every record of several stripes."""
import numpy as np
import pytest


def _ref(name, *a):
    """The obj_ec.h macros, restated."""
    if name == "stripe_rec_nr":
        k, e_len = a
        return k * e_len
    if name == "tgt_of_recx_idx":
        idx, srn, e_len = a
        return (idx % srn) // e_len
    if name == "daos2vos":
        idx, srn, e_len = a
        return (idx // srn) * e_len + idx % e_len
    if name == "vos2daos":
        vos, srn, e_len, tgt = a
        return (vos // e_len) * srn + tgt * e_len + vos % e_len
    if name == "parity2daos":
        off, e_len, srn = a
        return (off // e_len) * srn
    raise KeyError(name)


@pytest.mark.parametrize("k,e_len", [(2, 1), (4, 1024), (8, 1 << 20), (16, 32768), (8, 3)])
def test_index_maps(ecglib, k, e_len):
    L = ecglib.lib()
    srn = L.ecg_obj_ec_stripe_rec_nr(k, e_len)
    assert srn == _ref("stripe_rec_nr", k, e_len)
    rng = np.random.default_rng(k * 7 + e_len)
    idxs = list(rng.integers(0, 50 * srn, 400, dtype=np.uint64)) + [0, srn - 1, srn, 7 * srn + e_len]
    for idx in map(int, idxs):
        tgt = L.ecg_obj_ec_tgt_of_recx_idx(idx, srn, e_len)
        vos = L.ecg_obj_ec_idx_daos2vos(idx, srn, e_len)
        assert tgt == _ref("tgt_of_recx_idx", idx, srn, e_len) and tgt < k
        assert vos == _ref("daos2vos", idx, srn, e_len)
        back = L.ecg_obj_ec_idx_vos2daos(vos, srn, e_len, tgt)
        assert back == _ref("vos2daos", vos, srn, e_len, tgt) == idx      # round trip
        # parity cell of the same stripe: VOS offset vos maps back to the stripe start
        assert L.ecg_obj_ec_idx_parity2daos(vos, e_len, srn) == (idx // srn) * srn


def test_cell_bytes_and_shard_off(ecglib):
    L = ecglib.lib()
    assert L.ecg_obj_ec_cell_bytes(1 << 20, 1) == 1 << 20
    assert L.ecg_obj_ec_cell_bytes(32768, 8) == 262144
    for n in (3, 6, 10, 18):
        for start in range(n):
            offs = [L.ecg_obj_ec_shard_off_by_start(t, n, start) for t in range(n)]
            assert sorted(offs) == list(range(n)) and offs[start] == 0      # a rotation
    assert ecglib.lib().ecg_obj_ec_idx_daos2vos(2**63 + 5, 8, 4) == (2**63 + 5) // 8 * 4 + 1
