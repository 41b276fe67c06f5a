"""The DAOS recovery codec's reuse contract (CPU; no device needed).

The reference keeps one recovery codec per object's fail info
(efi_recov_codec) and returns from obj_ec_recov_codec_init without building
anything when the error list is unchanged (ref:src/object/cli_ec.c:2176-2185,
obj_ec_err_match :2141-2150).  ecg_obj_ec_recov_codec_init does the same;
er_builds counts the builds."""
import ctypes as C

import numpy as np


OC_EC_8P2 = (37 << 24) | 1     # OR_RS_8P2 (ref:src/include/daos_obj_class.h:70-80), one group
OC_EC_4P2 = (35 << 24) | 1


def _init(L, oc, err, rv):
    return L.ecg_obj_ec_recov_codec_init(oc, (C.c_uint32 * len(err))(*err), len(err), rv)


def test_repeat_init_builds_nothing(ecglib, oracle):
    L = ecglib.lib()
    h = L.ecg_obj_ec_recov_codec_alloc()
    try:
        rv = ecglib.RecovCodec.from_address(h)
        k, p = C.c_int(), C.c_int()
        assert L.ecg_obj_ec_class_kp(OC_EC_8P2, C.byref(k), C.byref(p)) == 0 and (k.value, p.value) == (8, 2)
        assert rv.er_builds == 0 and rv.er_nerrs == 0          # zeroed by alloc
        assert _init(L, OC_EC_8P2, [1, 8], h) == 0
        assert rv.er_builds == 1
        rows = bytes(rv.er_de_matrix)
        tbls = bytes(rv.er_gftbls)
        dec = list(rv.er_dec_idx)
        # the rows are the oracle's (the reference's obj_ec_recov_codec_init restated)
        rc, de, odec, _, _, _ = oracle.recov_codec(8, 2, [1, 8])
        assert rc == 0
        assert np.array_equal(np.frombuffer(rows, np.uint8)[:2 * 8].reshape(2, 8), de)
        assert dec[:8] == list(odec)
        for _ in range(5):                                      # same erasures: no rebuild
            assert _init(L, OC_EC_8P2, [1, 8], h) == 0
        assert rv.er_builds == 1
        assert bytes(rv.er_de_matrix) == rows and bytes(rv.er_gftbls) == tbls and list(rv.er_dec_idx) == dec
        # another order, another list, another class, fewer erasures: each rebuilds
        assert _init(L, OC_EC_8P2, [8, 1], h) == 0 and rv.er_builds == 2
        assert _init(L, OC_EC_8P2, [8, 1], h) == 0 and rv.er_builds == 2
        assert _init(L, OC_EC_8P2, [0, 3], h) == 0 and rv.er_builds == 3
        assert _init(L, OC_EC_4P2, [0, 3], h) == 0 and rv.er_builds == 4 and rv.k == 4
        assert _init(L, OC_EC_4P2, [0], h) == 0 and rv.er_builds == 5 and rv.er_nerrs == 1
        # a failed init leaves no cached state behind: the next good one builds
        assert _init(L, OC_EC_4P2, [0, 1, 2], h) == -ecglib.DER_DATA_LOSS
        assert _init(L, OC_EC_4P2, [0, 9], h) == -ecglib.DER_INVAL
        assert rv.er_nerrs == 0
        assert _init(L, OC_EC_4P2, [0, 3], h) == 0 and rv.er_builds == 6
    finally:
        L.ecg_obj_ec_recov_codec_free(h)


def test_repeat_init_is_cheap(ecglib):
    """Timing form of the same: 2000 repeat inits of a 16P3 3-erasure codec
    (k^3 GF work per build) take far less than 2000 builds."""
    import time

    L = ecglib.lib()
    oc = (42 << 24) | 1                                        # OR_RS_16P3
    h = L.ecg_obj_ec_recov_codec_alloc()
    h2 = L.ecg_obj_ec_recov_codec_alloc()
    try:
        err_a, err_b = [0, 5, 17], [1, 6, 18]
        t0 = time.perf_counter()
        for _ in range(2000):
            _init(L, oc, err_a, h)
        cached = time.perf_counter() - t0
        t0 = time.perf_counter()
        for i in range(2000):
            _init(L, oc, err_a if i % 2 else err_b, h2)         # alternating: every call rebuilds
        built = time.perf_counter() - t0
        assert ecglib.RecovCodec.from_address(h).er_builds == 1
        assert ecglib.RecovCodec.from_address(h2).er_builds == 2000
        assert cached < built, (cached, built)
    finally:
        L.ecg_obj_ec_recov_codec_free(h)
        L.ecg_obj_ec_recov_codec_free(h2)
