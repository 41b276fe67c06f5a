"""The drop-in surfaces in a process WITHOUT a GPU (run by
tests/test_cpu_path.py with HIP_VISIBLE_DEVICES=""): ISA-L's ec_encode_data /
ec_encode_data_update / xor_gen and the synchronous DAOS calls must run the
product's CPU path and produce the scalar oracle's bytes -- never abort.
That is every process libdaos runs in on a client node
(ref:src/object/SConscript:19-23, ec_encode_data at ref:src/object/cli_ec.c:540).

Cases: the golden fixtures (tests/golden/fixtures.npz: the reference's own
test patterns and sizes), the reference sizes 4 MiB+347 / 933 / 311x3 /
8569 / 37 bytes (ref:src/tests/suite/daos_rebuild_common.c:654-658), odd
alignments, every DAOS class.  Prints one JSON line; exit status 0 = pass.
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)

from daos_amd import ecg  # noqa: E402
from oracle import ref  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden", "fixtures.npz")
CLASSES = [(2, 1), (2, 2), (4, 1), (4, 2), (8, 1), (8, 2), (16, 1), (16, 2), (4, 3), (8, 3), (16, 3)]
OC_ID = {(2, 1): 32, (2, 2): 33, (4, 1): 34, (4, 2): 35, (8, 1): 36, (8, 2): 37, (16, 1): 38, (16, 2): 39,
         (4, 3): 40, (8, 3): 41, (16, 3): 42}


def rand(shape, seed):
    return np.random.default_rng(seed).integers(0, 256, shape, dtype=np.uint8)


def offset_views(arrs, off):
    """Copies of arrs at byte offset `off` of a fresh buffer (any alignment)."""
    out = []
    for a in arrs:
        b = np.zeros(a.size + 64, dtype=np.uint8)
        v = b[off: off + a.size]
        v[:] = a
        out.append(v)
    return out


def main():
    L = ecg.lib()
    kernels = set()
    n = 0
    assert ecg.device_count() == 0, "run with HIP_VISIBLE_DEVICES=''"

    # golden fixtures through ec_encode_data
    fx = np.load(GOLD)
    for name in sorted({f.split("/")[0] for f in fx.files}):
        k, p = (int(x) for x in fx[f"{name}/kp"])
        data, want = fx[f"{name}/data"], fx[f"{name}/parity"]
        tb = ecg.isal_init_tables(ref.cauchy1(k, p)[k:])
        out = [np.zeros(data.shape[1], dtype=np.uint8) for _ in range(p)]
        ecg.isal_encode_data(tb, k, p, list(data), out)
        assert np.array_equal(np.stack(out), want), name
        kernels.add(ecg.last_kernel())
        n += 1

    # every class at the reference sizes, odd offsets, vs the scalar oracle
    sizes = [4 * 1024 * 1024 + 347, 933, 311 * 3, 8569, 37, 32768, 1]
    for ci, (k, p) in enumerate(CLASSES):
        en = ref.cauchy1(k, p)
        tb = ecg.isal_init_tables(en[k:])
        for si, ln in enumerate(sizes):
            if ln > 1 << 20 and ci % 4:
                continue                     # the 4 MiB value on every 4th class keeps this fast
            off = (ci + si) % 7
            data = offset_views([rand(ln, 1000 + 31 * ci + si + j) for j in range(k)], off)
            coding = offset_views([np.zeros(ln, dtype=np.uint8) for _ in range(p)], (off * 3) % 5)
            ecg.isal_encode_data(tb, k, p, data, coding)
            want = ref.encode_data(en[k:], np.stack(data))
            assert np.array_equal(np.stack(coding), want), (k, p, ln)
            # ec_encode_data_update of one cell
            vi = (si * 5) % k
            delta = rand(ln, 77 + si)
            ecg.isal_encode_data_update(tb, k, p, vi, delta, coding)
            want = ref.encode_data_update(en[k:], vi, delta, want)
            assert np.array_equal(np.stack(coding), want), ("update", k, p, ln)
            kernels.add(ecg.last_kernel())
            n += 2

    # xor_gen: 3 vectors (agg_update_parity's diff), and more than 64 sources
    for nv, ln in ((3, 32768 + 3), (3, 37), (70, 4099), (321, 512)):
        arrs = [rand(ln, 500 + i) for i in range(nv - 1)] + [np.zeros(ln, dtype=np.uint8)]
        want = arrs[0].copy()
        assert ref.xor_gen([a.copy() for a in arrs[:-1]] + [want]) == 0
        assert ecg.isal_xor_gen(arrs) == 0
        assert np.array_equal(arrs[-1], want), ("xor_gen", nv, ln)
        n += 1

    # DAOS surface, no context: obj_ec_encode_buf, recovery, stripes, aggregation, single value
    assert L.ecg_obj_ec_codec_init() == 0
    k, p, cell = 8, 2, 65536 + 8
    oc = (OC_ID[(k, p)] << 24) | 1
    buf = rand(k * cell, 70)
    pbufs = (ecg.u8p * p)()
    assert L.ecg_obj_ec_encode_buf(oc, cell, buf.ctypes.data_as(ecg.u8p), pbufs) == 0
    par = np.stack([np.ctypeslib.as_array(pbufs[r], shape=(cell,)).copy() for r in range(p)])
    libc = C.CDLL(None)
    for r in range(p):
        libc.free(C.cast(pbufs[r], C.c_void_p))
    assert np.array_equal(par, ref.encode_data(ref.cauchy1(k, p)[k:], buf.reshape(k, cell)))
    n += 1

    S = 3
    data = rand((S, k, cell), 71)
    parity = np.zeros((p, S, cell), dtype=np.uint8)
    assert L.ecg_obj_ec_encode_stripes(None, oc, cell, S, data.ctypes.data_as(ecg.u8p),
                                       parity.ctypes.data_as(ecg.u8p)) == 0
    en = ref.cauchy1(k, p)
    for s in range(S):
        assert np.array_equal(parity[:, s], ref.encode_data(en[k:], data[s])), s
    stripes = np.concatenate([data, parity.transpose(1, 0, 2)], axis=1).copy()
    for err in ([1, 9], [0, 1], [8, 9], [5]):
        broken = stripes.copy()
        broken[:, err] = 0xA5
        rv = L.ecg_obj_ec_recov_codec_alloc()
        assert L.ecg_obj_ec_recov_codec_init(oc, (C.c_uint32 * len(err))(*err), len(err), rv) == 0
        assert L.ecg_obj_ec_recov_data(None, rv, cell, broken.ctypes.data_as(ecg.u8p), S) == 0
        L.ecg_obj_ec_recov_codec_free(rv)
        assert np.array_equal(broken, stripes), err
        n += 1

    old = data[0, [1, 3]].copy()
    new = rand((2, cell), 81)
    par0 = stripes[0, k:].copy()
    bm = np.array([0b1010], dtype=np.uint8)
    assert L.ecg_agg_update_parity(None, oc, cell, 1, bm.ctypes.data_as(ecg.u8p), 2, old.ctypes.data_as(ecg.u8p),
                                   new.ctypes.data_as(ecg.u8p), None, None, 0, par0.ctypes.data_as(ecg.u8p)) == 0
    d2 = data[0].copy()
    d2[[1, 3]] = new
    assert np.array_equal(par0, ref.encode_data(en[k:], d2))
    rbuf, lbuf = rand((4, cell), 93), rand((4, cell), 94)
    par1 = np.zeros((p, cell), dtype=np.uint8)
    bm = np.array([0b10010110], dtype=np.uint8)
    assert L.ecg_agg_recalc_parity(None, oc, cell, bm.ctypes.data_as(ecg.u8p), 4, rbuf.ctypes.data_as(ecg.u8p),
                                   lbuf.ctypes.data_as(ecg.u8p), par1.ctypes.data_as(ecg.u8p)) == 0
    mix = np.stack([rbuf[[1, 2, 4, 7].index(j)] if j in (1, 2, 4, 7) else lbuf[[0, 3, 5, 6].index(j)]
                    for j in range(k)])
    assert np.array_equal(par1, ref.encode_data(en[k:], mix))
    for (kk, pp), size in (((4, 2), 8569), ((16, 3), 933), ((2, 1), 37)):
        value = rand(size, 95 + size)
        cb = ref.singv_cell_bytes(size, kk)
        pb = [np.zeros(cb, dtype=np.uint8) for _ in range(pp)]
        pbp = (ecg.u8p * pp)(*[a.ctypes.data_as(ecg.u8p) for a in pb])
        assert L.ecg_obj_ec_singv_encode((OC_ID[(kk, pp)] << 24) | 1, size, value.ctypes.data_as(ecg.u8p), pbp) == 0
        assert np.array_equal(np.stack(pb), ref.singv_encode(kk, pp, value)), (kk, pp, size)
    n += 5
    kernels.add(ecg.last_kernel())
    assert all(x.startswith("cpu:") for x in kernels), kernels
    print(json.dumps({"ok": True, "cases": n, "kernels": sorted(kernels), "isa": ecg.cpu_isa()}))


if __name__ == "__main__":
    main()
