"""GPU parity of the degraded-read byte movement: stripes of the stripe list
recovered on the device (ecg_recover), then the fill-back into a device
scatter-gather list (ecg_obj_ec_recov_fill_back, restating
obj_ec_recov_fill_back, ref:src/object/cli_ec.c:2710-2812), against the
Python restatement (oracle/sgl_py.py) -- every byte of every iov, iov_len
and sg_nr_out.  Also the batched copy kernel itself at every source /
destination alignment (single-value fill-back, :2725-2729)."""
import ctypes as ct

import numpy as np
import pytest

from oracle import sgl_py
from tests.sgl_cases import expected_user_bytes, make_case, stripe_image
from tests.test_sgl import CASES, c_stripe_list

pytestmark = pytest.mark.gpu


def device_sgl(ctx, ecglib, rng, lens, fill=0xEE, align=False):
    """iovs of the given capacities inside one device buffer, at gaps and
    (unless align) odd byte offsets; filled with `fill`."""
    offs, pos = [], 0
    for n in lens:
        pos += int(rng.integers(1, 40)) if not align else 64
        if align:
            pos = (pos + 15) & ~15
        offs.append(pos)
        pos += n
    buf = ctx.alloc(pos + 64)
    buf.upload(np.full(pos + 64, fill, np.uint8))
    iovs = (ecglib.Iov * max(1, len(lens)))(*[ecglib.Iov(buf.ptr + o, n, 0) for o, n in zip(offs, lens)])
    sgl = ecglib.Sgl(len(lens), 0, iovs)
    return buf, offs, iovs, sgl


def read_sgl(buf, offs, lens):
    host = buf.download()
    return [host[o:o + n] for o, n in zip(offs, lens)], host


def recx_arrays(ecglib, case, stripes):
    iod = (ecglib.Recx * max(1, len(case["iod"])))(*[ecglib.Recx(a, n) for a, n in case["iod"]])
    rec = (ecglib.RecxEp * max(1, len(case["recov"])))(
        *[ecglib.RecxEp(ecglib.Recx(r["idx"], r["nr"]), r["ep"], case["iod_size"], r["type"]) for r in case["recov"]])
    st = (ecglib.RecxEp * max(1, len(stripes)))(
        *[ecglib.RecxEp(ecglib.Recx(s["idx"], s["nr"]), s["ep"], case["iod_size"], s["type"]) for s in stripes])
    return iod, rec, st


@pytest.mark.parametrize("case_args", CASES + [(6, 8, 512, 8, 6, 4, 12, 9, 1, 64), (7, 2, 4096, 1, 4, 2, 3, 3, 0, 0)])
@pytest.mark.parametrize("lost", [(1, "k"), (0, 1)])
def test_recover_and_fill_back(oracle, ecglib, ctx, case_args, lost):
    case = make_case(*case_args)
    k, p, isz, srn = case["k"], 2, case["iod_size"], case["srn"]
    C = case["e_len"] * isz
    lost = [k if x == "k" else x for x in lost]
    stripes = c_stripe_list(ecglib, srn, case["recov"])
    assert stripes == sgl_py.stripe_list_init(srn, case["recov"])
    en = oracle.cauchy1(k, p)
    img = stripe_image(case, stripes, p, parity_fn=lambda d: oracle.encode_data(en[k:], d))
    nst = img.size // ((k + p) * C)
    broken = img.reshape(nst, k + p, C).copy()
    broken[:, lost] = 0x5A
    rng = np.random.default_rng(case_args[0])
    dimg = ctx.to_device(broken)
    buf, offs, iovs, sgl = device_sgl(ctx, ecglib, rng, case["lens"])
    try:
        ctx.recover(k, p, C, nst, dimg.ptr, (k + p) * C, lost)
        iod, rec, st = recx_arrays(ecglib, case, stripes)
        rc = ecglib.lib().ecg_obj_ec_recov_fill_back(ctx.h, isz, 0, iod, len(case["iod"]), ct.byref(sgl), rec,
                                                     len(case["recov"]), st, len(stripes), dimg.ptr, (k + p) * C,
                                                     srn, None)
        assert rc == 0, ecglib.lib().ecg_strerror()
        ctx.sync()
        assert ecglib.last_kernel() == "ecg_copy_segs_kernel"
        got, host = read_sgl(buf, offs, case["lens"])
        want = sgl_py.Sgl([np.full(n, 0xEE, np.uint8) for n in case["lens"]])
        sgl_py.recov_fill_back(isz, case["iod"], want, case["recov"], stripes, img, (k + p) * C, srn)
        for i, (g, w) in enumerate(zip(got, want.bufs)):
            assert np.array_equal(g, w), i
        assert np.array_equal(np.concatenate(got), expected_user_bytes(case))
        assert [iovs[i].iov_len for i in range(len(case["lens"]))] == want.iov_len
        assert sgl.sg_nr_out == want.nr_out
        gaps = np.ones(host.size, bool)            # nothing outside the iovs was written
        for o, n in zip(offs, case["lens"]):
            gaps[o:o + n] = False
        assert (host[gaps] == 0xEE).all()
    finally:
        buf.free()
        dimg.free()


@pytest.mark.parametrize("src_skew", [0, 1, 3, 4, 7, 8, 13, 15])
def test_copy_kernel_alignments(ecglib, ctx, src_skew):
    """Single-value fill-back = one sgl copy of iod_size bytes: every source
    misalignment against iovs at random byte offsets, lengths from 0 to
    several 16 KiB tiles."""
    rng = np.random.default_rng(src_skew)
    lens = [0, 1, 15, 16, 17, 255, 4096 + 3, 16384, 16384 * 3 + 9, 70001, 2, 31]
    rng.shuffle(lens)
    total = sum(lens)
    src_host = rng.integers(0, 256, total + 64, dtype=np.uint8)
    src = ctx.to_device(src_host)
    buf, offs, iovs, sgl = device_sgl(ctx, ecglib, rng, lens, fill=0x11)
    try:
        rc = ecglib.lib().ecg_obj_ec_recov_fill_back(ctx.h, total - 5, 1, None, 0, ct.byref(sgl), None, 0, None, 0,
                                                     src.ptr + src_skew, 0, 1, None)
        assert rc == 0, ecglib.lib().ecg_strerror()
        ctx.sync()
        got, host = read_sgl(buf, offs, lens)
        want = sgl_py.Sgl([np.full(n, 0x11, np.uint8) for n in lens])
        sgl_py.recov_fill_back(total - 5, [], want, [], [], src_host[src_skew:], 0, 1, singv=True)
        for g, w in zip(got, want.bufs):
            assert np.array_equal(g, w)
        assert [iovs[i].iov_len for i in range(len(lens))] == want.iov_len
        assert sgl.sg_nr_out == want.nr_out
    finally:
        buf.free()
        src.free()


def test_fill_back_errors(ecglib, ctx):
    L = ecglib.lib()
    buf = ctx.alloc(4096)
    iovs = (ecglib.Iov * 1)(ecglib.Iov(buf.ptr, 4096, 0))
    sgl = ecglib.Sgl(1, 0, iovs)
    iod = (ecglib.Recx * 1)(ecglib.Recx(10, 100))
    st = (ecglib.RecxEp * 1)(ecglib.RecxEp(ecglib.Recx(0, 64), 1, 1, 2))
    try:
        bad_rec = (ecglib.RecxEp * 1)(ecglib.RecxEp(ecglib.Recx(70, 10), 1, 1, 2))   # beyond the stripe list
        assert L.ecg_obj_ec_recov_fill_back(ctx.h, 1, 0, iod, 1, ct.byref(sgl), bad_rec, 1, st, 1, buf.ptr, 128, 64,
                                            None) == -ecglib.DER_INVAL
        st2 = (ecglib.RecxEp * 1)(ecglib.RecxEp(ecglib.Recx(0, 60), 1, 1, 2))          # not whole stripes
        ok_rec = (ecglib.RecxEp * 1)(ecglib.RecxEp(ecglib.Recx(20, 10), 1, 1, 2))
        assert L.ecg_obj_ec_recov_fill_back(ctx.h, 1, 0, iod, 1, ct.byref(sgl), ok_rec, 1, st2, 1, buf.ptr, 128, 64,
                                            None) == -ecglib.DER_INVAL
        early = (ecglib.RecxEp * 1)(ecglib.RecxEp(ecglib.Recx(5, 10), 1, 1, 2))           # starts before iod recx
        assert L.ecg_obj_ec_recov_fill_back(ctx.h, 1, 0, iod, 1, ct.byref(sgl), early, 1, st, 1, buf.ptr, 128, 64,
                                            None) == -ecglib.DER_INVAL
        assert L.ecg_obj_ec_recov_fill_back(ctx.h, 1, 0, iod, 1, ct.byref(sgl), ok_rec, 1, st, 1, buf.ptr, 128, 64,
                                            None) == 0
        ctx.sync()
    finally:
        buf.free()


def test_recov_data_dev_iods(oracle, ecglib, ctx):
    """obj_ec_recov_data over three iods in one call: an array iod (stripe
    list, fill-back into a scattered sgl), an evenly distributed single
    value (one stripe of obj_ec_singv_cell_bytes cells), and a short single
    value stored on one target (no recovery, only the copy)."""
    L = ecglib.lib()
    k, p = 4, 2
    oc = (35 << 24) | 1
    case = make_case(11, k, 256, 2, 6, 3, 7, 5, 1, 3)
    isz, srn = case["iod_size"], case["srn"]
    C = case["e_len"] * isz
    lost = [1, k]
    en = oracle.cauchy1(k, p)
    rng = np.random.default_rng(11)
    stripes = c_stripe_list(ecglib, srn, case["recov"])
    img = stripe_image(case, stripes, p, parity_fn=lambda d: oracle.encode_data(en[k:], d))
    nst = img.size // ((k + p) * C)
    broken = img.reshape(nst, k + p, C).copy()
    broken[:, lost] = 0
    # evenly distributed single value: 100 000 bytes -> 4 cells of 25 000 (last one padded)
    sv = rng.integers(0, 256, 100000, dtype=np.uint8)
    scell = L.ecg_obj_ec_singv_cell_bytes(oc, sv.size)
    cells = np.zeros(k * scell, np.uint8)
    cells[:sv.size] = sv
    simg = np.concatenate([cells, oracle.encode_data(en[k:], cells.reshape(k, scell)).reshape(-1)])
    sbroken = simg.reshape(k + p, scell).copy()
    sbroken[lost] = 0
    # short single value: lives on one target, the buffer already holds it
    small = rng.integers(0, 256, 1000, dtype=np.uint8)
    codec = L.ecg_obj_ec_recov_codec_alloc()
    dimg, dsv, dsmall = ctx.to_device(broken), ctx.to_device(sbroken), ctx.to_device(small)
    b1, offs1, iovs1, sgl1 = device_sgl(ctx, ecglib, rng, case["lens"])
    b2, offs2, iovs2, sgl2 = device_sgl(ctx, ecglib, rng, [60000, 50000], fill=0)
    b3, offs3, iovs3, sgl3 = device_sgl(ctx, ecglib, rng, [4096], fill=0)
    try:
        assert L.ecg_obj_ec_recov_codec_init(oc, ecglib._u32(lost), len(lost), codec) == 0
        iod, rec, st = recx_arrays(ecglib, case, stripes)
        io = (ecglib.RecovIod * 3)()
        io[0] = ecglib.RecovIod(isz, 0, len(case["iod"]), iod, ct.pointer(sgl1), rec, len(case["recov"]),
                                len(stripes), st, dimg.ptr)
        io[1] = ecglib.RecovIod(sv.size, 1, 0, None, ct.pointer(sgl2), None, 0, 0, None, dsv.ptr)
        io[2] = ecglib.RecovIod(small.size, 1, 0, None, ct.pointer(sgl3), None, 0, 0, None, dsmall.ptr)
        assert L.ecg_obj_ec_recov_data_dev(ctx.h, oc, case["e_len"], codec, io, 3, None) == 0, L.ecg_strerror()
        ctx.sync()
        got1, _ = read_sgl(b1, offs1, case["lens"])
        assert np.array_equal(np.concatenate(got1), expected_user_bytes(case))
        got2, _ = read_sgl(b2, offs2, [60000, 50000])
        assert np.array_equal(np.concatenate(got2)[:sv.size], sv)
        assert np.array_equal(dsv.download().reshape(k + p, scell), simg.reshape(k + p, scell))
        got3, _ = read_sgl(b3, offs3, [4096])
        assert np.array_equal(got3[0][:small.size], small)
        assert sgl2.sg_nr_out == 2 and iovs2[1].iov_len == sv.size - 60000
    finally:
        L.ecg_obj_ec_recov_codec_free(codec)
        for b in (dimg, dsv, dsmall, b1, b2, b3):
            b.free()
