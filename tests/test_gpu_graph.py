"""The batched device calls are HIP-graph capturable: the GF tables travel in
the kernel arguments and the calls issue nothing but launches and copies on
the given stream, so a rebuild step (encode, 2-erasure recovery, checksum of
the recovered cells) recorded once replays on new stripe contents.  Captured
with hipStreamBeginCapture on a libecg stream (the HIP runtime libecg links),
replayed three times, checked against the oracle each time."""
import ctypes as ct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _hip():
    hip = ct.CDLL("libamdhip64.so.7")          # the runtime libecg.so links (already loaded)
    vp = ct.c_void_p
    hip.hipStreamBeginCapture.argtypes = [vp, ct.c_int]
    hip.hipStreamEndCapture.argtypes = [vp, ct.POINTER(vp)]
    hip.hipGraphInstantiate.argtypes = [ct.POINTER(vp), vp, vp, vp, ct.c_size_t]
    hip.hipGraphLaunch.argtypes = [vp, vp]
    hip.hipGraphExecDestroy.argtypes = [vp]
    hip.hipGraphDestroy.argtypes = [vp]
    return hip


def test_capture_and_replay(oracle, ecglib, ctx):
    hip = _hip()
    L = ecglib.lib()
    k, p, C_, S = 8, 2, 64 << 10, 16
    stride = (k + p) * C_
    nch = L.ecg_csum_chunk_count(32768, 1, 0, C_)
    stripes = ctx.alloc(S * stride)
    work = ctx.alloc(S * stride)
    csums = ctx.alloc(2 * S * nch * 4)
    st = ctx.stream()
    graph, gexec = ct.c_void_p(), ct.c_void_p()
    try:
        stripes.fill(0)
        # warm the decode-matrix cache and the CRC tables outside the capture
        ctx.recover(k, p, C_, S, stripes.ptr, stride, [0, k + 1])
        ctx.csum_extents(ecglib.HASH_CRC32, 32768, 1, 0, C_, stripes.ptr, C_, 1, csums.ptr)
        ctx.sync()
        assert hip.hipStreamBeginCapture(st, 0) == 0
        ctx.encode(k, p, C_, S, stripes.ptr, stride, stripes.ptr + k * C_, C_, stride, stream=st)
        assert L.ecg_memcpy(ctx.h, work.ptr, stripes.ptr, S * stride, 2, st) == 0
        assert L.ecg_memset(ctx.h, work.ptr, 0, C_, st) == 0                 # lose d0 of stripe 0
        ctx.recover(k, p, C_, S, work.ptr, stride, [0, k + 1], stream=st)
        for i, cell in enumerate((0, k + 1)):
            ctx.csum_extents(ecglib.HASH_CRC32, 32768, 1, 0, C_, work.ptr + cell * C_, stride, S,
                             csums.ptr + i * S * nch * 4, stream=st)
        assert hip.hipStreamEndCapture(st, ct.byref(graph)) == 0
        assert hip.hipGraphInstantiate(ct.byref(gexec), graph, None, None, 0) == 0
        en = oracle.cauchy1(k, p)
        for rep in range(3):
            data = np.random.default_rng(rep).integers(0, 256, (S, k, C_), dtype=np.uint8)
            img = np.zeros((S, k + p, C_), dtype=np.uint8)
            img[:, :k] = data
            stripes.upload(img, stream=st)
            assert hip.hipGraphLaunch(gexec, st) == 0
            ctx.sync(st)
            enc = stripes.download(stream=st).reshape(S, k + p, C_)
            rec = work.download(stream=st).reshape(S, k + p, C_)
            for s in range(S):
                assert np.array_equal(enc[s, k:], oracle.encode_data(en[k:], data[s])), (rep, s)
            assert np.array_equal(rec, enc), rep
            got = csums.download(2 * S * nch * 4, stream=st).view(np.uint32).reshape(2, S, nch)
            for i, cell in enumerate((0, k + 1)):
                want = oracle.csum_extents(oracle.HASH_CRC32, 32768, 1, 0, C_, enc[:, cell].reshape(-1),
                                           ext_stride=C_, n_ext=S)
                assert np.array_equal(got[i], want), (rep, cell)
    finally:
        if gexec:
            hip.hipGraphExecDestroy(gexec)
        if graph:
            hip.hipGraphDestroy(graph)
        ctx.destroy_stream(st)
        stripes.free()
        work.free()
        csums.free()
