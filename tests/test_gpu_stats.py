"""Codec telemetry (ecg_get_stats, include/ecg.h): the counters follow the
work done -- full-stripe encodes, regenerations, partial updates, checksum
chunks, launches and the host pipelines' PCIe bytes -- and reset to zero."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_stats_count_codec_work(ctx, ecglib):
    k, p, C_, S = 8, 2, 8192, 6
    ctx.stats(reset=True)
    assert all(v == 0 for v in ctx.stats().values())
    rng = np.random.default_rng(5)
    stripes = rng.integers(0, 256, (S, k + p, C_), dtype=np.uint8)
    d = ctx.to_device(stripes)
    st = (k + p) * C_
    ctx.encode(k, p, C_, S, d.ptr, st, d.ptr + k * C_, C_, st)
    ctx.recover(k, p, C_, S, d.ptr, st, [0, 9])
    ctx.update(k, p, C_, S, [3], d.ptr + 3 * C_, d.ptr + 4 * C_, st, d.ptr + k * C_, C_, st)
    out = ctx.alloc(p * S * (C_ // 4096) * 4)
    ctx.encode_csum(k, p, C_, S, d.ptr, st, d.ptr + k * C_, C_, st, ecglib.HASH_CRC32, 4096, 1, out.ptr)
    ctx.csum_extents(ecglib.HASH_CRC32, 4096, 1, 0, C_, d.ptr, st, S, out.ptr)
    ctx.sync()
    s = ctx.stats()
    assert s["encode_stripes"] == 2 * S and s["encode_bytes"] == 2 * k * C_ * S
    assert s["recover_stripes"] == S and s["recover_bytes"] == 2 * C_ * S
    assert s["update_cells"] == S and s["update_bytes"] == C_ * S
    assert s["csum_chunks"] == p * S * (C_ // 4096) + S * (C_ // 4096)
    assert s["launches"] >= 5
    assert s["h2d_bytes"] == 0 and s["d2h_bytes"] == 0
    hd = np.ascontiguousarray(stripes[:, :k])
    par = np.zeros((p, S, C_), dtype=np.uint8)
    ctx.encode_host(k, p, C_, S, hd, par, chunk=4)
    s2 = ctx.stats(reset=True)
    assert s2["h2d_bytes"] == k * C_ * S and s2["d2h_bytes"] == p * C_ * S
    assert s2["encode_stripes"] == 3 * S
    assert all(v == 0 for v in ctx.stats().values())
    d.free()
    out.free()
