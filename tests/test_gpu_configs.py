"""BASELINE.json configs at their full sizes, every output byte compared with
the CPU oracle: the scalar ISA-L ec_encode_data_base restatement
(oracle/ec_ref.c) for configs[0] and [4], and for the multi-GiB configs[1]-[3]
the oracle's SIMD restatement (oracle/ec_simd.c, OpenMP over stripes), itself
compared with the scalar one on sampled stripes inside the same test.

  configs[0]  EC_2P1, 128 KiB cells, 1024 stripes: encode + verify
              (the reference's loop: obj_ec_recx_encode,
              ref:src/object/cli_ec.c:627-659)
  configs[1]  EC_4P2, 1 MiB cells, 1024 stripes (4 GiB): encode in the client
              layout + {d0,d1} decode in the recovery layout, every byte
  configs[2]  EC_8P2, 1 MiB cells, 512 stripes: {d0,d1} degraded decode into
              marker-filled cells (obj_ec_recov_data,
              ref:src/object/cli_ec.c:2814-2885, loop :2874-2878), every byte
  configs[3]  EC_16P2, 128 KiB cells, 8192 stripes (16 GiB): the 8 shard
              launches of the 8-GPU split, every parity byte
  configs[4]  the EC_8P2 rebuild stream at its real shape: 1 MiB cells, a
              64-stripe batch streamed through 16-stripe staging chunks,
              host memory on both ends (ecg_encode_host / ecg_recover_host;
              migrate_update_parity ref:src/object/srv_obj_migrate.c:1116-1177,
              obj_ec_recov_data ref:src/object/cli_ec.c:2814-2885)
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NTHREADS = max(1, min(16, len(os.sched_getaffinity(0))))   # the GPU box's CPU share is 16
MARKER = 0x5A


def big_data(nbytes, config_id, tile=256 << 20):
    """nbytes of seeded stripe bytes: one 256 MiB xoshiro tile (tools/datagen),
    rolled by a different amount for every tile so no two tiles are alike
    (generating 16 GiB with the numpy generator alone takes a minute)."""
    from tools.datagen import stripe_bytes

    base = stripe_bytes(min(tile, nbytes), config_id)
    out = np.empty(nbytes, dtype=np.uint8)
    for i, off in enumerate(range(0, nbytes, base.size)):
        n = min(base.size, nbytes - off)
        out[off:off + n] = np.roll(base, i * 4099 + 1)[:n]
    return out


def simd_parity(oracle, k, p, C_, S, data, sample):
    """Parity [p][S][C] of every stripe from the SIMD oracle; the SIMD path is
    checked against the scalar ec_encode_data_base restatement on `sample`."""
    want = oracle.encode_batch(k, p, C_, S, data, nthreads=NTHREADS, simd=True).reshape(p, S, C_)
    d3 = data.reshape(S, k, C_)
    for s in sample:
        one = oracle.encode_batch(k, p, C_, 1, np.ascontiguousarray(d3[s]).reshape(-1)).reshape(p, C_)
        assert np.array_equal(one, want[:, s]), f"SIMD oracle != scalar oracle at stripe {s}"
    return want


def test_config1_ec2p1_128k_full_size(ctx, oracle):
    """configs[0]: EC_2P1, 128 KiB x 1024 stripes (256 MiB data, 128 MiB
    parity) in the client write layout; every parity byte equals the
    oracle's, and a d0 erasure recovered on the device equals the data."""
    from tools.datagen import stripe_bytes

    k, p, C_, S = 2, 1, 128 << 10, 1024
    data = stripe_bytes(S * k * C_, 0).reshape(S, k, C_)
    d = ctx.to_device(data)
    par = ctx.alloc(p * S * C_)
    ctx.encode(k, p, C_, S, d.ptr, k * C_, par.ptr, S * C_, C_)
    ctx.sync()
    assert ctx_kernel_ok("ecg_mm_kernel<2,1,")
    got = par.download().reshape(p, S, C_)
    want = oracle.encode_batch(k, p, C_, S, np.ascontiguousarray(data).reshape(-1),
                               nthreads=NTHREADS).reshape(p, S, C_)
    assert np.array_equal(got, want)

    # verify by decode: stripes [S][k+p][C] with d0 erased -> recovered == data
    stripes = np.empty((S, k + p, C_), dtype=np.uint8)
    stripes[:, :k] = data
    stripes[:, k:] = got.transpose(1, 0, 2)
    stripes[:, 0] = 0x5A
    sd = ctx.to_device(stripes)
    ctx.recover(k, p, C_, S, sd.ptr, (k + p) * C_, [0])
    ctx.sync()
    rec = sd.download().reshape(S, k + p, C_)
    assert np.array_equal(rec[:, :k], data)
    for b in (d, par, sd):
        b.free()


def ctx_kernel_ok(prefix):
    from daos_amd import ecg

    return ecg.last_kernel().startswith(prefix)


def test_config5_rebuild_stream_shape_vs_oracle(ctx, oracle):
    """configs[4] at its real shape: EC_8P2, 1 MiB cells, one 64-stripe
    encode batch and one {d0,d1} recovery batch streamed through 16-stripe
    staging chunks from pinned host memory.  Parity is compared byte for
    byte with the oracle (not only through a round trip); the erased cells
    are overwritten with a marker first, so a recovery that wrote nothing
    fails."""
    from tools.datagen import stripe_bytes

    k, p, C_, S, chunk = 8, 2, 1 << 20, 64, 16
    hd = ctx.host_alloc(S * k * C_)
    hp = ctx.host_alloc(S * p * C_)
    hs = ctx.host_alloc(S * (k + p) * C_)
    try:
        data = hd.array
        data[:] = stripe_bytes(S * k * C_, 9)
        hp.array[:] = 0xA5
        ctx.encode_host(k, p, C_, S, data, hp.array, chunk=chunk)
        want = oracle.encode_batch(k, p, C_, S, data, nthreads=NTHREADS)
        assert np.array_equal(hp.array, want)

        img = hs.array.reshape(S, k + p, C_)
        img[:, :k] = data.reshape(S, k, C_)
        img[:, k:] = want.reshape(p, S, C_).transpose(1, 0, 2)
        img[:, [0, 1]] = 0x5A                        # erased cells: marker bytes
        ctx.recover_host(k, p, C_, S, hs.array, [0, 1], chunk=chunk)
        assert np.array_equal(img[:, :k], data.reshape(S, k, C_))
        assert np.array_equal(img[:, k:], want.reshape(p, S, C_).transpose(1, 0, 2))
    finally:
        for b in (hd, hp, hs):
            b.free()


def test_config2_ec4p2_1mib_every_byte(ctx, oracle):
    """configs[1] (the headline step): EC_4P2, 1 MiB cells, 1024 stripes.
    Encode in the client write layout (data [S][k][C] -> parity [p][S][C] at
    the bench's padded row pitch): all 2 GiB of parity equal the oracle's.
    Then the {d0,d1} degraded decode in the recovery layout [S][k+p][C] with
    the erased cells marker-filled: all 6 GiB of the image equal data+parity."""
    k, p, C_, S = 4, 2, 1 << 20, 1024
    pitch = S * C_ + 4096
    data = big_data(S * k * C_, 2)
    d = ctx.to_device(data)
    par = ctx.alloc(p * pitch)
    par.fill(0xA5)
    ctx.encode(k, p, C_, S, d.ptr, k * C_, par.ptr, pitch, C_)
    ctx.sync()
    assert ctx_kernel_ok("ecg_mm_kernel<4,2,")
    got = par.download().reshape(p, pitch)[:, :S * C_].reshape(p, S, C_)
    d.free()
    par.free()
    want = simd_parity(oracle, k, p, C_, S, data, [0, 1, 511, 1023])
    assert np.array_equal(got, want)
    del got

    img = np.empty((S, k + p, C_), dtype=np.uint8)
    img[:, :k] = data.reshape(S, k, C_)
    img[:, k:] = want.transpose(1, 0, 2)
    del data, want
    img_dev = ctx.to_device(img)
    stride = (k + p) * C_
    for s0 in range(0, S, 256):                  # erase d0,d1 of every stripe
        blk = img[s0:s0 + 256].copy()
        blk[:, [0, 1]] = MARKER
        img_dev.upload(blk, offset=s0 * stride)
    ctx.recover(k, p, C_, S, img_dev.ptr, stride, [0, 1])
    ctx.sync()
    assert ctx_kernel_ok("ecg_mm_kernel<4,2,")
    rec = img_dev.download().reshape(S, k + p, C_)
    img_dev.free()
    assert np.array_equal(rec, img)


def test_config3_ec8p2_1mib_decode_every_byte(ctx, oracle):
    """configs[2]: EC_8P2, 1 MiB cells, 512 stripes in [S][k+p][C].  The
    parity (encoded on the device in place) equals the SIMD oracle's for
    every stripe; then every stripe's d0,d1 are marker-filled and recovered
    in place: the whole 5 GiB image equals data + oracle parity, and the
    oracle's own {d0,d1} recovery of the same marker-filled image agrees."""
    k, p, C_, S = 8, 2, 1 << 20, 512
    stride = (k + p) * C_
    data = big_data(S * k * C_, 3)
    img = np.empty((S, k + p, C_), dtype=np.uint8)
    img[:, :k] = data.reshape(S, k, C_)
    img[:, k:] = MARKER
    buf = ctx.to_device(img)
    ctx.encode(k, p, C_, S, buf.ptr, stride, buf.ptr + k * C_, C_, stride)
    ctx.sync()
    par = buf.download().reshape(S, k + p, C_)[:, k:].copy()
    want = simd_parity(oracle, k, p, C_, S, data, [0, 255, 511])
    assert np.array_equal(par, want.transpose(1, 0, 2))
    img[:, k:] = par
    del data, want, par

    broken = img.copy()
    broken[:, [0, 1]] = MARKER
    buf.upload(broken)
    ctx.recover(k, p, C_, S, buf.ptr, stride, [0, 1])
    ctx.sync()
    assert ctx_kernel_ok("ecg_mm_kernel<8,2,")
    got = buf.download().reshape(S, k + p, C_)
    buf.free()
    assert np.array_equal(got, img)
    del got
    rc, _, dec, el, gt, _ = oracle.recov_codec(k, p, [0, 1])
    assert rc == 0
    oracle.recov_batch(k, 2, gt, dec, el, C_, stride, S, broken, nthreads=NTHREADS, simd=True)
    assert np.array_equal(broken, img)


def test_config4_ec16p2_8192_stripes_every_byte(ctx, oracle):
    """configs[3]: EC_16P2, 128 KiB cells, 8192 stripes (16 GiB of data)
    split over 8 GPUs by contiguous stripe ranges (bench.py --workload
    enc_16p2_strong, ecg_multi_range).  The 8 shard launches -- what the 8
    GPUs each run -- write all 2 GiB of parity; every byte equals the SIMD
    oracle's, and one launch over all 8192 stripes writes the same bytes."""
    from daos_amd import ecg

    k, p, C_, S, G = 16, 2, 128 << 10, 8192, 8
    data = big_data(S * k * C_, 4)
    d = ctx.to_device(data)
    shard = ctx.alloc(p * S * C_)
    full = ctx.alloc(p * S * C_)
    shard.fill(0xA5)
    full.fill(0x3C)
    try:
        m = ecg.Multi([0] * G)
        try:
            ranges = [m.range(S, g) for g in range(G)]
        finally:
            m.close()
        assert sum(c for _, c in ranges) == S and ranges[0] == (0, S // G)
        for f, c in ranges:
            ctx.encode(k, p, C_, c, d.ptr + f * k * C_, k * C_, shard.ptr + f * C_, S * C_, C_)
        ctx.encode(k, p, C_, S, d.ptr, k * C_, full.ptr, S * C_, C_)
        ctx.sync()
        assert ctx_kernel_ok("ecg_mm_kernel<16,2,")
        got = shard.download().reshape(p, S, C_)
        assert np.array_equal(full.download().reshape(p, S, C_), got)
    finally:
        d.free()
        shard.free()
        full.free()
    want = simd_parity(oracle, k, p, C_, S, data, [0, 1023, 1024, 8191])
    assert np.array_equal(got, want)
