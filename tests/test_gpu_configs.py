"""BASELINE.json configs at their full sizes, every output byte compared with
the CPU oracle (oracle/ec_ref.c, the scalar ISA-L ec_encode_data_base
restatement, OpenMP over stripes).

  configs[0]  EC_2P1, 128 KiB cells, 1024 stripes: encode + verify
              (the reference's loop: obj_ec_recx_encode,
              ref:src/object/cli_ec.c:627-659)
  configs[4]  the EC_8P2 rebuild stream at its real shape: 1 MiB cells, a
              64-stripe batch streamed through 16-stripe staging chunks,
              host memory on both ends (ecg_encode_host / ecg_recover_host;
              migrate_update_parity ref:src/object/srv_obj_migrate.c:1116-1177,
              obj_ec_recov_data ref:src/object/cli_ec.c:2814-2885)
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NTHREADS = 16


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
