"""Launch-shape knobs never change results: every block -> (stripe, column)
order of the product kernel (ecg_set_launch_order) gives the oracle's bytes,
including accumulating launches (a duplicated item would XOR twice) and
ragged shapes whose item count the XCD-blocked orders cannot split evenly."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def rand(shape, seed):
    return np.random.default_rng(seed).integers(0, 256, shape, dtype=np.uint8)


@pytest.mark.parametrize("order", [0, 1, 2, 3])
@pytest.mark.parametrize("S,C_", [(24, 8192), (13, 5000), (7, 4096 * 3 + 16)])
def test_orders_encode_and_update(ctx, oracle, order, S, C_):
    k, p = 8, 2
    data = rand((S, k, C_), S * 7 + C_)
    en = oracle.cauchy1(k, p)
    want = np.stack([oracle.encode_data(en[k:], data[s]) for s in range(S)], axis=1)   # [p][S][C]
    ctx.set_order(order)
    try:
        d = ctx.to_device(data)
        par = ctx.alloc(p * S * C_)
        ctx.encode(k, p, C_, S, d.ptr, k * C_, par.ptr, S * C_, C_)
        ctx.sync()
        got = par.download().reshape(p, S, C_)
        assert np.array_equal(got, want)
        # accumulate: replace cell 3 of every stripe (old ^ new), parity in place
        new = rand((S, 1, C_), 99)
        nd = ctx.to_device(new)
        old3 = ctx.to_device(np.ascontiguousarray(data[:, 3:4]))
        ctx.update(k, p, C_, S, [3], old3.ptr, nd.ptr, C_, par.ptr, S * C_, C_)
        ctx.sync()
        d2 = data.copy()
        d2[:, 3] = new[:, 0]
        want2 = np.stack([oracle.encode_data(en[k:], d2[s]) for s in range(S)], axis=1)
        assert np.array_equal(par.download().reshape(p, S, C_), want2)
        for b in (d, par, nd, old3):
            b.free()
    finally:
        ctx.set_order(0)


@pytest.mark.parametrize("cap", [0, 2, 3, 6, 255])
@pytest.mark.parametrize("k,p,S,C_", [(16, 2, 9, 8192), (8, 3, 11, 4096 * 2 + 48), (4, 2, 5, 4096)])
def test_wg_per_cu_caps_encode_and_recover(ctx, oracle, ecglib, cap, k, p, S, C_):
    """ecg_set_wg_per_cu only changes how many blocks share a CU: encode and
    recovery bytes equal the oracle's under every cap."""
    data = rand((S, k, C_), k * 131 + S)
    en = oracle.cauchy1(k, p)
    want = np.stack([oracle.encode_data(en[k:], data[s]) for s in range(S)], axis=1)   # [p][S][C]
    ctx.set_wg_per_cu(cap)
    try:
        d = ctx.to_device(data)
        par = ctx.alloc(p * S * C_)
        ctx.encode(k, p, C_, S, d.ptr, k * C_, par.ptr, S * C_, C_)
        ctx.sync()
        got = par.download().reshape(p, S, C_)
        assert np.array_equal(got, want)
        assert ecglib.last_kernel().startswith("ecg_mm_kernel")
        img = np.concatenate([data, want.transpose(1, 0, 2)], axis=1)          # [S][k+p][C]
        lost = img.copy()
        lost[:, [0, k]] = 0x5A
        st = ctx.to_device(lost)
        ctx.recover(k, p, C_, S, st.ptr, (k + p) * C_, [0, k])
        ctx.sync()
        assert np.array_equal(st.download().reshape(S, k + p, C_), img)
        for b in (d, par, st):
            b.free()
    finally:
        ctx.set_wg_per_cu(0)


def test_wg_per_cu_rejects_bad_values(ctx):
    with pytest.raises(Exception):
        ctx.set_wg_per_cu(17)
    ctx.set_wg_per_cu(0)
