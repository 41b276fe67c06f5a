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
