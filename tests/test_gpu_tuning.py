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


PROBE = 23   # ecg_tune.c ECG_TUNE_PROBE: launches before the decision


def test_autotune_probes_decides_and_keeps_bytes(ctx, oracle):
    """The launch tuner (ecg_tune.c) runs the first 23 launches of a wide shape
    as 4 uncapped + 19 capped, then keeps the faster: every launch -- probing,
    capped or not, and after the decision -- writes the oracle's parity, and
    the decision is one of the two arms."""
    k, p, S, C_ = 16, 2, 300, 32768          # 8 columns x 300 stripes = 2400 blocks (> 2048: tuned)
    data = rand((S, k, C_), 1601)
    en = oracle.cauchy1(k, p)
    want = np.stack([oracle.encode_data(en[k:], data[s]) for s in range(S)], axis=1)   # [p][S][C]
    ctx.set_autotune(2)
    try:
        d = ctx.to_device(data)
        assert ctx.tune_state(k, p, C_, S, k * C_, C_) is None
        pars = [ctx.alloc(p * S * C_) for _ in range(PROBE + 2)]
        for par in pars:
            ctx.encode(k, p, C_, S, d.ptr, k * C_, par.ptr, S * C_, C_)
        ctx.sync()
        st = ctx.tune_state(k, p, C_, S, k * C_, C_)
        assert st is not None and st[0] in (2, 255) and st[1] > 0 and st[2] > 0
        for par in pars:
            assert np.array_equal(par.download().reshape(p, S, C_), want)
        # decided shapes keep their choice; the recovery shape (rows = 2, in
        # place) is tuned on its own and recovers the same bytes
        img = np.concatenate([data, want.transpose(1, 0, 2)], axis=1)          # [S][k+p][C]
        for i in range(PROBE + 1):
            lost = img.copy()
            lost[:, [i % k, k]] = 0x3C
            stb = ctx.to_device(lost)
            ctx.recover(k, p, C_, S, stb.ptr, (k + p) * C_, [i % k, k])
            ctx.sync()
            assert np.array_equal(stb.download().reshape(S, k + p, C_), img)
            stb.free()
        st = ctx.tune_state(k, p, C_, S, (k + p) * C_, (k + p) * C_)
        assert st is not None and st[0] in (2, 255)
        for b in pars + [d]:
            b.free()
    finally:
        ctx.set_autotune(1)


def test_autotune_off_and_explicit_cap_skip_tuning(ctx):
    k, p, S, C_ = 8, 2, 96, 131072            # 32 columns x 96 stripes = 3072 blocks
    d = ctx.alloc(S * k * C_)
    par = ctx.alloc(p * S * C_)
    try:
        ctx.set_autotune(2)
        ctx.set_autotune(0)
        for _ in range(PROBE + 2):
            ctx.encode(k, p, C_, S, d.ptr, k * C_, par.ptr, S * C_, C_)
        ctx.sync()
        assert ctx.tune_state(k, p, C_, S, k * C_, C_) is None
        ctx.set_autotune(1)
        ctx.set_wg_per_cu(255)
        for _ in range(PROBE + 2):
            ctx.encode(k, p, C_, S, d.ptr, k * C_, par.ptr, S * C_, C_)
        ctx.sync()
        assert ctx.tune_state(k, p, C_, S, k * C_, C_) is None
    finally:
        ctx.set_wg_per_cu(0)
        ctx.set_autotune(1)
        d.free()
        par.free()


def test_autotune_varying_batches_one_probe(ctx, oracle):
    """Batches of varying size (a queue's flushes, a rebuild's last batch,
    per-shard counts) are one tuner shape: ten batch sizes of an EC_16P2
    encode run ONE probe cycle (23 probing launches), not ten, and every
    output -- probing or decided -- equals the oracle's."""
    k, p, C_ = 16, 2, 65536                    # 16 columns per stripe
    sizes = [130, 200, 131, 257, 140, 190, 300, 150, 170, 222] * 3   # 2080..4800 blocks (> 2048: tuned)
    en = oracle.cauchy1(k, p)
    data = rand((max(sizes), k, C_), 808)
    want = np.stack([oracle.encode_data(en[k:], data[s]) for s in range(max(sizes))], axis=1)   # [p][S][C]
    ctx.set_autotune(2)
    try:
        d = ctx.to_device(data)
        par = ctx.alloc(p * max(sizes) * C_)
        for i, S in enumerate(sizes):
            par.fill(0)
            ctx.encode(k, p, C_, S, d.ptr, k * C_, par.ptr, S * C_, C_)
            ctx.sync()
            got = par.download(p * S * C_).reshape(p, S, C_)
            assert np.array_equal(got, want[:, :S]), (i, S)
        cycles, launches, shapes = ctx.tune_counters()
        assert cycles == 1 and shapes == 1, (cycles, launches, shapes)
        assert launches == PROBE, launches
        st = ctx.tune_state(k, p, C_, sizes[0], k * C_, C_)
        assert st is not None and st[0] in (2, 255)
        # the in-place recovery layout is a second shape, tuned on its own
        img = np.concatenate([data[:150], want[:, :150].transpose(1, 0, 2)], axis=1)
        stb = ctx.to_device(img)
        for _ in range(3):
            ctx.recover(k, p, C_, 150, stb.ptr, (k + p) * C_, [0, 1])
        ctx.sync()
        assert np.array_equal(stb.download().reshape(150, k + p, C_), img)
        assert ctx.tune_counters()[0] == 2
        for b in (d, par, stb):
            b.free()
    finally:
        ctx.set_autotune(1)


def test_autotune_probe_other_stream_not_timed(ctx, ecglib, oracle):
    """Launches of a probing shape from another stream run uncapped and do not
    count toward the probe (their events would time other work)."""
    k, p, S, C_ = 16, 2, 300, 32768
    data = rand((S, k, C_), 1602)
    en = oracle.cauchy1(k, p)
    want = np.stack([oracle.encode_data(en[k:], data[s]) for s in range(S)], axis=1)
    ctx.set_autotune(2)
    st2 = ctx.stream()
    try:
        d = ctx.to_device(data)
        par = ctx.alloc(p * S * C_)
        ctx.encode(k, p, C_, S, d.ptr, k * C_, par.ptr, S * C_, C_)          # starts the probe (default stream)
        for _ in range(5):
            ctx.encode(k, p, C_, S, d.ptr, k * C_, par.ptr, S * C_, C_, stream=st2)
        ctx.sync()
        assert ctx.tune_counters()[1] == 1
        for _ in range(PROBE + 1):
            ctx.encode(k, p, C_, S, d.ptr, k * C_, par.ptr, S * C_, C_)
        ctx.sync()
        assert ctx.tune_counters()[1] == PROBE
        assert ctx.tune_state(k, p, C_, S, k * C_, C_) is not None
        assert np.array_equal(par.download().reshape(p, S, C_), want)
        d.free()
        par.free()
    finally:
        ctx.destroy_stream(st2)
        ctx.set_autotune(1)


def test_autotune_probe_moves_off_idle_stream(ctx, ecglib, oracle):
    """A probe whose starting stream goes idle (its thread exits, its stream is
    destroyed) moves to the stream that keeps launching the shape after
    ECG_TUNE_STALL (64) such launches, and decides there: the
    shape is not left probing -- and uncapped -- for good."""
    k, p, S, C_ = 16, 2, 300, 32768
    data = rand((S, k, C_), 1603)
    en = oracle.cauchy1(k, p)
    want = np.stack([oracle.encode_data(en[k:], data[s]) for s in range(S)], axis=1)
    ctx.set_autotune(2)
    st2 = ctx.stream()
    try:
        d = ctx.to_device(data)
        par = ctx.alloc(p * S * C_)
        ctx.encode(k, p, C_, S, d.ptr, k * C_, par.ptr, S * C_, C_, stream=st2)     # starts the probe on st2
        ctx.sync(st2)
        ctx.destroy_stream(st2)
        st2 = None
        for _ in range(63):             # foreign launches: uncapped, probe untouched
            ctx.encode(k, p, C_, S, d.ptr, k * C_, par.ptr, S * C_, C_)
        ctx.sync()
        assert ctx.tune_counters()[1] == 1
        assert ctx.tune_state(k, p, C_, S, k * C_, C_) is None
        for _ in range(PROBE):          # the 64th hands the probe over; it completes here
            ctx.encode(k, p, C_, S, d.ptr, k * C_, par.ptr, S * C_, C_)
        ctx.sync()
        assert ctx.tune_counters()[1] == 1 + PROBE
        assert ctx.tune_state(k, p, C_, S, k * C_, C_) is not None
        assert np.array_equal(par.download().reshape(p, S, C_), want)
        d.free()
        par.free()
    finally:
        if st2 is not None:
            ctx.destroy_stream(st2)
        ctx.set_autotune(1)


def test_autotune_pointer_tables(ctx, oracle, ecglib):
    """Pointer-table launches (ecg_matmul_ptrs with a table that is not affine:
    the stripes listed in shuffled order) go through the launch tuner as
    their own layout class: one probe of PROBE launches for the wide shape,
    kept apart from the strided encode of the same (k, rows, C), and every
    launch writes the oracle's parity."""
    k, p, S, C_ = 16, 2, 300, 32768          # 2400 blocks: tuned
    data = rand((S, k, C_), 1701)
    en = oracle.cauchy1(k, p)
    want = np.stack([oracle.encode_data(en[k:], data[s]) for s in range(S)], axis=1)   # [p][S][C]
    order = np.random.default_rng(3).permutation(S)
    ctx.set_autotune(2)
    try:
        d = ctx.to_device(data)
        pars = [ctx.alloc(p * S * C_) for _ in range(PROBE + 2)]
        for par in pars:
            cells = []
            for s in order:
                cells += [d.ptr + (int(s) * k + j) * C_ for j in range(k)]
                cells += [par.ptr + r * S * C_ + int(s) * C_ for r in range(p)]
            ctx.matmul_ptrs(k, p, en[k:], C_, S, cells)
            assert ecglib.last_kernel().startswith("ecg_mm_ptr_kernel<16,2"), ecglib.last_kernel()
        ctx.sync()
        cycles, launches, shapes = ctx.tune_counters()
        assert cycles == 1 and launches == PROBE and shapes == 1, (cycles, launches, shapes)
        for par in pars:
            assert np.array_equal(par.download().reshape(p, S, C_), want)
        # the strided encode of the same shape is a different layout class: a probe of its own
        ctx.encode(k, p, C_, S, d.ptr, k * C_, pars[0].ptr, S * C_, C_)
        ctx.sync()
        assert ctx.tune_counters()[0] == 2
        for b in pars + [d]:
            b.free()
    finally:
        ctx.set_autotune(1)
