"""GPU parity tests: the HIP path (through the C-ABI) vs the CPU oracle.

Bit-exact for every byte (integer GF(2^8) work): every case here compares
every output byte with the oracle, at sizes the oracle finishes in seconds.
The BASELINE.json configs are byte-compared at their full sizes in
tests/test_gpu_configs.py (every parity byte and every recovered byte of
configs 1-4, the rebuild-stream shape of config 5), and the product kernels'
operand alignments (16 / 8 / 4 / 1 bytes) in tests/test_gpu_align.py.
"""
import ctypes as C
import itertools
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CLASSES = [(2, 1), (2, 2), (4, 1), (4, 2), (8, 1), (8, 2), (16, 1), (16, 2), (4, 3), (8, 3), (16, 3)]


def rand(shape, seed):
    return np.random.default_rng(seed).integers(0, 256, shape, dtype=np.uint8)


def encode_dev(ctx, k, p, C_, data):
    """data [S][k][C] -> parity [p][S][C] through ecg_encode (client layout)."""
    S = data.shape[0]
    d = ctx.to_device(data)
    par = ctx.alloc(p * S * C_)
    ctx.encode(k, p, C_, S, d.ptr, k * C_, par.ptr, S * C_, C_)
    ctx.sync()
    out = par.download().reshape(p, S, C_)
    d.free()
    par.free()
    return out


def oracle_parity(oracle, k, p, data):
    en = oracle.cauchy1(k, p)
    return np.stack([oracle.encode_data(en[k:], data[s]) for s in range(data.shape[0])], axis=1)


def check_route(ecglib, route):
    k = ecglib.last_kernel()
    assert k.startswith("cpu:") if route == "cpu" else k.startswith("ecg_mm"), (route, k)


# --------------------------------------------------------------- field level
def test_every_gf_product(ctx, oracle):
    """All 256 x 256 products: coefficient c applied to bytes 0..255."""
    src = np.tile(np.arange(256, dtype=np.uint8), 16)       # 4 KiB cell
    want = np.array([[oracle.gf_mul(a, b) for b in range(256)] for a in range(256)], dtype=np.uint8)
    d = ctx.to_device(src)
    out = ctx.alloc(8 * src.size)
    for c0 in range(0, 256, 8):
        coef = np.arange(c0, c0 + 8, dtype=np.uint8).reshape(8, 1)
        ctx.matmul(coef, src.size, 1, d.ptr, [0], 0, out.ptr, [r * src.size for r in range(8)], 0)
        got = out.download().reshape(8, 16, 256)
        for r in range(8):
            assert np.array_equal(got[r, 0], want[c0 + r]), c0 + r
            assert np.array_equal(got[r, 7], want[c0 + r])
    d.free()
    out.free()


# --------------------------------------------------------------- encode
@pytest.mark.parametrize("k,p", CLASSES)
def test_encode_all_classes(ctx, oracle, ecglib, k, p):
    S, C_ = 5, 8192 + 4096
    data = rand((S, k, C_), k * 31 + p)
    got = encode_dev(ctx, k, p, C_, data)
    assert ecglib.last_kernel().startswith(f"ecg_mm_kernel<{k},{p},"), ecglib.last_kernel()
    assert np.array_equal(got, oracle_parity(oracle, k, p, data))


@pytest.mark.parametrize("C_", [1, 15, 16, 17, 32, 37, 311 * 3, 933, 4095, 4096, 4097, 8569, 65536 + 48])
def test_encode_ragged_cells(ctx, oracle, C_):
    k, p, S = 4, 2, 3
    data = rand((S, k, C_), C_)
    assert np.array_equal(encode_dev(ctx, k, p, C_, data), oracle_parity(oracle, k, p, data))


@pytest.mark.parametrize("k,rows", [(1, 1), (3, 5), (5, 4), (7, 8), (12, 6), (16, 8), (17, 3), (33, 2), (64, 8)])
def test_generic_and_split_shapes(ctx, oracle, ecglib, k, rows):
    """Shapes without a specialised kernel (runtime-shaped kernel), k > 16
    (accumulating launches) and rows up to 8, random coefficients."""
    S, C_ = 3, 4096 + 512
    coef = rand((rows, k), 1000 + k * rows)
    data = rand((S, k, C_), k + rows)
    d = ctx.to_device(data)
    out = ctx.alloc(S * rows * C_)
    ctx.matmul(coef, C_, S, d.ptr, [j * C_ for j in range(k)], k * C_, out.ptr, [r * C_ for r in range(rows)],
               rows * C_, 0)
    got = out.download().reshape(S, rows, C_)
    for s in range(S):
        assert np.array_equal(got[s], oracle.encode_data(coef, data[s]))
    d.free()
    out.free()


def test_accumulate_flag(ctx, oracle):
    k, rows, C_, S = 4, 3, 5000, 2
    coef = rand((rows, k), 5)
    data = rand((S, k, C_), 6)
    base = rand((S, rows, C_), 7)
    d = ctx.to_device(data)
    o = ctx.to_device(base)
    ctx.matmul(coef, C_, S, d.ptr, [j * C_ for j in range(k)], k * C_, o.ptr, [r * C_ for r in range(rows)],
               rows * C_, 1)
    got = o.download().reshape(S, rows, C_)
    for s in range(S):
        assert np.array_equal(got[s], base[s] ^ oracle.encode_data(coef, data[s]))


@pytest.mark.parametrize("variant,kernel", [(0, "ecg_mm_kernel<4,2,0,0,g1>"), (2, "ecg_mm_byte_kernel")])
def test_misaligned_cells(ctx, oracle, ecglib, variant, kernel):
    """Cells at odd byte offsets and an odd cell size (user sgl offsets carry
    no alignment): the funnel-shift lanes with misaligned dword
    stores, and the byte kernel (launch variant 2, the independent second
    implementation); same bytes."""
    k, p, C_, S = 4, 2, 1001, 3
    data = rand((S, k, C_), 11)
    buf = np.zeros(S * k * C_ + 64, dtype=np.uint8)
    buf[3:3 + data.size] = data.reshape(-1)
    d = ctx.to_device(buf)
    par = ctx.alloc(p * S * C_ + 64)
    par.fill(0xEE)
    coef = oracle.cauchy1(k, p)[k:]
    ctx.set_launch(0, 0, variant)
    try:
        ctx.matmul(coef, C_, S, d.ptr + 3, [j * C_ for j in range(k)], k * C_, par.ptr + 5,
                   [r * S * C_ for r in range(p)], C_, 0)
        ctx.sync()
    finally:
        ctx.set_launch(0, 0, 0)
    assert ecglib.last_kernel() == kernel
    raw = par.download()
    assert np.array_equal(raw[5:5 + p * S * C_].reshape(p, S, C_), oracle_parity(oracle, k, p, data))
    assert (raw[:5] == 0xEE).all() and (raw[5 + p * S * C_:] == 0xEE).all()
    d.free()
    par.free()


def test_golden_fixtures(ctx):
    fx = np.load(os.path.join(GOLD, "fixtures.npz"))
    for name in sorted({n.split("/")[0] for n in fx.files}):
        k, p = (int(x) for x in fx[f"{name}/kp"])
        data = fx[f"{name}/data"]
        C_ = data.shape[1]
        got = encode_dev(ctx, k, p, C_, data[None])
        assert np.array_equal(got[:, 0], fx[f"{name}/parity"]), name


# --------------------------------------------------------------- recovery
def _recovery_check(ctx, oracle, k, p, C_, S, patterns, seed):
    data = rand((S, k, C_), seed)
    par = oracle_parity(oracle, k, p, data)
    stripes = np.concatenate([data, par.transpose(1, 0, 2)], axis=1)   # [S][k+p][C]
    d = ctx.alloc(stripes.nbytes)
    for pat in patterns:
        broken = stripes.copy()
        broken[:, list(pat)] = 0xA5
        d.upload(broken)
        ctx.recover(k, p, C_, S, d.ptr, (k + p) * C_, list(pat))
        got = d.download().reshape(S, k + p, C_)
        assert np.array_equal(got, stripes), pat
        # where the reference's data-first assumption holds, its recovery
        # (oracle restatement) writes the same bytes
        rc, de, dec, el, gt, reused = oracle.recov_codec(k, p, list(pat))
        s0 = broken[0].copy()
        data_first = all(a < k or b >= k for a, b in zip(pat, pat[1:]))
        if not reused:
            out = oracle.encode_data(de, s0[dec])
            for i, e in enumerate(el):
                if e < k or data_first:
                    assert np.array_equal(out[i], got[0, e])
    d.free()


@pytest.mark.parametrize("k,p", [(2, 1), (2, 2), (4, 1), (4, 2), (4, 3), (8, 2)])
def test_recover_every_erasure_set(ctx, oracle, k, p):
    pats = [c for e in range(1, p + 1) for c in itertools.combinations(range(k + p), e)]
    _recovery_check(ctx, oracle, k, p, 4096 + 64, 3, pats, k * 7 + p)


@pytest.mark.parametrize("k,p", [(8, 3), (16, 2), (16, 3), (16, 1), (8, 1)])
def test_recover_sampled_erasure_sets(ctx, oracle, k, p):
    rng = np.random.default_rng(k + p)
    pats = [c for e in range(1, p + 1) for c in itertools.combinations(range(k + p), e)]
    pick = [pats[i] for i in rng.choice(len(pats), min(40, len(pats)), replace=False)]
    pick += [tuple(range(k, k + p)), tuple(range(p))]          # all parity lost / leading data lost
    _recovery_check(ctx, oracle, k, p, 8192, 2, pick, 99 + k)


def test_recover_parity_first_order(ctx, oracle):
    """err_list in failure-insertion order with parity before data
    (ref:src/object/cli_ec.c:1388-1391): the reference indexes its zero-filled
    (k+p) x k inverse buffer past the k x k head for a parity cell listed
    among the first er_data_nerrs entries, so it writes that parity cell as
    ALL ZEROS (oracle restatement, tests/test_oracle.py); data cells match it.
    The product builds its rows data-first and regenerates the true parity
    there -- the one deliberate byte divergence, in a cell degraded reads
    never return."""
    _recovery_check(ctx, oracle, 4, 2, 4096, 2, [(5, 0), (4, 3), (5, 1)], 3)
    k, p, C_ = 4, 2, 4096
    data = rand((1, k, C_), 4)
    stripes = np.concatenate([data, oracle_parity(oracle, k, p, data).transpose(1, 0, 2)], axis=1)
    rc, de, dec, el, gt, reused = oracle.recov_codec(k, p, [5, 0])
    ref_out = oracle.encode_data(de, stripes[0][dec])
    assert not ref_out[0].any() and np.array_equal(ref_out[1], stripes[0, 0])
    d = ctx.to_device(np.where(np.isin(np.arange(k + p), [5, 0])[None, :, None], 0xA5, stripes).astype(np.uint8))
    ctx.recover(k, p, C_, 1, d.ptr, (k + p) * C_, [5, 0])
    got = d.download().reshape(1, k + p, C_)
    d.free()
    assert np.array_equal(got, stripes) and got[0, 5].any()


def test_recover_data_loss(ctx, ecglib):
    d = ctx.alloc(6 * 4096)
    with pytest.raises(ecglib.EcgError) as ei:
        ctx.recover(4, 2, 4096, 1, d.ptr, 6 * 4096, [0, 1, 2])
    assert ei.value.rc == -ecglib.DER_DATA_LOSS
    d.free()


# --------------------------------------------------------------- update
@pytest.mark.parametrize("k,p,cells", [(4, 2, [1]), (8, 2, [0, 5]), (8, 3, [2, 3, 7]), (16, 2, list(range(16))),
                                     (4, 1, [2]), (8, 1, [0, 1, 2, 3]), (16, 3, [4, 9]), (4, 3, [0, 1, 2, 3]),
                                     (8, 2, [1, 2, 4, 6, 7])])
def test_update_matches_oracle(ctx, oracle, ecglib, k, p, cells):
    """Delta parity update (ACC + DIFF): 1-4 cells per stripe on their own
    instantiations, more on the runtime-shaped kernel."""
    C_, S = 6000, 3
    en = oracle.cauchy1(k, p)
    data = rand((S, k, C_), 21)
    par = oracle_parity(oracle, k, p, data)               # [p][S][C]
    new = rand((S, len(cells), C_), 22)
    old = data[:, cells].copy()
    dold, dnew = ctx.to_device(old), ctx.to_device(new)
    dpar = ctx.to_device(par)
    ctx.update(k, p, C_, S, cells, dold.ptr, dnew.ptr, len(cells) * C_, dpar.ptr, S * C_, C_)
    ctx.sync()
    n = len(cells)
    assert ecglib.last_kernel() == (f"ecg_mm_kernel<{n},{p},1,1>" if n <= 4 else "ecg_mm_kernel<0,0,1,1>"), \
        ecglib.last_kernel()
    got = dpar.download().reshape(p, S, C_)
    for s in range(S):
        want = par[:, s].copy()
        for u, j in enumerate(cells):
            want = oracle.encode_data_update(en[k:], j, old[s, u] ^ new[s, u], want)
        assert np.array_equal(got[:, s], want)
        data[s, cells] = new[s]
    assert np.array_equal(got, oracle_parity(oracle, k, p, data))
    for b in (dold, dnew, dpar):
        b.free()


# --------------------------------------------------------------- ISA-L drop-in
def test_isal_drop_in(ecglib, oracle, ctx, route):
    k, p, n = 8, 3, 32768 + 5
    en = np.zeros((k + p) * k, dtype=np.uint8)
    ecglib.lib().gf_gen_cauchy1_matrix(en.ctypes.data_as(ecglib.u8p), k + p, k)
    en = en.reshape(k + p, k)
    tbls = ecglib.isal_init_tables(en[k:])
    data = [rand(n, 40 + j) for j in range(k)]
    coding = [np.zeros(n, dtype=np.uint8) for _ in range(p)]
    ecglib.isal_encode_data(tbls, k, p, data, coding)
    check_route(ecglib, route)
    want = oracle.encode_data(en[k:], np.stack(data))
    assert all(np.array_equal(coding[r], want[r]) for r in range(p))
    # ec_encode_data_update on one cell
    delta = rand(n, 50)
    ecglib.isal_encode_data_update(tbls, k, p, 3, delta, coding)
    want2 = oracle.encode_data_update(en[k:], 3, delta, want)
    assert all(np.array_equal(coding[r], want2[r]) for r in range(p))
    # xor_gen
    a, b, c = rand(n, 60), rand(n, 61), np.zeros(n, dtype=np.uint8)
    assert ecglib.isal_xor_gen([a, b, c]) == 0
    assert np.array_equal(c, a ^ b)
    assert ecglib.isal_xor_gen([a, c]) != 0


def test_isal_drop_in_device_cells(ecglib, oracle, ctx):
    """The ISA-L data-plane calls with cells in device memory (an engine whose
    buffers live in HBM keeps its ec_encode_data call sites,
    ref:src/object/cli_ec.c:540): scattered cells at odd offsets of
    hipMalloc'd buffers, used in place -- ec_encode_data, then
    ec_encode_data_update of one cell, then xor_gen."""
    L = ecglib.lib()
    k, p, n = 8, 3, 32768 + 5
    en = np.zeros((k + p) * k, dtype=np.uint8)
    L.gf_gen_cauchy1_matrix(en.ctypes.data_as(ecglib.u8p), k + p, k)
    en = en.reshape(k + p, k)
    tbls = ecglib.isal_init_tables(en[k:])
    data = np.stack([rand(n, 140 + j) for j in range(k)])
    slot = n + 64
    dbuf, pbuf = ctx.alloc((k + 2) * slot), ctx.alloc((p + 1) * slot)
    order = [5, 0, 9, 2, 7, 1, 3, 8]                # cells scattered over the slots, odd offsets
    dofs = [order[j] * slot + 2 * j + 1 for j in range(k)]
    pofs = [r * slot + 3 for r in range(p)]
    try:
        for j in range(k):
            dbuf.upload(data[j], offset=dofs[j])
        pbuf.fill(0xEE)
        dp = (ecglib.u8p * k)(*[C.cast(C.c_void_p(dbuf.ptr + o), ecglib.u8p) for o in dofs])
        cp = (ecglib.u8p * p)(*[C.cast(C.c_void_p(pbuf.ptr + o), ecglib.u8p) for o in pofs])
        L.ec_encode_data(n, k, p, tbls.ctypes.data_as(ecglib.u8p), dp, cp)
        want = oracle.encode_data(en[k:], data)
        raw = pbuf.download()
        assert all(np.array_equal(raw[pofs[r]: pofs[r] + n], want[r]) for r in range(p))
        assert (raw[:3] == 0xEE).all() and (raw[pofs[0] + n: pofs[1]] == 0xEE).all()
        # one cell updated: parity ^= coef * delta
        delta = rand(n, 150)
        dbuf.upload(delta, offset=dofs[0])
        L.ec_encode_data_update(n, k, p, 3, tbls.ctypes.data_as(ecglib.u8p), dp[0], cp)
        want2 = oracle.encode_data_update(en[k:], 3, delta, want)
        raw = pbuf.download()
        assert all(np.array_equal(raw[pofs[r]: pofs[r] + n], want2[r]) for r in range(p))
        # xor_gen: the last pointer is the destination
        v = (C.c_void_p * 3)(dbuf.ptr + dofs[1], dbuf.ptr + dofs[2], pbuf.ptr + pofs[0])
        assert L.xor_gen(3, n, v) == 0
        assert np.array_equal(pbuf.download(n, offset=pofs[0]), data[1] ^ data[2])
    finally:
        dbuf.free()
        pbuf.free()


def test_dropin_routes_by_placement_and_size(ecglib, oracle, ctx):
    """SURVEY §8b's rule, observed through ecg_last_kernel: a 4 KiB host-cell
    ec_encode_data runs the CPU path at the default (measured) crossover,
    device cells run the HIP kernel, and a host call above the crossover
    runs the HIP kernel through staging -- same bytes every time."""
    L = ecglib.lib()
    k, p = 8, 2
    en = oracle.cauchy1(k, p)
    tbls = ecglib.isal_init_tables(en[k:])
    small = [rand(4096, 300 + j) for j in range(k)]
    out = [np.zeros(4096, dtype=np.uint8) for _ in range(p)]
    ecglib.isal_encode_data(tbls, k, p, small, out)
    assert ecglib.last_kernel().startswith("cpu:"), ecglib.last_kernel()
    assert np.array_equal(np.stack(out), oracle.encode_data(en[k:], np.stack(small)))
    # device cells of the same call
    dbuf = ctx.to_device(np.stack(small + out))
    try:
        dp = (ecglib.u8p * k)(*[C.cast(C.c_void_p(dbuf.ptr + j * 4096), ecglib.u8p) for j in range(k)])
        cp = (ecglib.u8p * p)(*[C.cast(C.c_void_p(dbuf.ptr + (k + r) * 4096), ecglib.u8p) for r in range(p)])
        L.ec_encode_data(4096, k, p, tbls.ctypes.data_as(ecglib.u8p), dp, cp)
        assert ecglib.last_kernel().startswith("ecg_mm_kernel<8,2"), ecglib.last_kernel()
        got = dbuf.download().reshape(k + p, 4096)
        assert np.array_equal(got[k:], np.stack(out))
    finally:
        dbuf.free()
    # host cells above a crossover of 64 KiB * (k + p)
    old = ecglib.dropin_crossover()
    ecglib.set_dropin_crossover(65536 * (k + p))
    try:
        for n, gpu in ((65536 - 1, False), (65536, True), (1 << 20, True)):
            data = [rand(n, 400 + j) for j in range(k)]
            coding = [np.zeros(n, dtype=np.uint8) for _ in range(p)]
            ecglib.isal_encode_data(tbls, k, p, data, coding)
            assert ecglib.last_kernel().startswith("ecg_mm" if gpu else "cpu:"), (n, ecglib.last_kernel())
            assert np.array_equal(np.stack(coding), oracle.encode_data(en[k:], np.stack(data)))
    finally:
        ecglib.set_dropin_crossover(old)


def test_dropin_routes_after_placement_cache(ecglib, oracle, ctx):
    """The per-thread placement cache remembers only memory HIP does not know
    (plain malloc): interleaving calls on cached malloc cells with pinned host
    cells (ecg_host_alloc) and device cells keeps every call on its own
    route -- pinned host cells take the CPU path at the default crossover and
    the staging above a set one, device cells the kernel -- with oracle
    bytes every time."""
    L = ecglib.lib()
    k, p, n = 4, 2, 8192
    en = oracle.cauchy1(k, p)
    tbls = ecglib.isal_init_tables(en[k:])
    tp = tbls.ctypes.data_as(ecglib.u8p)
    src = np.stack([rand(n, 500 + j) for j in range(k)])
    want = oracle.encode_data(en[k:], src)
    plain = [np.ascontiguousarray(s) for s in src]
    pinned = ctx.host_alloc((k + p) * n)
    dev = ctx.to_device(np.concatenate([src, np.zeros((p, n), np.uint8)]))
    old = ecglib.dropin_crossover()

    def ptrs(base):
        return ((ecglib.u8p * k)(*[C.cast(C.c_void_p(base + j * n), ecglib.u8p) for j in range(k)]),
                (ecglib.u8p * p)(*[C.cast(C.c_void_p(base + (k + r) * n), ecglib.u8p) for r in range(p)]))

    try:
        pinned.array[:] = np.concatenate([src, np.zeros((p, n), np.uint8)]).ravel()
        pd, pc = ptrs(pinned.ptr)
        vd, vc = ptrs(dev.ptr)
        for crossover, pinned_route in ((old, "cpu:"), (0, "ecg_mm")):
            ecglib.set_dropin_crossover(crossover)
            for rnd in range(3):
                out = [np.zeros(n, np.uint8) for _ in range(p)]
                ecglib.isal_encode_data(tbls, k, p, plain, out)
                route = ecglib.last_kernel()
                assert route.startswith("cpu:" if crossover else "ecg_mm"), (crossover, route)
                assert np.array_equal(np.stack(out), want)
                pinned.array[k * n:] = 0
                L.ec_encode_data(n, k, p, tp, pd, pc)
                assert ecglib.last_kernel().startswith(pinned_route), (crossover, ecglib.last_kernel())
                assert np.array_equal(pinned.array[k * n:].reshape(p, n), want)
                L.ec_encode_data(n, k, p, tp, vd, vc)
                assert ecglib.last_kernel().startswith("ecg_mm_kernel<4,2"), ecglib.last_kernel()
                assert np.array_equal(dev.download().reshape(k + p, n)[k:], want)
    finally:
        ecglib.set_dropin_crossover(old)
        dev.free()
        pinned.free()


def test_force_cpu_keeps_device_cells_on_gpu():
    """ECG_FORCE_CPU=1 sends host cells to the CPU path even above the
    crossover, but device cells -- which no CPU can read -- still run the HIP
    kernel."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = r"""
import ctypes as C, sys, numpy as np
sys.path.insert(0, %r)
from daos_amd import ecg
from oracle import ref
ecg.set_dropin_crossover(0)
k, p, n = 4, 2, 8192
en = ref.cauchy1(k, p)
tb = ecg.isal_init_tables(en[k:])
d = np.random.default_rng(3).integers(0, 256, (k, n), dtype=np.uint8)
o = [np.zeros(n, np.uint8) for _ in range(p)]
ecg.isal_encode_data(tb, k, p, list(d), o)
host = ecg.last_kernel()
assert np.array_equal(np.stack(o), ref.encode_data(en[k:], d))
ctx = ecg.Context(0)
buf = ctx.to_device(np.concatenate([d, np.zeros((p, n), np.uint8)]))
dp = (ecg.u8p * k)(*[C.cast(C.c_void_p(buf.ptr + j * n), ecg.u8p) for j in range(k)])
cp = (ecg.u8p * p)(*[C.cast(C.c_void_p(buf.ptr + (k + r) * n), ecg.u8p) for r in range(p)])
ecg.lib().ec_encode_data(n, k, p, tb.ctypes.data_as(ecg.u8p), dp, cp)
dev = ecg.last_kernel()
assert np.array_equal(buf.download().reshape(k + p, n)[k:], np.stack(o))
buf.free(); ctx.close()
print(host, dev)
""" % root
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, ECG_FORCE_CPU="1"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    host, dev = r.stdout.split()
    assert host.startswith("cpu:") and dev.startswith("ecg_mm_kernel<4,2"), (host, dev)


def test_isal_device_cells_16_threads(ecglib, oracle, ctx):
    """16 threads at once calling ec_encode_data on device cells at odd
    offsets (the engine's xstreams, ref:src/engine/ult.c:394-470): calls
    spread over the context's drop-in stream pool and each waits for its own
    launch; every output equals the oracle's."""
    import threading

    L = ecglib.lib()
    T, iters = 16, 6
    errs = []

    def worker(t):
        try:
            k, p = ((4, 2), (8, 2), (16, 3), (8, 3))[t % 4]
            n = 32768 + 7 * t + 1
            en = oracle.cauchy1(k, p)
            tbls = ecglib.isal_init_tables(en[k:])
            slot = n + 64
            buf = ctx.alloc((k + p) * slot)
            try:
                for it in range(iters):
                    data = rand((k, n), 1000 * t + it)
                    offs = [j * slot + 1 + (t + j) % 13 for j in range(k)]
                    pofs = [(k + r) * slot + 3 + r for r in range(p)]
                    for j in range(k):
                        buf.upload(data[j], offset=offs[j])
                    dp = (ecglib.u8p * k)(*[C.cast(C.c_void_p(buf.ptr + o), ecglib.u8p) for o in offs])
                    cp = (ecglib.u8p * p)(*[C.cast(C.c_void_p(buf.ptr + o), ecglib.u8p) for o in pofs])
                    L.ec_encode_data(n, k, p, tbls.ctypes.data_as(ecglib.u8p), dp, cp)
                    raw = buf.download()
                    want = oracle.encode_data(en[k:], data)
                    for r in range(p):
                        if not np.array_equal(raw[pofs[r]: pofs[r] + n], want[r]):
                            errs.append((t, it, r))
            finally:
                buf.free()
        except Exception as e:          # noqa: BLE001 -- reported below
            errs.append((t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs[:5]


def test_isal_device_cells_one_shape_16_threads(ecglib, oracle, ctx):
    """16 threads released together calling ec_encode_data on device cells of
    ONE shape (EC_8P2, same tables and length -- the engine's xstreams
    encoding one class), 12 calls each: every output equals the oracle's and
    every caller's last_kernel names a product kernel."""
    import threading

    L = ecglib.lib()
    T, iters, k, p, n = 16, 12, 8, 2, 65536 + 20
    en = oracle.cauchy1(k, p)
    tbls = ecglib.isal_init_tables(en[k:])
    errs, kernels = [], set()
    bufs = [ctx.alloc((k + p) * (n + 64)) for _ in range(T)]
    start = threading.Barrier(T)

    def worker(t):
        try:
            buf = bufs[t]
            offs = [j * (n + 64) + (t % 5) for j in range(k + p)]
            dp = (ecglib.u8p * k)(*[C.cast(C.c_void_p(buf.ptr + o), ecglib.u8p) for o in offs[:k]])
            cp = (ecglib.u8p * p)(*[C.cast(C.c_void_p(buf.ptr + o), ecglib.u8p) for o in offs[k:]])
            datas = [rand((k, n), 5000 + 100 * t + it) for it in range(iters)]
            start.wait()
            for it in range(iters):
                for j in range(k):
                    buf.upload(datas[it][j], offset=offs[j])
                L.ec_encode_data(n, k, p, tbls.ctypes.data_as(ecglib.u8p), dp, cp)
                kernels.add(ecglib.last_kernel().split("<")[0])
                raw = buf.download()
                want = oracle.encode_data(en[k:], datas[it])
                for r in range(p):
                    if not np.array_equal(raw[offs[k + r]: offs[k + r] + n], want[r]):
                        errs.append((t, it, r))
        except Exception as e:          # noqa: BLE001 -- reported below
            errs.append((t, repr(e)))

    try:
        th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
        for x in th:
            x.start()
        for x in th:
            x.join()
    finally:
        for b in bufs:
            b.free()
    assert not errs, errs[:5]
    assert kernels <= {"ecg_mm_kernel", "ecg_mm_ptr_kernel"} and kernels, kernels


def test_xor_gen_many_device_cells(ecglib, ctx):
    """xor_gen with more sources than one launch takes (ECG_MAX_K = 64) on
    device cells: accumulating launches, not an error."""
    L = ecglib.lib()
    nv, n = 70, 4096 + 3
    srcs = rand((nv - 1, n), 77)
    buf = ctx.alloc(nv * (n + 16))
    try:
        for i in range(nv - 1):
            buf.upload(srcs[i], offset=i * (n + 16) + 1)
        v = (C.c_void_p * nv)(*[buf.ptr + i * (n + 16) + 1 for i in range(nv)])
        assert L.xor_gen(nv, n, v) == 0
        got = buf.download(n, offset=(nv - 1) * (n + 16) + 1)
        assert np.array_equal(got, np.bitwise_xor.reduce(srcs, axis=0))
    finally:
        buf.free()


def test_device_cell_past_allocation_refused(ecglib, ctx):
    """A device cell that runs past the end of its allocation is refused on
    the host (-DER_INVAL) instead of faulting the GPU."""
    L = ecglib.lib()
    buf = ctx.alloc(4 * 4096)
    try:
        coef = np.ones((1, 2), dtype=np.uint8)
        sp = (ecglib.u8p * 2)(C.cast(C.c_void_p(buf.ptr), ecglib.u8p),
                              C.cast(C.c_void_p(buf.ptr + 3 * 4096 + 100), ecglib.u8p))
        dp = (ecglib.u8p * 1)(C.cast(C.c_void_p(buf.ptr + 4096), ecglib.u8p))
        rc = L.ecg_matmul_host(ctx.h, 4096, 2, 1, coef.ctypes.data_as(ecglib.u8p), sp, dp, 0)
        assert rc == -ecglib.DER_INVAL and "past the end" in ecglib.lib().ecg_strerror().decode()
    finally:
        buf.free()


def test_isal_reference_aggregate_pattern(ecglib, oracle, ctx, route):
    """The reference's only byte-level parity test
    (ref:src/tests/suite/daos_aggregate_ec.c:371-395): cell j filled with j
    (or 0x80), TEST_EC_CELL_SZ = 32 KiB, ec_encode_data with the codec tables."""
    L = ecglib.lib()
    assert L.ecg_obj_ec_codec_init() == 0
    for oc, overwrite in (((35 << 24) | 1, False), ((37 << 24) | 2, True), ((32 << 24) | 1, False)):
        kk, pp = C.c_int(), C.c_int()
        L.ecg_obj_ec_class_kp(oc, C.byref(kk), C.byref(pp))
        k, p, ln = kk.value, pp.value, 32768
        codec = C.cast(L.ecg_obj_ec_codec_get(oc), C.POINTER(C.c_void_p))
        tbls_ptr = C.cast(codec[1], C.POINTER(C.c_ubyte))
        tbls = np.ctypeslib.as_array(tbls_ptr, shape=(k * p * 32,)).copy()
        data = [np.full(ln, 0x80 if overwrite else j, dtype=np.uint8) for j in range(k)]
        parity = [np.zeros(ln, dtype=np.uint8) for _ in range(p)]
        ecglib.isal_encode_data(tbls, k, p, data, parity)
        check_route(ecglib, route)
        want = oracle.encode_data(oracle.cauchy1(k, p)[k:], np.stack(data))
        assert all(np.array_equal(parity[r], want[r]) for r in range(p))


# --------------------------------------------------------------- DAOS surface
def test_daos_encode_buf_and_recovery(ecglib, oracle, ctx, route):
    L = ecglib.lib()
    assert L.ecg_obj_ec_codec_init() == 0
    oc = (37 << 24) | 1                 # OC_EC_8P2G1
    k, p, cell = 8, 2, 128 * 1024
    buf = rand(k * cell, 70)
    pbufs = (ecglib.u8p * p)()         # NULL -> allocated by the callee
    assert L.ecg_obj_ec_encode_buf(oc, cell, buf.ctypes.data_as(ecglib.u8p), pbufs) == 0
    check_route(ecglib, route)
    par = np.stack([np.ctypeslib.as_array(pbufs[r], shape=(cell,)).copy() for r in range(p)])
    libc = C.CDLL(None)
    for r in range(p):
        libc.free(C.cast(pbufs[r], C.c_void_p))
    want = oracle.encode_data(oracle.cauchy1(k, p)[k:], buf.reshape(k, cell))
    assert np.array_equal(par, want)

    # recovery codec + obj_ec_recov_data on 4 host stripes
    S = 4
    data = rand((S, k, cell), 71)
    stripes = np.concatenate([data, oracle_parity(oracle, k, p, data).transpose(1, 0, 2)], axis=1).copy()
    broken = stripes.copy()
    err = [1, 9]
    broken[:, err] = 0
    rv = L.ecg_obj_ec_recov_codec_alloc()
    assert rv
    assert L.ecg_obj_ec_recov_codec_init(oc, (C.c_uint32 * 2)(*err), 2, rv) == 0
    assert L.ecg_obj_ec_recov_data(None, rv, cell, broken.ctypes.data_as(ecglib.u8p), S) == 0
    assert np.array_equal(broken, stripes)
    assert L.ecg_obj_ec_recov_codec_init(oc, (C.c_uint32 * 3)(0, 1, 2), 3, rv) == -ecglib.DER_DATA_LOSS
    L.ecg_obj_ec_recov_codec_free(rv)


def test_daos_encode_stripes_and_agg_update(ecglib, oracle, ctx, route):
    L = ecglib.lib()
    oc = (35 << 24) | 1                 # OC_EC_4P2G1
    k, p, cell, S = 4, 2, 32768, 6
    data = rand((S, k, cell), 80)
    par = np.zeros((p, S, cell), dtype=np.uint8)
    assert L.ecg_obj_ec_encode_stripes(None, oc, cell, S, data.ctypes.data_as(ecglib.u8p),
                                       par.ctypes.data_as(ecglib.u8p)) == 0
    assert np.array_equal(par, oracle_parity(oracle, k, p, data))
    # agg_update_parity on stripe 0: cells 1 and 3 replaced
    old = data[0, [1, 3]].copy()
    new = rand((2, cell), 81)
    parity = par[:, 0].copy()
    bitmap = np.array([0b1010], dtype=np.uint8)
    assert L.ecg_agg_update_parity(None, oc, cell, 1, bitmap.ctypes.data_as(ecglib.u8p), 2,
                                   old.ctypes.data_as(ecglib.u8p), new.ctypes.data_as(ecglib.u8p),
                                   None, None, 0, parity.ctypes.data_as(ecglib.u8p)) == 0
    check_route(ecglib, route)
    d2 = data[0].copy()
    d2[[1, 3]] = new
    assert np.array_equal(parity, oracle.encode_data(oracle.cauchy1(k, p)[k:], d2))


# --------------------------------------------------------------- host pipeline
def test_host_pipeline(ctx, oracle):
    k, p, C_, S = 8, 2, 65536, 37
    data = rand((S, k, C_), 90)
    par = np.zeros((p, S, C_), dtype=np.uint8)
    ctx.encode_host(k, p, C_, S, data, par, chunk=8)
    want = oracle_parity(oracle, k, p, data)
    assert np.array_equal(par, want)
    stripes = np.concatenate([data, want.transpose(1, 0, 2)], axis=1).copy()
    broken = stripes.copy()
    broken[:, [2, 8]] = 0
    ctx.recover_host(k, p, C_, S, broken, [2, 8], chunk=5)
    assert np.array_equal(broken, stripes)


@pytest.mark.parametrize("k,p,C_,S", [(8, 2, 1 << 20, 11), (4, 2, 4096 + 16, 9)])
def test_host_pipeline_default_chunk(ctx, oracle, k, p, C_, S):
    """chunk_stripes = 0: the library sizes chunks to ~32 MiB of input cells
    (EC_8P2 1 MiB: 4 stripes, so 11 stripes take 3 chunks with a ragged last
    one; tiny cells: one chunk for the whole batch)."""
    data = rand((S, k, C_), 91 + k)
    par = np.zeros((p, S, C_), dtype=np.uint8)
    ctx.encode_host(k, p, C_, S, data, par)
    want = oracle_parity(oracle, k, p, data)
    assert np.array_equal(par, want)
    stripes = np.concatenate([data, want.transpose(1, 0, 2)], axis=1).copy()
    broken = stripes.copy()
    broken[:, [0, k]] = 0x5A
    ctx.recover_host(k, p, C_, S, broken, [0, k])
    assert np.array_equal(broken, stripes)


@pytest.mark.parametrize("errs", [[0, 1], [8, 9], [1, 2], [9, 8], [3], [7, 8]])
def test_recover_host_erasure_runs(ctx, oracle, errs):
    """Host-resident recovery moves survivors and regenerated cells in runs
    of consecutive cells (one strided copy per run): every erasure shape,
    including runs that straddle the data/parity boundary."""
    k, p, C_, S = 8, 2, 8192 + 64, 11
    data = rand((S, k, C_), 95 + sum(errs))
    want = oracle_parity(oracle, k, p, data)
    stripes = np.concatenate([data, want.transpose(1, 0, 2)], axis=1).copy()
    broken = stripes.copy()
    broken[:, errs] = 0x5A
    ctx.recover_host(k, p, C_, S, broken, errs, chunk=4)
    assert np.array_equal(broken, stripes)


# --------------------------------------------------------------- batching facade
def test_queue_batches_concurrent_one_stripe_calls(ctx, oracle, ecglib, route):
    """8 threads x 40 one-stripe EC_8P2 encodes (the reference's calling
    pattern) complete bit-exact -- host cells computed on the completion
    threads (below the drop-in crossover, route "cpu": nothing crosses PCIe)
    or staged through the device and coalesced into far fewer batches
    (crossover 0, route "gpu")."""
    import threading

    k, p, C_ = 8, 2, 32768
    h2d0 = ctx.stats()["h2d_bytes"]
    q = ecglib.Queue(ctx, max_batch=64, max_wait_us=2000)
    en = oracle.cauchy1(k, p)
    jobs = {}
    for t in range(8):                 # inputs ready before the burst of calls
        for i in range(40):
            rid = t * 1000 + i
            jobs[rid] = ([rand(C_, rid * 16 + j) for j in range(k)], [np.zeros(C_, dtype=np.uint8) for _ in range(p)])

    def worker(t):
        for i in range(40):
            rid = t * 1000 + i
            q.encode(rid, k, p, *jobs[rid])

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    q.flush()
    nreq, nbatch = q.stats()
    assert nreq == 320 and len(q.done) == 320
    assert all(rc == 0 for rc in q.done.values())
    # staged batches coalesce; CPU-route batches close whenever a completion
    # thread idles (batching buys the CPU nothing then)
    assert nbatch < nreq / 4 if route == "gpu" else nbatch <= nreq, (nreq, nbatch)
    for rid, (data, par) in jobs.items():
        want = oracle.encode_data(en[k:], np.stack(data))
        assert np.array_equal(np.stack(par), want), rid
    q.close()
    h2d = ctx.stats()["h2d_bytes"] - h2d0
    assert (h2d == 0) if route == "cpu" else (h2d == 320 * k * C_), (route, h2d)


def test_queue_mixed_classes_and_recovery(ctx, oracle, ecglib, route):
    """Interleaved encode 4P2 / encode 8P3 (odd cell size) / recover with two
    different erasure sets: each class batched separately, all bit-exact, on
    either host-cell route."""
    q = ecglib.Queue(ctx, max_batch=16, max_wait_us=100)
    checks = []
    rid = 0
    for i in range(24):
        kind = i % 4
        if kind == 0:
            k, p, C_ = 4, 2, 4096
        elif kind == 1:
            k, p, C_ = 8, 3, 933
        else:
            k, p, C_ = 4, 2, 8192
        data = rand((k, C_), 7000 + i)
        en = oracle.cauchy1(k, p)
        par = oracle.encode_data(en[k:], data)
        if kind < 2:
            outp = [np.zeros(C_, dtype=np.uint8) for _ in range(p)]
            q.encode(rid, k, p, list(data), outp)
            checks.append((rid, lambda outp=outp, par=par: np.array_equal(np.stack(outp), par)))
        else:
            stripe = np.concatenate([data, par]).copy()
            err = [0, 5] if kind == 2 else [3]
            broken = stripe.copy()
            broken[err] = 0
            q.recover(rid, k, p, broken, err)
            checks.append((rid, lambda broken=broken, stripe=stripe: np.array_equal(broken, stripe)))
        rid += 1
    q.flush()
    for r, ok in checks:
        assert q.done[r] == 0 and ok(), r
    nreq, nbatch = q.stats()
    assert nreq == 24 and nbatch >= 4
    q.close()


def test_queue_device_cells_batched_in_place(ctx, oracle, ecglib):
    """Device-cell requests (an engine whose buffers live in HBM): 8 threads x
    24 one-stripe EC_8P2 encodes and {d0, d9} recoveries on device stripes --
    some at odd byte offsets -- interleaved with host-cell encodes in the
    same queue.  Device batches are pointer-table launches on the cells in
    place; every byte equals the oracle's."""
    import threading

    k, p, C_, per = 8, 2, 32768 + 40, 24
    en = oracle.cauchy1(k, p)
    T = 8
    S = T * per
    slot = (k + p) * C_ + 64
    data = rand((S, k, C_), 8100)
    par = np.stack([oracle.encode_data(en[k:], data[s]) for s in range(S)])          # [S][p][C]
    skew = [(s * 7) % 16 for s in range(S)]
    img = np.zeros(S * slot, dtype=np.uint8)
    for s in range(S):
        base = s * slot + skew[s]
        img[base: base + k * C_] = data[s].reshape(-1)
        if s % 2:                      # recovery stripes: parity present, d0 and d9 erased below
            img[base + k * C_: base + (k + p) * C_] = par[s].reshape(-1)
            img[base: base + C_] = 0
            img[base + (k + 1) * C_: base + (k + 2) * C_] = 0
    dbuf = ctx.to_device(img)
    q = ecglib.Queue(ctx, max_batch=64, max_wait_us=100000)
    host_jobs = {}
    try:
        def worker(t):
            for i in range(per):
                s = t * per + i
                base = dbuf.ptr + s * slot + skew[s]
                if s % 2:
                    q.recover_ptr(s, k, p, C_, base, [0, 9])
                else:
                    q.encode_ptrs(s, k, p, C_, [base + j * C_ for j in range(k)],
                                  [base + (k + r) * C_ for r in range(p)])
                if i % 6 == 0:         # a host-cell request of the same class in between
                    rid = 100000 + s
                    hd = [rand(C_, rid + j) for j in range(k)]
                    ho = [np.zeros(C_, dtype=np.uint8) for _ in range(p)]
                    host_jobs[rid] = (hd, ho)
                    q.encode(rid, k, p, hd, ho)

        th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        q.flush()
        nreq, nbatch = q.stats()
        assert nreq == S + len(host_jobs) and all(rc == 0 for rc in q.done.values()), q.done
        # device batches launch whenever the device is idle and host-cell
        # (CPU-route) batches whenever a completion thread is (latency first),
        # so only requests that arrive while work runs coalesce
        assert nbatch <= nreq, (nreq, nbatch)
        got = dbuf.download()
        for s in range(S):
            base = s * slot + skew[s]
            stripe = got[base: base + (k + p) * C_].reshape(k + p, C_)
            assert np.array_equal(stripe[:k], data[s]), s
            assert np.array_equal(stripe[k:], par[s]), s
        for rid, (hd, ho) in host_jobs.items():
            assert np.array_equal(np.stack(ho), oracle.encode_data(en[k:], np.stack(hd))), rid
    finally:
        q.close()
        dbuf.free()


def test_queue_device_cell_alone_launches_at_once(ctx, oracle, ecglib):
    """A lone device-cell request does not wait max_wait_us for company: its
    slot closes as soon as the device has no batch of the queue in flight."""
    import time

    k, p, C_ = 4, 2, 65536
    data = rand((k, C_), 8200)
    dbuf = ctx.to_device(np.concatenate([data, np.zeros((p, C_), np.uint8)]))
    q = ecglib.Queue(ctx, max_batch=256, max_wait_us=5000000)      # host classes would wait 5 s
    try:
        t0 = time.perf_counter()
        q.encode_ptrs(1, k, p, C_, [dbuf.ptr + j * C_ for j in range(k)],
                      [dbuf.ptr + (k + r) * C_ for r in range(p)])
        while 1 not in q.done and time.perf_counter() - t0 < 2.0:
            time.sleep(0.0005)
        assert q.done.get(1) == 0, "not completed within 2 s"
        assert time.perf_counter() - t0 < 1.0
        got = dbuf.download().reshape(k + p, C_)
        assert np.array_equal(got[k:], oracle.encode_data(oracle.cauchy1(k, p)[k:], data))
    finally:
        q.close()
        dbuf.free()


def test_queue_host_cell_alone_closes_at_once(ctx, oracle, ecglib):
    """A lone host-cell request on the CPU route (default crossover) does not
    wait max_wait_us either: its batch closes while a completion thread is
    free and it is the queue's only work.  On the staged route (crossover 0)
    the same request waits for company, up to max_wait_us."""
    import time

    k, p, C_ = 4, 2, 65536
    data = rand((k, C_), 8300)
    old = ecglib.dropin_crossover()
    try:
        for cross, wait_ok in (((1 << 64) - 1, lambda dt: dt < 1.0), (0, lambda dt: dt >= 0.2)):
            ecglib.set_dropin_crossover(cross)
            q = ecglib.Queue(ctx, max_batch=256, max_wait_us=300000)      # 0.3 s for company
            par = [np.zeros(C_, np.uint8) for _ in range(p)]
            try:
                t0 = time.perf_counter()
                q.encode(1, k, p, list(data), par)
                while 1 not in q.done and time.perf_counter() - t0 < 3.0:
                    time.sleep(0.0005)
                dt = time.perf_counter() - t0
                assert q.done.get(1) == 0, ("not completed", cross)
                assert wait_ok(dt), (cross, dt)
                assert np.array_equal(np.stack(par), oracle.encode_data(oracle.cauchy1(k, p)[k:], data))
            finally:
                q.close()
    finally:
        ecglib.set_dropin_crossover(old)


def test_queue_device_cell_errors(ctx, ecglib):
    """Device cells: a request mixing host and device cells (an update whose
    old cell is host memory), a cell running past its allocation and more than
    16 data cells are refused (-DER_INVAL) -- before anything reaches the GPU."""
    L = ecglib.lib()
    k, p, C_ = 8, 2, 4096
    dbuf = ctx.alloc((k + p) * C_)
    q = ecglib.Queue(ctx)
    try:
        dp = (ecglib.u8p * p)(*[C.cast(C.c_void_p(dbuf.ptr + (k + r) * C_), ecglib.u8p) for r in range(p)])
        host_old = np.zeros(C_, dtype=np.uint8)
        new = C.cast(C.c_void_p(dbuf.ptr + C_), ecglib.u8p)
        rc = L.ecg_queue_update(q.h, k, p, C_, 0, host_old.ctypes.data_as(ecglib.u8p), new, dp, None, None)
        assert rc == -ecglib.DER_INVAL, rc
        assert "host memory" in L.ecg_strerror().decode(), L.ecg_strerror()
        sp = (ecglib.u8p * k)(*[C.cast(C.c_void_p(dbuf.ptr + j * C_ + (C_ // 2 if j == k - 1 else 0)),
                                       ecglib.u8p) for j in range(k)])
        dp_bad = (ecglib.u8p * p)(*[C.cast(C.c_void_p(dbuf.ptr + (k + p) * C_ - C_ // 2 if r == p - 1 else
                                                      dbuf.ptr + (k + r) * C_), ecglib.u8p) for r in range(p)])
        rc = L.ecg_queue_encode(q.h, k, p, C_, sp, dp_bad, None, None)
        assert rc == -ecglib.DER_INVAL, rc
        big = ctx.alloc(20 * C_)
        try:
            sp20 = (ecglib.u8p * 18)(*[C.cast(C.c_void_p(big.ptr + j * C_), ecglib.u8p) for j in range(18)])
            dp20 = (ecglib.u8p * 2)(*[C.cast(C.c_void_p(big.ptr + (18 + r) * C_), ecglib.u8p) for r in range(2)])
            rc = L.ecg_queue_encode(q.h, 18, 2, C_, sp20, dp20, None, None)
            assert rc == -ecglib.DER_INVAL, rc
        finally:
            big.free()
        q.flush()
        assert q.stats()[0] == 0
    finally:
        q.close()
        dbuf.free()


def test_queue_destroy_drains(ctx, oracle, ecglib, route):
    k, p, C_ = 2, 1, 4096
    q = ecglib.Queue(ctx, max_batch=1000, max_wait_us=1000000)   # would wait 1 s for company
    data = [rand(C_, 1), rand(C_, 2)]
    par = [np.zeros(C_, dtype=np.uint8)]
    q.encode(1, k, p, data, par)
    keep = q.done
    q.close()                       # must drain: callback runs before destroy returns
    assert keep.get(1) == 0
    assert np.array_equal(par[0], oracle.encode_data(oracle.cauchy1(k, p)[k:], np.stack(data))[0])



# --------------------------------------------------------------- aggregation / single value
def _u64(seq):
    return (C.c_uint64 * max(1, len(seq)))(*seq)


@pytest.mark.parametrize("exts", [
    [],                                   # n_ext = 0: no hole processing
    [(2 * 64 + 5, 10), (2 * 64 + 30, 4)],  # holes before, between and after (cell 2)
    [(0, 3 * 64)],                        # covers cells 0-2 entirely
    [(3 * 64 + 60, 40)],                  # overruns cell 3's end: no tail zeroing
    [(7 * 64, 8)],                        # touches no updated cell -> whole diffs kept
])
def test_agg_update_parity_holes(ctx, oracle, ecglib, exts, route):
    """agg_update_parity + agg_diff_preprocess semantics, including the
    reference's rules for cells no extent touches (ref:src/object/
    srv_ec_aggregate.c:1006-1105), vs the oracle restatement."""
    L = ecglib.lib()
    oc = (37 << 24) | 1                      # EC_8P2
    k, p, recs, rsize = 8, 2, 64, 8          # 512-byte cells
    cb = recs * rsize
    bitmap = bytes([0b00001110])             # cells 1, 2, 3 updated
    old = rand((3, cb), 90)
    new = rand((3, cb), 91)
    parity = rand((p, cb), 92)
    want = oracle.agg_update_parity(k, p, recs, rsize, bitmap, old, new, exts, parity)
    got = parity.copy()
    bm = np.frombuffer(bitmap, dtype=np.uint8).copy()
    rc = L.ecg_agg_update_parity(None, oc, recs, rsize, bm.ctypes.data_as(ecglib.u8p), 3,
                                 old.ctypes.data_as(ecglib.u8p), new.ctypes.data_as(ecglib.u8p),
                                 _u64([e[0] for e in exts]) if exts else None,
                                 _u64([e[1] for e in exts]) if exts else None, len(exts),
                                 got.ctypes.data_as(ecglib.u8p))
    assert rc == 0
    check_route(ecglib, route)
    assert np.array_equal(got, want)


def test_agg_recalc_parity(ctx, oracle, ecglib, route):
    L = ecglib.lib()
    oc = (41 << 24) | 1                      # EC_8P3
    k, p, cb = 8, 3, 4096 + 8
    bitmap = np.array([0b10010110], dtype=np.uint8)     # cells 1,2,4,7 from peers
    rbuf = rand((4, cb), 93)
    lbuf = rand((4, cb), 94)
    parity = np.zeros((p, cb), dtype=np.uint8)
    assert L.ecg_agg_recalc_parity(None, oc, cb, bitmap.ctypes.data_as(ecglib.u8p), 4,
                                   rbuf.ctypes.data_as(ecglib.u8p), lbuf.ctypes.data_as(ecglib.u8p),
                                   parity.ctypes.data_as(ecglib.u8p)) == 0
    check_route(ecglib, route)
    data = np.stack([rbuf[[1, 2, 4, 7].index(j)] if j in (1, 2, 4, 7) else lbuf[[0, 3, 5, 6].index(j)]
                     for j in range(k)])
    assert np.array_equal(parity, oracle.encode_data(oracle.cauchy1(k, p)[k:], data))


@pytest.mark.parametrize("oc,size", [((32 << 24) | 1, 8569), ((35 << 24) | 1, 8569), ((37 << 24) | 1, 8569),
                                     ((42 << 24) | 1, 8569), ((35 << 24) | 1, 4 * 1048576 + 347),
                                     ((39 << 24) | 1, 65536 + 3)])
def test_singv_encode(ctx, oracle, ecglib, oc, size, route):
    """Single values of the reference's test sizes (LARGE_SINGLE_VALUE_SIZE
    8569, DATA_SIZE 4 MiB + 347; ref:src/tests/suite/daos_rebuild_common.c:
    654-658): zero-padded last cell, parity vs the oracle restatement."""
    L = ecglib.lib()
    kk, pp = C.c_int(), C.c_int()
    L.ecg_obj_ec_class_kp(oc, C.byref(kk), C.byref(pp))
    k, p = kk.value, pp.value
    cb = L.ecg_obj_ec_singv_cell_bytes(oc, size)
    assert cb == oracle.singv_cell_bytes(size, k)
    value = rand(size, size)
    pbufs = (ecglib.u8p * p)()
    assert L.ecg_obj_ec_singv_encode(oc, size, value.ctypes.data_as(ecglib.u8p), pbufs) == 0
    check_route(ecglib, route)
    got = np.stack([np.ctypeslib.as_array(pbufs[r], shape=(cb,)).copy() for r in range(p)])
    libc = C.CDLL(None)
    for r in range(p):
        libc.free(C.cast(pbufs[r], C.c_void_p))
    assert np.array_equal(got, oracle.singv_encode(k, p, value))
