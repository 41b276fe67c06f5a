"""GPU parity of the product kernels at every operand alignment.

The product kernels pick their lane access per launch from the common
alignment of every cell address (ecg_mm_dev.h align_granule): dwordx4 lanes
when all are 16-byte aligned; dword lanes (g4) for 8- and 4-byte alignment
(DAOS rounds its parity rows to 8 bytes, ref:src/object/cli_ec.c:86); dword
lanes whose source dwords are funnel-shifted out of aligned loads (g1: user
sgl cells carry no alignment, ref:src/object/cli_ec.c:510-536, while DAOS
allocates the parity aligned); for k = 8, sources off a 16-byte boundary
run 16-byte lanes funnel-shifted out of dword-aligned loads (g2);
destinations at any byte take the same lanes' stores as misaligned dwords
(the hardware's unaligned access mode).  Every case is compared byte for byte with the oracle, and
the test asserts which kernel ran.  Offsets 1, 4, 8 and 12 of the data and/or parity bases, cells whose last
4 KiB column is partial, and cell sizes that are not multiples of 4 / 16.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def rand(shape, seed):
    return np.random.default_rng(seed).integers(0, 256, shape, dtype=np.uint8)


def granule(*vals):
    bits = 0
    for v in vals:
        bits |= v
    return 16 if bits % 16 == 0 else 8 if bits % 8 == 0 else 4 if bits % 4 == 0 else 1


def launch_granule(src_vals, dst_vals, k=0, rows=0, acc=False):
    """ecg_mm_dev.h align_granule + ecg_k_launch_matmul: the lanes a launch
    runs, from its source / destination base offsets, cell offsets and
    strides.  16 / 4: dwordx4 / dword lanes (8-byte alignment runs the dword
    lanes); 1: a source at any byte (funnel-shifted loads); 2: k = 8 (rows
    1-3, no accumulate) with a source off a 16-byte boundary (16-byte lanes,
    funnel-shifted).  Destinations at any byte take the lanes' stores as
    misaligned dwords; the byte kernel (0) is never chosen."""
    gs, gd = granule(*src_vals), granule(*dst_vals)
    if gs < 16 and k == 8 and 1 <= rows <= 3 and not acc:
        return 2
    return 1 if gs < 4 else 16 if gs == gd == 16 else 4


def expect_kernel(name, g, k, rows):
    if g == 0:
        assert name == "ecg_mm_byte_kernel", name
    elif g == 16:
        assert name.startswith("ecg_mm_kernel<") and ",g" not in name, name
    else:
        assert name.startswith("ecg_mm_kernel<") and name.endswith(f",g{g}>"), name


def oracle_parity(oracle, k, p, data):
    en = oracle.cauchy1(k, p)
    return np.stack([oracle.encode_data(en[k:], data[s]) for s in range(data.shape[0])], axis=1)


CELLS = [65536, 2 * 4096 + 1024 + 8, 3 * 4096 + 20, 4096 + 13]


@pytest.mark.parametrize("C_", CELLS)
@pytest.mark.parametrize("doff,poff", [(1, 0), (4, 0), (8, 0), (12, 0), (0, 1), (0, 4), (0, 8), (0, 12),
                                       (8, 8), (4, 12), (12, 8)])
def test_encode_offsets(ctx, oracle, ecglib, C_, doff, poff):
    """Client-layout encode (data [S][k][C] -> parity [p][S][C]) with the data
    and parity bases at byte offsets: the launch runs the 16 / g4 / g1 lanes
    as the addresses allow, with the oracle's parity."""
    k, p, S = 8, 2, 3
    data = rand((S, k, C_), C_ + doff * 16 + poff)
    d = ctx.alloc(data.nbytes + 64)
    d.upload(data.reshape(-1), offset=doff)
    pitch = S * C_ + 8
    par = ctx.alloc(p * pitch + 64)
    par.fill(0xEE)
    try:
        ctx.encode(k, p, C_, S, d.ptr + doff, k * C_, par.ptr + poff, pitch, C_)
        ctx.sync()
        expect_kernel(ecglib.last_kernel(), launch_granule((doff, k * C_, C_), (poff, pitch, C_), k, p), k, p)
        raw = par.download()
        got = np.stack([raw[poff + r * pitch: poff + r * pitch + S * C_].reshape(S, C_) for r in range(p)])
        assert np.array_equal(got, oracle_parity(oracle, k, p, data))
        # nothing written between or after the rows
        assert (raw[:poff] == 0xEE).all()
        for r in range(p):
            assert (raw[poff + r * pitch + S * C_: poff + (r + 1) * pitch] == 0xEE).all()
    finally:
        d.free()
        par.free()


@pytest.mark.parametrize("k,p", [(2, 1), (4, 2), (8, 2), (8, 3), (16, 2), (16, 3)])
@pytest.mark.parametrize("off", [4, 8, 1])
def test_encode_classes_at_offset(ctx, oracle, ecglib, k, p, off):
    """Every specialised (k, p) has g4 (4- or 8-byte aligned operands) and g1
    instantiations (g1: the data cells at a byte offset, the parity
    dword-aligned); k = 8 runs g2 for both."""
    S, C_ = 4, 8192 + 4096
    data = rand((S, k, C_), k * 10 + p + off)
    d = ctx.alloc(data.nbytes + 64)
    d.upload(data.reshape(-1), offset=off)
    par = ctx.alloc(p * S * C_ + 64)
    poff = 0 if off == 1 else off
    try:
        ctx.encode(k, p, C_, S, d.ptr + off, k * C_, par.ptr + poff, S * C_, C_)
        ctx.sync()
        name = ecglib.last_kernel()
        g = 2 if k == 8 else min(off, 4)
        assert name.startswith(f"ecg_mm_kernel<{k},{p},") and name.endswith(f",g{g}>"), name
        got = par.download(p * S * C_, offset=poff).reshape(p, S, C_)
        assert np.array_equal(got, oracle_parity(oracle, k, p, data))
    finally:
        d.free()
        par.free()


@pytest.mark.parametrize("off", [1, 4, 8, 12])
@pytest.mark.parametrize("C_", [32768, 4096 * 5 + 8, 4096 + 12])
@pytest.mark.parametrize("errs", [[0, 1], [3, 9], [8]])
def test_recover_in_place_at_offset(ctx, oracle, ecglib, off, C_, errs):
    """Degraded-read recovery in place in [S][k+p][C] at an image offset."""
    k, p, S = 8, 2, 3
    data = rand((S, k, C_), off + C_ + len(errs))
    stripes = np.concatenate([data, oracle_parity(oracle, k, p, data).transpose(1, 0, 2)], axis=1)
    broken = stripes.copy()
    broken[:, errs] = 0x5A
    d = ctx.alloc(stripes.nbytes + 64)
    d.upload(broken.reshape(-1), offset=off)
    try:
        ctx.recover(k, p, C_, S, d.ptr + off, (k + p) * C_, errs)
        ctx.sync()
        vals = (off, (k + p) * C_, C_)             # in place: sources and destinations alike
        expect_kernel(ecglib.last_kernel(), launch_granule(vals, vals, k, len(errs)), k, len(errs))
        got = d.download(stripes.nbytes, offset=off).reshape(S, k + p, C_)
        assert np.array_equal(got, stripes)
    finally:
        d.free()


@pytest.mark.parametrize("off", [1, 4, 8, 12])
def test_update_at_offset(ctx, oracle, ecglib, off):
    """Delta parity update (ACC + DIFF, the runtime-shaped kernel) with the
    old/new cells and the parity at an offset."""
    k, p, C_, S = 8, 2, 6000 + 8, 3
    cells = [0, 5]
    en = oracle.cauchy1(k, p)
    data = rand((S, k, C_), 31 + off)
    par = oracle_parity(oracle, k, p, data)
    new = rand((S, len(cells), C_), 32 + off)
    old = data[:, cells].copy()
    dold, dnew, dpar = ctx.alloc(old.nbytes + 64), ctx.alloc(new.nbytes + 64), ctx.alloc(par.nbytes + 64)
    dold.upload(old.reshape(-1), offset=off)
    dnew.upload(new.reshape(-1), offset=off)
    dpar.upload(par.reshape(-1), offset=off)
    try:
        ctx.update(k, p, C_, S, cells, dold.ptr + off, dnew.ptr + off, len(cells) * C_, dpar.ptr + off, S * C_, C_)
        ctx.sync()
        got = dpar.download(par.nbytes, offset=off).reshape(p, S, C_)
        data[:, cells] = new
        assert np.array_equal(got, oracle_parity(oracle, k, p, data))
        name = ecglib.last_kernel()
        g = launch_granule((off, C_, len(cells) * C_), (off, S * C_, C_))   # the parity is read and written (ACC)
        assert name.endswith(f",1,1,g{g}>") if g < 16 else name.endswith(",1,1>"), name
    finally:
        for b in (dold, dnew, dpar):
            b.free()


@pytest.mark.parametrize("off", [4, 8])
@pytest.mark.parametrize("k,rows", [(5, 4), (12, 6), (33, 2)])
def test_generic_shapes_at_offset(ctx, oracle, ecglib, off, k, rows):
    """Runtime-shaped kernels (and k > 16 split into accumulating launches)
    at 4 / 8-byte aligned operands."""
    S, C_ = 3, 4096 + 512
    coef = rand((rows, k), 77 + k)
    data = rand((S, k, C_), 78 + rows)
    d = ctx.alloc(data.nbytes + 64)
    d.upload(data.reshape(-1), offset=off)
    out = ctx.alloc(S * rows * C_ + 64)
    try:
        ctx.matmul(coef, C_, S, d.ptr + off, [j * C_ for j in range(k)], k * C_, out.ptr + off,
                   [r * C_ for r in range(rows)], rows * C_, 0)
        ctx.sync()
        assert ecglib.last_kernel().endswith(",g4>"), ecglib.last_kernel()
        got = out.download(S * rows * C_, offset=off).reshape(S, rows, C_)
        for s in range(S):
            assert np.array_equal(got[s], oracle.encode_data(coef, data[s]))
    finally:
        d.free()
        out.free()


@pytest.mark.parametrize("off", [1, 2, 3, 5])
def test_update_unaligned_cells_aligned_parity(ctx, oracle, ecglib, off):
    """Aggregation delta update with the old / new cells at a byte offset and
    the parity dword-aligned: the ACC + DIFF runtime kernel with
    funnel-shifted loads of both sources (g1)."""
    k, p, C_, S = 8, 2, 3 * 4096 + 44, 3
    cells = [1, 6]
    data = rand((S, k, C_), 41 + off)
    par = oracle_parity(oracle, k, p, data)
    new = rand((S, len(cells), C_), 42 + off)
    old = data[:, cells].copy()
    dold, dnew = ctx.alloc(old.nbytes + 64), ctx.alloc(new.nbytes + 64)
    dold.upload(old.reshape(-1), offset=off)
    dnew.upload(new.reshape(-1), offset=(off * 3) % 7)
    dpar = ctx.to_device(par)
    try:
        ctx.update(k, p, C_, S, cells, dold.ptr + off, dnew.ptr + (off * 3) % 7, len(cells) * C_, dpar.ptr,
                   S * C_, C_)
        ctx.sync()
        assert ecglib.last_kernel().endswith(",1,1,g1>"), ecglib.last_kernel()
        got = dpar.download().reshape(p, S, C_)
        data[:, cells] = new
        assert np.array_equal(got, oracle_parity(oracle, k, p, data))
    finally:
        for b in (dold, dnew, dpar):
            b.free()


def test_unaligned_access_served(ctx):
    """The context's start-up probe (ecg_k_unaligned_check: misaligned dword
    loads and stores by 4 lanes) found them served on this MI355X, so
    misaligned destinations run on the vector lanes."""
    assert ctx.unaligned_ok()


CHILD_NO_UNALIGNED = r'''
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from daos_amd import ecg
from oracle import ref as oracle
ctx = ecg.Context(0)
assert not ctx.unaligned_ok()
k, p, C, S = 8, 2, 3 * 4096 + 20, 3
rng = np.random.default_rng(9)
data = rng.integers(0, 256, (S, k, C), dtype=np.uint8)
en = oracle.cauchy1(k, p)
want = np.stack([oracle.encode_data(en[k:], data[s]) for s in range(S)])      # [S][p][C]
for doff, poff, kern in ((0, 0, "ecg_mm_kernel<8,2,0,0,g4>"), (0, 1, "ecg_mm_byte_kernel"),
                         (1, 0, "ecg_mm_byte_kernel"), (4, 8, "ecg_mm_kernel<8,2,0,0,g4>")):
    d = ctx.alloc(data.nbytes + 64)
    d.upload(data.reshape(-1), offset=doff)
    par = ctx.alloc(p * S * C + 64)
    ctx.encode(k, p, C, S, d.ptr + doff, k * C, par.ptr + poff, S * C, C)
    ctx.sync()
    assert ecg.last_kernel() == kern, (doff, poff, ecg.last_kernel())
    got = par.download(p * S * C, offset=poff).reshape(p, S, C).transpose(1, 0, 2)
    assert np.array_equal(got, want), (doff, poff)
    # the pointer-table path: stripes listed as 1, 0, 2 (not an affine table)
    cells = []
    for s in (1, 0, 2):
        cells += [d.ptr + doff + (s * k + j) * C for j in range(k)]
        cells += [par.ptr + poff + r * S * C + s * C for r in range(p)]
    ctx.matmul_ptrs(k, p, en[k:], C, S, cells)
    ctx.sync()
    assert (ecg.last_kernel() == "ecg_mm_ptr_byte_kernel") == (doff % 4 != 0 or poff % 4 != 0), ecg.last_kernel()
    got = par.download(p * S * C, offset=poff).reshape(p, S, C).transpose(1, 0, 2)
    assert np.array_equal(got, want), ("ptr", doff, poff)
    d.free()
    par.free()
print("OK")
'''


def test_no_unaligned_access_takes_byte_kernels():
    """A device that does not serve misaligned dwords (forced with
    ECG_UNALIGNED=0): launches whose sources or destinations are off a dword
    boundary run the byte kernels, the rest the vector lanes; every output
    equals the oracle's.  In a child process (the flag is read at context
    creation)."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, ECG_UNALIGNED="0")
    r = subprocess.run([sys.executable, "-c", CHILD_NO_UNALIGNED, root], capture_output=True, text=True, env=env,
                       timeout=110)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout + r.stderr
