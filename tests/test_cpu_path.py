"""The product's CPU path (daos_amd/csrc/host/ecg_cpu.c) and the drop-in's
routing without a GPU -- no GPU needed.

ISA-L's data-plane calls are `void` and succeed on any CPU; DAOS calls them
from libdaos on client nodes that have no GPU (ref:src/object/SConscript:
19-23, ref:src/object/cli_ec.c:540).  So: every SIMD variant of the CPU path
equals the scalar oracle byte for byte (ragged lengths, odd alignments,
more than 8 rows, more than 32 sources, accumulate), and in a process with
HIP_VISIBLE_DEVICES="" the ISA-L and DAOS surfaces run it instead of
aborting (tests/dropin_nogpu.py)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
ISAS = ["avx512-gfni", "avx2-gfni", "avx2", "scalar"]


def rand(shape, seed):
    return np.random.default_rng(seed).integers(0, 256, shape, dtype=np.uint8)


@pytest.fixture
def isa(ecglib, request):
    yield
    ecglib.cpu_set_isa("auto")


@pytest.mark.parametrize("name", ISAS)
@pytest.mark.parametrize("k,rows", [(2, 1), (4, 2), (8, 2), (8, 3), (16, 3), (1, 1), (5, 9), (33, 2), (64, 8),
                                    (70, 1)])
def test_cpu_variants_match_oracle(ecglib, oracle, isa, name, k, rows):
    if ecglib.cpu_set_isa(name) != 0:
        pytest.skip(f"this CPU has no {name}")
    rng = np.random.default_rng(k * 31 + rows)
    for ln in (1, 31, 63, 64, 65, 127, 4096 + 37, 65536 + 5):
        coef = rng.integers(0, 256, (rows, k), dtype=np.uint8)
        off = int(rng.integers(0, 16))
        src = [np.zeros(ln + 16, dtype=np.uint8)[off: off + ln] for _ in range(k)]
        for j, s in enumerate(src):
            s[:] = rand(ln, 7 * j + ln)
        dst = [np.zeros(ln + 16, dtype=np.uint8)[3: 3 + ln] for _ in range(rows)]
        ecglib.cpu_matmul(coef, src, dst)
        want = oracle.encode_data(coef, np.stack(src))
        assert np.array_equal(np.stack(dst), want), (name, k, rows, ln)
        assert ecglib.last_kernel() == f"cpu:{name}"
        # accumulate: dst ^= product
        prev = [d.copy() for d in dst]
        ecglib.cpu_matmul(coef, src, dst, ecglib.F_ACCUMULATE)
        assert all(not d.any() for d in dst) and all(p.any() or ln < 4 for p in prev)


def test_cpu_xor_only_and_zero_coefficients(ecglib, oracle, isa):
    """All-ones coefficients (xor_gen) take the XOR-only loop; zero
    coefficients contribute nothing."""
    for name in ISAS:
        if ecglib.cpu_set_isa(name) != 0:
            continue
        src = [rand(1000, 60 + j) for j in range(5)]
        dst = [np.full(1000, 0x5A, dtype=np.uint8)]
        ecglib.cpu_matmul(np.ones((1, 5), dtype=np.uint8), src, dst)
        assert np.array_equal(dst[0], np.bitwise_xor.reduce(np.stack(src)))
        ecglib.cpu_matmul(np.zeros((1, 5), dtype=np.uint8), src, dst)
        assert not dst[0].any()


def test_cpu_bad_arguments(ecglib):
    a = [np.zeros(16, dtype=np.uint8)]
    with pytest.raises(ecglib.EcgError):
        ecglib.cpu_matmul(np.ones((1, 400), dtype=np.uint8), a * 400, a)
    assert ecglib.cpu_set_isa("sse9") == -ecglib.DER_INVAL


def test_dropin_without_gpu():
    """ec_encode_data / ec_encode_data_update / xor_gen and the synchronous
    DAOS calls in a process that sees no GPU: CPU path, oracle bytes, no
    abort."""
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "dropin_nogpu.py")], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["ok"] and res["cases"] > 150
    assert all(k.startswith("cpu:") for k in res["kernels"])


def test_force_cpu_env():
    """ECG_FORCE_CPU=1 keeps host cells on the CPU even where a GPU exists
    (here: none, so this checks the switch is read without side effects)."""
    code = ("import numpy as np; from daos_amd import ecg; from oracle import ref; "
            "tb = ecg.isal_init_tables(ref.cauchy1(4, 2)[4:]); d = [np.full(100, j + 1, np.uint8) for j in range(4)]; "
            "o = [np.zeros(100, np.uint8) for _ in range(2)]; ecg.isal_encode_data(tb, 4, 2, d, o); "
            "assert (o[0] == 0x48).all() and (o[1] == 0x0f).all(); print(ecg.last_kernel())")
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, ECG_FORCE_CPU="1"), cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().startswith("cpu:")


def test_cpu_random_shapes(ecglib, oracle, isa):
    """Seeded random calls of every variant: k 1..80, rows 1..12, lengths
    1 byte..20 KiB, every cell at its own byte offset, overwrite or
    accumulate -- bytes equal to the scalar oracle's."""
    rng = np.random.default_rng(0xC9)
    for name in ISAS:
        if ecglib.cpu_set_isa(name) != 0:
            continue
        for _ in range(40):
            k, rows = int(rng.integers(1, 81)), int(rng.integers(1, 13))
            n = int(rng.choice([1, 2, 7, 31, 32, 33, 63, 64, 65, 200, 4096, 20000 + int(rng.integers(0, 64))]))
            coef = rng.integers(0, 256, (rows, k), dtype=np.uint8)
            buf = rng.integers(0, 256, (k + rows) * (n + 64), dtype=np.uint8)
            offs = [i * (n + 64) + int(rng.integers(0, 64)) for i in range(k + rows)]
            src = [buf[o: o + n] for o in offs[:k]]
            dst = [buf[o: o + n] for o in offs[k:]]
            acc = bool(rng.integers(0, 2))
            before = np.stack([d.copy() for d in dst])
            ecglib.cpu_matmul(coef, src, dst, ecglib.F_ACCUMULATE if acc else 0)
            want = oracle.encode_data(coef, np.stack(src))
            if acc:
                want = want ^ before
            assert np.array_equal(np.stack(dst), want), (name, k, rows, n, acc)


@pytest.mark.parametrize("isa,want", [("scalar", 64 << 10), ("avx2", 64 << 20), ("auto", None)])
def test_default_crossover_follows_cpu_path(isa, want):
    """the drop-in's default crossover is per CPU path, measured on
    the MI355X box (daos_amd/csrc/host/ecg_dropin.c crossover_for_isa, DESIGN
    §7): GFNI never hands host cells to the GPU, the nibble-table path from
    64 MiB of len * (k + rows), the scalar path from 64 KiB.  An explicit
    crossover ($ECG_DROPIN_CROSSOVER) overrides it whatever the path."""
    code = ("from daos_amd import ecg; import sys; "
            f"assert ecg.cpu_set_isa({isa!r}) == 0 or {isa!r} != 'auto'; "
            "print(ecg.cpu_isa(), ecg.dropin_crossover())")
    for env_x, expect_set in (({}, False), ({"ECG_DROPIN_CROSSOVER": "12345"}, True)):
        r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **env_x), cwd=ROOT,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        got_isa, got = r.stdout.split()
        if expect_set:
            assert int(got) == 12345
        elif "gfni" in got_isa:
            assert int(got) == (1 << 64) - 1, (got_isa, got)
        elif want is not None and got_isa == isa:
            assert int(got) == want, (got_isa, got)
