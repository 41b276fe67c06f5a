"""C-ABI checks that need no GPU: the library loads, exports exactly what
include/*.h declares, keeps the oracle out of the product, and its host-side
math (field, matrices, recovery rows) matches the oracle."""
import itertools
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
HEADERS = ["include/ecg.h", "include/ecg_isal.h", "include/ecg_daos.h", "include/ecg_csum.h", "include/ecg_multi.h"]


def declared_functions():
    names = []
    for h in HEADERS:
        txt = open(os.path.join(ROOT, h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        txt = re.sub(r"#.*", "", txt)
        txt = re.sub(r"typedef[^;]*;", "", txt)
        for m in re.finditer(r"\b([a-z_][a-z0-9_]*)\s*\(", txt):
            if m.group(1) not in ("if", "for", "while", "sizeof", "return") and m.group(1) not in names:
                names.append(m.group(1))
    return names


def exported_symbols(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], check=True, capture_output=True, text=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_exports_match_headers(ecglib):
    decl = set(declared_functions())
    exp = exported_symbols(ecglib.LIB_PATH)
    assert decl == exp, (sorted(decl - exp), sorted(exp - decl))
    assert set(ecglib.EXPORTED) == decl
    for name in decl:                      # ctypes can bind every one
        assert getattr(ecglib.lib(), name) is not None


def test_isal_and_daos_surfaces_present():
    names = set(declared_functions())
    for isal in ("gf_gen_cauchy1_matrix", "ec_init_tables", "ec_encode_data", "ec_encode_data_update",
                 "gf_invert_matrix", "gf_mul", "xor_gen"):
        assert isal in names
    for daos in ("ecg_obj_ec_codec_init", "ecg_obj_ec_codec_get", "ecg_obj_ec_encode_buf",
                 "ecg_obj_ec_recov_codec_init", "ecg_obj_ec_recov_data"):
        assert daos in names


def test_product_does_not_link_oracle(ecglib):
    """The oracle is test infrastructure: the product library neither links
    nor exports it, and no product source includes or imports it."""
    needed = subprocess.run(["readelf", "-d", ecglib.LIB_PATH], check=True, capture_output=True,
                            text=True).stdout
    assert "oracle" not in needed
    assert "libamdhip64" in needed
    assert not any(s.startswith("ref_") for s in exported_symbols(ecglib.LIB_PATH))
    undefined = subprocess.run(["nm", "-D", "--undefined-only", ecglib.LIB_PATH], check=True,
                               capture_output=True, text=True).stdout
    assert "ref_" not in undefined
    bad = re.compile(r"ec_ref\.h|^\s*(from|import)\s+oracle|oracle/", re.M)
    for dp, _, fs in os.walk(os.path.join(ROOT, "daos_amd")):
        for f in fs:
            if f.endswith((".c", ".h", ".hip", ".py", "Makefile")):
                assert not bad.search(open(os.path.join(dp, f)).read()), f


def test_gpu_kernels_built_for_gfx950(ecglib):
    blob = open(ecglib.LIB_PATH, "rb").read()
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in blob      # offload bundle target id
    sec = subprocess.run(["readelf", "-S", ecglib.LIB_PATH], check=True, capture_output=True, text=True).stdout
    assert ".hip_fatbin" in sec


def test_build_info_names_this_tree(ecglib):
    """The library carries the hash of the sources it was built from
    (ecg_build_info, Makefile HASHED); it equals this tree's, so the .so that
    travels to the GPU box is the build of the committed sources."""
    info = ecglib.build_info()
    assert info["src_sha256"] == ecglib.source_hash()
    assert info["arch"] == "gfx950" and info["hipcc"].startswith("HIP version")
    assert ecglib.code_object_targets() == ["gfx950"]


def test_no_device_fails_loudly(ecglib):
    if ecglib.device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(ecglib.EcgError) as ei:
        ecglib.Context(0)
    assert ei.value.rc == -ecglib.DER_NOSYS


def test_host_field_matches_oracle(ecglib, oracle):
    for a in range(256):
        for b in range(0, 256, 7):
            assert ecglib.gf_mul(a, b) == oracle.gf_mul(a, b)
        assert ecglib.gf_inv(a) == oracle.gf_inv(a)
    L = ecglib.lib()
    assert all(L.gf_mul(a, 0x53) == oracle.gf_mul(a, 0x53) for a in range(256))


@pytest.mark.parametrize("k,p", [(2, 1), (2, 2), (4, 2), (8, 2), (8, 3), (16, 3), (64, 8)])
def test_host_cauchy_matches_oracle(ecglib, oracle, k, p):
    assert np.array_equal(ecglib.cauchy1(k, p), oracle.cauchy1(k, p))
    m = np.zeros((k + p) * k, dtype=np.uint8)
    ecglib.lib().gf_gen_cauchy1_matrix(m.ctypes.data_as(ecglib.u8p), k + p, k)
    assert np.array_equal(m.reshape(k + p, k), oracle.cauchy1(k, p))


def test_host_tables_match_oracle(ecglib, oracle):
    coef = np.random.default_rng(0).integers(0, 256, (8, 16), dtype=np.uint8)
    assert np.array_equal(ecglib.isal_init_tables(coef), oracle.init_tables(coef))


def test_host_invert_matches_oracle(ecglib, oracle):
    rng = np.random.default_rng(4)
    for n in (1, 3, 8, 16):
        for _ in range(4):
            m = rng.integers(0, 256, (n, n), dtype=np.uint8)
            a, b = ecglib.invert(m), oracle.invert(m)
            assert (a is None) == (b is None)
            if a is not None:
                assert np.array_equal(a, b)
    z = np.zeros((2, 2), dtype=np.uint8)
    assert ecglib.lib().gf_invert_matrix(z.ctypes.data_as(ecglib.u8p),
                                         np.zeros(4, np.uint8).ctypes.data_as(ecglib.u8p), 2) == -1


@pytest.mark.parametrize("k,p", [(2, 1), (2, 2), (4, 2), (4, 3), (8, 2), (8, 3), (16, 2)])
def test_recov_rows_match_reference_logic(ecglib, oracle, k, p):
    """Decode rows equal the reference's (oracle restatement of
    ref:src/object/cli_ec.c:2152-2250) for every erasure set listed
    data-errors-first; the all-parity-lost shortcut is flagged the same."""
    for e in range(1, p + 1):
        for pat in itertools.combinations(range(k + p), e):
            rows, dec, reused = ecglib.recov_matrix(k, p, list(pat))
            rc, de, dec_r, el, gt, reused_r = oracle.recov_codec(k, p, list(pat))
            assert rc == 0 and reused == reused_r
            if reused:
                assert np.array_equal(rows, oracle.cauchy1(k, p)[k:])
            else:
                assert np.array_equal(rows, de), pat
                assert list(dec) == list(dec_r)


def test_recov_rows_data_loss(ecglib):
    with pytest.raises(ecglib.EcgError) as ei:
        ecglib.recov_matrix(4, 2, [0, 1, 2])
    assert ei.value.rc == -ecglib.DER_DATA_LOSS


def test_daos_codec_table(ecglib, oracle):
    import ctypes as C

    L = ecglib.lib()
    assert L.ecg_obj_ec_codec_init() == 0
    assert L.ecg_obj_ec_codec_init() == 0      # idempotent
    for redun, (k, p) in zip(range(32, 43), [(2, 1), (2, 2), (4, 1), (4, 2), (8, 1), (8, 2), (16, 1), (16, 2),
                                              (4, 3), (8, 3), (16, 3)]):
        for grp in (1, 2, 32, (1 << 16) - 1):
            oc = (redun << 24) | grp
            kk, pp = C.c_int(), C.c_int()
            assert L.ecg_obj_ec_class_kp(oc, C.byref(kk), C.byref(pp)) == 0
            assert (kk.value, pp.value) == (k, p)
            ptr = L.ecg_obj_ec_codec_get(oc)
            assert ptr
            en_ptr = C.cast(ptr, C.POINTER(C.c_void_p))[0]
            en = np.ctypeslib.as_array(C.cast(en_ptr, C.POINTER(C.c_ubyte)), shape=((k + p) * k,))
            assert np.array_equal(en.reshape(k + p, k), oracle.cauchy1(k, p))
    assert not L.ecg_obj_ec_codec_get((1 << 24) | 1)       # replicated class: not EC
    L.ecg_obj_ec_codec_fini()
    assert not L.ecg_obj_ec_codec_get((37 << 24) | 1)


def test_isal_rejects_foreign_table_layout(ecglib):
    """ec_encode_data reads coefficients out of ec_init_tables' 32-byte
    layout; tables in any other layout (a libisal GFNI build's, SURVEY
    App. A.4) must abort loudly before touching a device, never produce
    silently wrong parity."""
    import sys

    code = (
        "import sys, numpy as np; sys.path.insert(0, %r)\n"
        "from daos_amd import ecg\n"
        "k, p, C = 4, 2, 64\n"
        "tb = np.random.default_rng(1).integers(1, 256, k * p * 32, dtype=np.uint8)\n"
        "d = [np.zeros(C, np.uint8) for _ in range(k)]; o = [np.zeros(C, np.uint8) for _ in range(p)]\n"
        "ecg.isal_encode_data(tb, k, p, d, o)\n" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "32-byte layout" in r.stderr


def test_host_array_checks(ecglib):
    a = np.zeros(100, dtype=np.uint8)
    assert ecglib._host_array(a, 100, "x") == a.ctypes.data
    with pytest.raises(ValueError):
        ecglib._host_array(a, 101, "x")
    with pytest.raises(ValueError):
        ecglib._host_array(np.zeros(100, dtype=np.uint16), 10, "x")
    with pytest.raises(ValueError):
        ecglib._host_array(np.zeros((10, 10), dtype=np.uint8).T, 10, "x")


def test_stats_struct_matches_binding(ecglib):
    """The Python view of ecg_stats_t lists the header's fields in order."""
    import re

    src = open(os.path.join(ROOT, "include", "ecg.h")).read()
    body = re.search(r"typedef struct ecg_stats \{(.*?)\} ecg_stats_t;", src, re.S).group(1)
    fields = [f.strip() for line in body.split(";") if "uint64_t" in line
              for f in line.split("uint64_t", 1)[1].split(",")]
    assert tuple(fields) == ecglib.STATS_FIELDS
