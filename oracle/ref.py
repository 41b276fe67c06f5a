"""ctypes wrapper for the C oracle (oracle/build/libecg_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py.  The product (daos_amd/) never imports this.
See oracle/ec_ref.h for what is restated and why parity is "unpinned" by
reference fixtures.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# ECG_ORACLE_LIB: another build of the same sources (the ASan one,
# tests/test_oracle_asan.py)
LIB_PATH = os.environ.get("ECG_ORACLE_LIB") or os.path.join(_HERE, "build", "libecg_oracle.so")
_lib = None

u8p = C.POINTER(C.c_ubyte)
u32p = C.POINTER(C.c_uint32)


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.ref_gf_mul.restype = C.c_ubyte
        L.ref_gf_mul.argtypes = [C.c_ubyte, C.c_ubyte]
        L.ref_gf_inv.restype = C.c_ubyte
        L.ref_gf_inv.argtypes = [C.c_ubyte]
        L.ref_gf_gen_cauchy1_matrix.argtypes = [u8p, C.c_int, C.c_int]
        L.ref_gf_invert_matrix.argtypes = [u8p, u8p, C.c_int]
        L.ref_gf_invert_matrix.restype = C.c_int
        L.ref_ec_init_tables.argtypes = [C.c_int, C.c_int, u8p, u8p]
        L.ref_ec_encode_data.argtypes = [C.c_int, C.c_int, C.c_int, u8p, C.POINTER(u8p), C.POINTER(u8p)]
        L.ref_simd_encode_data.argtypes = L.ref_ec_encode_data.argtypes
        L.ref_ec_encode_data_update.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, u8p, u8p, C.POINTER(u8p)]
        L.ref_xor_gen.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_void_p)]
        L.ref_xor_gen.restype = C.c_int
        L.ref_obj_ec_recov_codec_init.argtypes = [C.c_int, C.c_int, u8p, u32p, C.c_int, u8p, u32p, u32p,
                                                  u8p, C.POINTER(C.c_int)]
        L.ref_obj_ec_recov_codec_init.restype = C.c_int
        L.ref_encode_batch.argtypes = [C.c_int, C.c_int, C.c_uint64, C.c_uint32, u8p, u8p, C.c_int]
        L.ref_simd_encode_batch.argtypes = L.ref_encode_batch.argtypes
        L.ref_recov_batch.argtypes = [C.c_int, C.c_int, u8p, u32p, u32p, C.c_uint64, C.c_uint64, C.c_uint32,
                                      u8p, C.c_int]
        L.ref_simd_recov_batch.argtypes = L.ref_recov_batch.argtypes
        L.ref_simd_variant.restype = C.c_int
        u64p = C.POINTER(C.c_uint64)
        L.ref_agg_diff_preprocess.argtypes = [u8p, C.c_uint64, C.c_uint64, C.c_uint, u64p, u64p, C.c_uint]
        L.ref_agg_update_parity.argtypes = [C.c_int, C.c_int, C.c_uint64, C.c_uint64, u8p, C.c_uint, u8p, u8p,
                                            u64p, u64p, C.c_uint, u8p]
        L.ref_agg_update_parity.restype = C.c_int
        L.ref_crc16_t10dif.restype = C.c_uint16
        L.ref_crc16_t10dif.argtypes = [C.c_uint16, u8p, C.c_uint64]
        L.ref_crc32_iscsi.restype = C.c_uint32
        L.ref_crc32_iscsi.argtypes = [u8p, C.c_uint64, C.c_uint32]
        L.ref_crc64_ecma_refl.restype = C.c_uint64
        L.ref_crc64_ecma_refl.argtypes = [C.c_uint64, u8p, C.c_uint64]
        L.ref_adler32.restype = C.c_uint32
        L.ref_adler32.argtypes = [C.c_uint32, u8p, C.c_uint64]
        L.ref_csum_record_chunksize.restype = C.c_uint64
        L.ref_csum_record_chunksize.argtypes = [C.c_uint64, C.c_uint64]
        L.ref_csum_chunk_count.restype = C.c_uint32
        L.ref_csum_chunk_count.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64]
        L.ref_csum_extent.restype = C.c_uint32
        L.ref_csum_extent.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, u8p, u8p]
        L.ref_csum_extents.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, u8p, C.c_int64,
                                       C.c_uint32, u8p, C.c_int]
        L.ref_singv_cell_bytes.argtypes = [C.c_uint64, C.c_int]
        L.ref_singv_cell_bytes.restype = C.c_uint64
        L.ref_singv_encode.argtypes = [C.c_int, C.c_int, C.c_uint64, u8p, C.POINTER(u8p)]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(u8p)


def _p32(a: np.ndarray):
    return a.ctypes.data_as(u32p)


def gf_mul(a: int, b: int) -> int:
    return lib().ref_gf_mul(a, b)


def gf_inv(a: int) -> int:
    return lib().ref_gf_inv(a)


def cauchy1(k: int, p: int) -> np.ndarray:
    m = np.zeros((k + p) * k, dtype=np.uint8)
    lib().ref_gf_gen_cauchy1_matrix(_p(m), k + p, k)
    return m.reshape(k + p, k)


def invert(mat: np.ndarray):
    n = mat.shape[0]
    a = np.ascontiguousarray(mat, dtype=np.uint8).copy()
    out = np.zeros((n, n), dtype=np.uint8)
    rc = lib().ref_gf_invert_matrix(_p(a), _p(out), n)
    return None if rc else out


def init_tables(coef: np.ndarray) -> np.ndarray:
    rows, k = coef.shape
    t = np.zeros(rows * k * 32, dtype=np.uint8)
    c = np.ascontiguousarray(coef, dtype=np.uint8)
    lib().ref_ec_init_tables(k, rows, _p(c), _p(t))
    return t


def _ptr_array(arrs):
    return (u8p * len(arrs))(*[_p(a) for a in arrs])


def encode_data(coef: np.ndarray, cells: np.ndarray, simd: bool = False) -> np.ndarray:
    """ec_encode_data over k cells [k, len] with coefficient matrix [rows, k]."""
    rows, k = coef.shape
    cells = np.ascontiguousarray(cells, dtype=np.uint8)
    n = cells.shape[1]
    out = np.zeros((rows, n), dtype=np.uint8)
    tb = init_tables(coef)
    f = lib().ref_simd_encode_data if simd else lib().ref_ec_encode_data
    f(n, k, rows, _p(tb), _ptr_array([cells[j] for j in range(k)]), _ptr_array([out[r] for r in range(rows)]))
    return out


def encode_data_update(coef: np.ndarray, vec_i: int, delta: np.ndarray, parity: np.ndarray) -> np.ndarray:
    rows, k = coef.shape
    par = np.ascontiguousarray(parity, dtype=np.uint8).copy()
    d = np.ascontiguousarray(delta, dtype=np.uint8)
    tb = init_tables(coef)
    lib().ref_ec_encode_data_update(d.shape[0], k, rows, vec_i, _p(tb), _p(d), _ptr_array([par[r] for r in range(rows)]))
    return par


def xor_gen(arrs) -> int:
    vp = (C.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    return lib().ref_xor_gen(len(arrs), arrs[0].shape[0], vp)


def recov_codec(k: int, p: int, err_list):
    """Returns (rc, de_matrix [nerrs,k], dec_idx [k], err_list, gftbls, reused)."""
    en = cauchy1(k, p).reshape(-1).copy()
    nerrs = len(err_list)
    el = np.array(list(err_list) + [0] * 8, dtype=np.uint32)
    de = np.zeros(max(nerrs, 1) * k, dtype=np.uint8)
    dec = np.zeros(k, dtype=np.uint32)
    oel = np.zeros(8, dtype=np.uint32)
    gt = np.zeros(k * p * 32, dtype=np.uint8)
    reused = C.c_int(0)
    rc = lib().ref_obj_ec_recov_codec_init(k, p, _p(en), _p32(el), nerrs, _p(de), _p32(dec), _p32(oel),
                                           _p(gt), C.byref(reused))
    return rc, de.reshape(-1, k)[:nerrs], dec, oel[:nerrs].copy(), gt, bool(reused.value)


def encode_batch(k: int, p: int, C_: int, S: int, data: np.ndarray, nthreads: int = 1, simd: bool = False,
                 out: np.ndarray | None = None):
    parity = np.zeros(p * S * C_, dtype=np.uint8) if out is None else out
    f = lib().ref_simd_encode_batch if simd else lib().ref_encode_batch
    f(k, p, C_, S, _p(data), _p(parity), nthreads)
    return parity


def recov_batch(k: int, nerrs: int, gftbls, dec_idx, err_list, C_: int, stride: int, S: int,
                stripes: np.ndarray, nthreads: int = 1, simd: bool = False):
    f = lib().ref_simd_recov_batch if simd else lib().ref_recov_batch
    f(k, nerrs, _p(gftbls), _p32(np.ascontiguousarray(dec_idx, dtype=np.uint32)),
      _p32(np.ascontiguousarray(err_list, dtype=np.uint32)), C_, stride, S, _p(stripes), nthreads)


def simd_variant() -> int:
    return lib().ref_simd_variant()


def _u64(seq):
    return (C.c_uint64 * max(1, len(seq)))(*seq)


def agg_diff_preprocess(diff: np.ndarray, len_: int, rsize: int, cell_idx: int, exts):
    d = np.ascontiguousarray(diff, dtype=np.uint8).copy()
    lib().ref_agg_diff_preprocess(_p(d), len_, rsize, cell_idx, _u64([e[0] for e in exts]),
                                  _u64([e[1] for e in exts]), len(exts))
    return d


def agg_update_parity(k: int, p: int, len_: int, rsize: int, bit_map: bytes, old: np.ndarray, new: np.ndarray,
                      exts, parity: np.ndarray) -> np.ndarray:
    par = np.ascontiguousarray(parity, dtype=np.uint8).copy()
    bm = np.frombuffer(bytes(bit_map), dtype=np.uint8).copy()
    o = np.ascontiguousarray(old, dtype=np.uint8)
    n = np.ascontiguousarray(new, dtype=np.uint8)
    rc = lib().ref_agg_update_parity(k, p, len_, rsize, _p(bm), o.shape[0], _p(o), _p(n),
                                     _u64([e[0] for e in exts]), _u64([e[1] for e in exts]), len(exts), _p(par))
    assert rc == 0
    return par


def singv_cell_bytes(size: int, k: int) -> int:
    return lib().ref_singv_cell_bytes(size, k)


def singv_encode(k: int, p: int, value: np.ndarray) -> np.ndarray:
    cb = singv_cell_bytes(value.size, k)
    out = np.zeros((p, cb), dtype=np.uint8)
    v = np.ascontiguousarray(value, dtype=np.uint8)
    lib().ref_singv_encode(k, p, v.size, _p(v), _ptr_array([out[r] for r in range(p)]))
    return out


# ---- chunked checksums (oracle/csum_ref.c) ----
HASH_CRC16, HASH_CRC32, HASH_CRC64, HASH_ADLER32 = 1, 2, 3, 7
CSUM_LEN = {HASH_CRC16: 2, HASH_CRC32: 4, HASH_CRC64: 8, HASH_ADLER32: 4}
_CSUM_DT = {2: np.uint16, 4: np.uint32, 8: np.uint64}


def crc16_t10dif(seed: int, data) -> int:
    b = np.frombuffer(bytes(data), dtype=np.uint8).copy()
    return lib().ref_crc16_t10dif(seed, _p(b), b.size)


def crc32_iscsi(data, seed: int) -> int:
    b = np.frombuffer(bytes(data), dtype=np.uint8).copy()
    return lib().ref_crc32_iscsi(_p(b), b.size, seed)


def crc64_ecma_refl(seed: int, data) -> int:
    b = np.frombuffer(bytes(data), dtype=np.uint8).copy()
    return lib().ref_crc64_ecma_refl(seed, _p(b), b.size)


def adler32(seed: int, data) -> int:
    b = np.frombuffer(bytes(data), dtype=np.uint8).copy()
    return lib().ref_adler32(seed, _p(b), b.size)


def csum_record_chunksize(chunksize: int, rec_size: int) -> int:
    return lib().ref_csum_record_chunksize(chunksize, rec_size)


def csum_chunk_count(chunksize: int, rec_size: int, rx_idx: int, rx_nr: int) -> int:
    return lib().ref_csum_chunk_count(csum_record_chunksize(chunksize, rec_size), rec_size, rx_idx, rx_nr)


def csum_extents(htype: int, chunksize: int, rec_size: int, rx_idx: int, rx_nr: int, buf: np.ndarray,
                 ext_stride: int = 0, n_ext: int = 1, nthreads: int = 8) -> np.ndarray:
    """Checksums [n_ext][nchunks] (uint16/32/64) of n_ext extents at buf + e*ext_stride."""
    n = csum_chunk_count(chunksize, rec_size, rx_idx, rx_nr)
    cl = CSUM_LEN[htype]
    out = np.zeros(max(1, n_ext * n * cl), dtype=np.uint8)
    b = np.ascontiguousarray(buf, dtype=np.uint8).reshape(-1)
    lib().ref_csum_extents(htype, chunksize, rec_size, rx_idx, rx_nr, _p(b), ext_stride, n_ext, _p(out),
                           nthreads)
    return out[:n_ext * n * cl].view(_CSUM_DT[cl]).reshape(n_ext, n)
