"""ctypes binding of libecg.so (include/ecg.h, ecg_isal.h, ecg_daos.h).

This is a thin host-side mirror used by the tests and bench.py: every call
goes through the C-ABI into the HIP kernels.  There is no Python or CPU
implementation of the codec here -- if the shared library is missing, or no
gfx950 device is present, calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libecg.so")

DER_INVAL = 1003
DER_NOMEM = 1009
DER_NOSYS = 1010
DER_IO = 2001
DER_REC2BIG = 2013
DER_DATA_LOSS = 2026
F_ACCUMULATE = 1

u8p = C.POINTER(C.c_ubyte)
u32p = C.POINTER(C.c_uint32)
i64p = C.POINTER(C.c_int64)
vp = C.c_void_p
# ecg_stats_t (include/ecg.h), in declaration order
STATS_FIELDS = ("encode_stripes", "encode_bytes", "recover_stripes", "recover_bytes", "update_cells",
                "update_bytes", "csum_chunks", "launches", "h2d_bytes", "d2h_bytes")

# (name, restype, argtypes) for every function of include/*.h
_SIGS = [
    ("ecg_device_count", C.c_int, []),
    ("ecg_ctx_create", C.c_int, [C.c_int, C.POINTER(vp)]),
    ("ecg_ctx_destroy", None, [vp]),
    ("ecg_ctx_unaligned_ok", C.c_int, [vp]),
    ("ecg_ctx_device", C.c_int, [vp]),
    ("ecg_ctx_stream", vp, [vp]),
    ("ecg_device_pci_bus_id", C.c_int, [C.c_int, C.c_char_p, C.c_int]),
    ("ecg_pci_numa_node", C.c_int, [C.c_char_p]),
    ("ecg_device_numa_node", C.c_int, [C.c_int]),
    ("ecg_strerror", C.c_char_p, []),
    ("ecg_last_kernel", C.c_char_p, []),
    ("ecg_build_info", C.c_char_p, []),
    ("ecg_gf_mul", C.c_ubyte, [C.c_ubyte, C.c_ubyte]),
    ("ecg_gf_inv", C.c_ubyte, [C.c_ubyte]),
    ("ecg_gen_cauchy1", C.c_int, [C.c_int, C.c_int, u8p]),
    ("ecg_invert_matrix", C.c_int, [u8p, u8p, C.c_int]),
    ("ecg_recov_matrix", C.c_int, [C.c_int, C.c_int, u8p, u32p, C.c_int, u8p, u32p, C.POINTER(C.c_int)]),
    ("ecg_matmul", C.c_int, [vp, C.c_int, C.c_int, u8p, C.c_uint64, C.c_uint32, vp, i64p, C.c_int64,
                             vp, i64p, C.c_int64, C.c_uint, vp]),
    ("ecg_encode", C.c_int, [vp, C.c_int, C.c_int, C.c_uint64, C.c_uint32, vp, C.c_int64, vp, C.c_int64,
                             C.c_int64, vp]),
    ("ecg_recover", C.c_int, [vp, C.c_int, C.c_int, C.c_uint64, C.c_uint32, vp, C.c_int64, u32p, C.c_int, vp]),
    ("ecg_update", C.c_int, [vp, C.c_int, C.c_int, C.c_uint64, C.c_uint32, C.c_int, u32p, vp, vp, C.c_int64,
                             vp, C.c_int64, C.c_int64, vp]),
    ("ecg_matmul_ptrs", C.c_int, [vp, C.c_int, C.c_int, u8p, C.c_uint64, C.c_uint32, C.POINTER(vp), vp]),
    ("ecg_update_ptrs", C.c_int, [vp, C.c_int, C.c_int, C.c_uint64, C.c_uint32, C.POINTER(vp), u8p, vp]),
    ("ecg_matmul_host", C.c_int, [vp, C.c_int, C.c_int, C.c_int, u8p, C.POINTER(u8p), C.POINTER(u8p), C.c_uint]),
    ("ecg_cpu_matmul", C.c_int, [C.c_int, C.c_int, C.c_int, u8p, C.POINTER(u8p), C.POINTER(u8p), C.c_uint]),
    ("ecg_cpu_isa", C.c_char_p, []),
    ("ecg_cpu_set_isa", C.c_int, [C.c_char_p]),
    ("ecg_set_dropin_crossover", C.c_int, [C.c_uint64]),
    ("ecg_dropin_crossover", C.c_uint64, []),
    ("ecg_encode_host", C.c_int, [vp, C.c_int, C.c_int, C.c_uint64, C.c_uint32, vp, vp, C.c_uint32]),
    ("ecg_recover_host", C.c_int, [vp, C.c_int, C.c_int, C.c_uint64, C.c_uint32, vp, u32p, C.c_int, C.c_uint32]),
    ("ecg_queue_create", C.c_int, [vp, vp, C.POINTER(vp)]),
    ("ecg_queue_destroy", None, [vp]),
    ("ecg_queue_encode", C.c_int, [vp, C.c_int, C.c_int, C.c_uint64, C.POINTER(u8p), C.POINTER(u8p), vp, vp]),
    ("ecg_queue_recover", C.c_int, [vp, C.c_int, C.c_int, C.c_uint64, u8p, u32p, C.c_int, vp, vp]),
    ("ecg_queue_update", C.c_int, [vp, C.c_int, C.c_int, C.c_uint64, C.c_int, u8p, u8p, C.POINTER(u8p), vp, vp]),
    ("ecg_queue_create_multi", C.c_int, [vp, vp, C.POINTER(vp)]),
    ("ecg_queue_flush", C.c_int, [vp]),
    ("ecg_queue_stats", C.c_int, [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("ecg_dev_alloc", C.c_int, [vp, C.c_size_t, C.POINTER(vp)]),
    ("ecg_dev_free", C.c_int, [vp, vp]),
    ("ecg_host_alloc", C.c_int, [vp, C.c_size_t, C.POINTER(vp)]),
    ("ecg_host_free", C.c_int, [vp, vp]),
    ("ecg_memcpy", C.c_int, [vp, vp, vp, C.c_size_t, C.c_int, vp]),
    ("ecg_memset", C.c_int, [vp, vp, C.c_int, C.c_size_t, vp]),
    ("ecg_stream_create", C.c_int, [vp, C.POINTER(vp)]),
    ("ecg_stream_destroy", C.c_int, [vp, vp]),
    ("ecg_stream_sync", C.c_int, [vp, vp]),
    ("ecg_event_create", C.c_int, [vp, C.POINTER(vp)]),
    ("ecg_event_destroy", C.c_int, [vp, vp]),
    ("ecg_event_record", C.c_int, [vp, vp, vp]),
    ("ecg_event_elapsed_ms", C.c_int, [vp, vp, vp, C.POINTER(C.c_float)]),
    ("ecg_device_sync", C.c_int, [vp]),
    ("ecg_dev_copy_kernel", C.c_int, [vp, vp, vp, C.c_size_t, C.c_int, vp]),
    ("ecg_set_launch", C.c_int, [vp, C.c_uint32, C.c_uint32, C.c_uint32]),
    ("ecg_set_launch_order", C.c_int, [vp, C.c_uint32]),
    ("ecg_set_wg_per_cu", C.c_int, [vp, C.c_uint32]),
    ("ecg_set_autotune", C.c_int, [vp, C.c_int]),
    ("ecg_tune_state", C.c_int, [vp, C.c_int, C.c_int, C.c_uint64, C.c_uint32, C.c_int64, C.c_int64, u32p,
                                 C.POINTER(C.c_float), C.POINTER(C.c_float)]),
    ("ecg_tune_counters", C.c_int, [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), u32p]),
    ("ecg_get_stats", C.c_int, [vp, vp, C.c_int]),
    # multi-device sharder (ecg_multi.h)
    ("ecg_multi_create", C.c_int, [C.POINTER(C.c_int), C.c_int, C.POINTER(vp)]),
    ("ecg_multi_destroy", None, [vp]),
    ("ecg_multi_count", C.c_int, [vp]),
    ("ecg_multi_numa_node", C.c_int, [vp, C.c_int]),
    ("ecg_multi_ctx", vp, [vp, C.c_int]),
    ("ecg_multi_range", C.c_int, [vp, C.c_uint32, C.c_int, u32p, u32p]),
    ("ecg_multi_encode", C.c_int, [vp, C.c_int, C.c_int, C.c_uint64, u32p, C.POINTER(vp), C.c_int64,
                                   C.POINTER(vp), C.c_int64, C.c_int64, C.c_uint]),
    ("ecg_multi_recover", C.c_int, [vp, C.c_int, C.c_int, C.c_uint64, u32p, C.POINTER(vp), C.c_int64, u32p,
                                    C.c_int, C.c_uint]),
    ("ecg_multi_sync", C.c_int, [vp]),
    ("ecg_multi_encode_csum", C.c_int, [vp, C.c_int, C.c_int, C.c_uint64, u32p, C.POINTER(vp), C.c_int64,
                                        C.POINTER(vp), C.c_int64, C.c_int64, C.c_int, C.c_uint64, C.c_uint64,
                                        C.POINTER(vp), C.c_uint]),
    ("ecg_multi_recover_csum", C.c_int, [vp, C.c_int, C.c_int, C.c_uint64, u32p, C.POINTER(vp), C.c_int64, u32p,
                                         C.c_int, C.c_int, C.c_uint64, C.c_uint64, C.POINTER(vp), C.c_uint]),
    ("ecg_multi_update", C.c_int, [vp, C.c_int, C.c_int, C.c_uint64, u32p, C.c_int, u32p, C.POINTER(vp),
                                   C.POINTER(vp), C.c_int64, C.POINTER(vp), C.c_int64, C.c_int64, C.c_uint]),
    ("ecg_multi_migrate_range", C.c_int, [vp, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int,
                                          C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("ecg_multi_migrate_update_parity", C.c_int, [vp, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint32,
                                                  C.POINTER(vp), C.c_uint64, C.c_uint64, C.c_int, C.c_int,
                                                  C.c_uint64, C.POINTER(vp), C.POINTER(vp), vp, C.c_uint32, u32p,
                                                  u32p, C.c_uint]),
    ("ecg_multi_encode_host", C.c_int, [vp, C.c_int, C.c_int, C.c_uint64, C.c_uint32, vp, vp, C.c_uint32]),
    ("ecg_multi_recover_host", C.c_int, [vp, C.c_int, C.c_int, C.c_uint64, C.c_uint32, vp, u32p, C.c_int,
                                         C.c_uint32]),
    # ISA-L drop-in (ecg_isal.h)
    ("ec_init_tables", None, [C.c_int, C.c_int, u8p, u8p]),
    ("ec_encode_data", None, [C.c_int, C.c_int, C.c_int, u8p, C.POINTER(u8p), C.POINTER(u8p)]),
    ("ec_encode_data_update", None, [C.c_int, C.c_int, C.c_int, C.c_int, u8p, u8p, C.POINTER(u8p)]),
    ("gf_vect_mul_init", None, [C.c_ubyte, u8p]),
    ("gf_mul", C.c_ubyte, [C.c_ubyte, C.c_ubyte]),
    ("gf_inv", C.c_ubyte, [C.c_ubyte]),
    ("gf_gen_rs_matrix", None, [u8p, C.c_int, C.c_int]),
    ("gf_gen_cauchy1_matrix", None, [u8p, C.c_int, C.c_int]),
    ("gf_invert_matrix", C.c_int, [u8p, u8p, C.c_int]),
    ("xor_gen", C.c_int, [C.c_int, C.c_int, C.POINTER(vp)]),
    # DAOS codec surface (ecg_daos.h)
    ("ecg_obj_ec_codec_init", C.c_int, []),
    ("ecg_obj_ec_codec_fini", None, []),
    ("ecg_obj_ec_codec_get", vp, [C.c_uint32]),
    ("ecg_obj_ec_class_kp", C.c_int, [C.c_uint32, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ("ecg_obj_ec_encode_buf", C.c_int, [C.c_uint32, C.c_uint64, u8p, C.POINTER(u8p)]),
    ("ecg_obj_ec_recov_codec_alloc", vp, []),
    ("ecg_obj_ec_recov_codec_free", None, [vp]),
    ("ecg_obj_ec_recov_codec_init", C.c_int, [C.c_uint32, u32p, C.c_uint32, vp]),
    ("ecg_obj_ec_recov_data", C.c_int, [vp, vp, C.c_uint64, u8p, C.c_uint32]),
    ("ecg_obj_ec_encode_stripes", C.c_int, [vp, C.c_uint32, C.c_uint64, C.c_uint32, u8p, u8p]),
    ("ecg_agg_update_parity", C.c_int, [vp, C.c_uint32, C.c_uint64, C.c_uint64, u8p, C.c_uint32, u8p, u8p,
                                        C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_uint32, u8p]),
    ("ecg_agg_recalc_parity", C.c_int, [vp, C.c_uint32, C.c_uint64, u8p, C.c_uint32, u8p, u8p, u8p]),
    ("ecg_obj_ec_singv_cell_bytes", C.c_uint64, [C.c_uint32, C.c_uint64]),
    ("ecg_obj_ec_singv_encode", C.c_int, [C.c_uint32, C.c_uint64, u8p, C.POINTER(u8p)]),
    ("ecg_obj_ec_recx_encode", C.c_int, [vp, C.c_uint32, C.c_uint64, vp, C.c_uint32, vp, C.c_uint32,
                                         C.POINTER(vp), vp]),
    ("ecg_obj_ec_stripe_list_init", C.c_int, [C.c_uint64, vp, C.c_uint32, vp, C.c_uint32, u32p]),
    ("ecg_obj_ec_recov_fill_back", C.c_int, [vp, C.c_uint64, C.c_int, vp, C.c_uint32, vp, vp, C.c_uint32, vp,
                                             C.c_uint32, vp, C.c_uint64, C.c_uint64, vp]),
    ("ecg_obj_ec_recov_data_dev", C.c_int, [vp, C.c_uint32, C.c_uint64, vp, vp, C.c_uint32, vp]),
    ("ecg_migrate_plan_size", C.c_int, [C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int,
                                        C.c_int, C.c_uint64, u32p, u32p, C.POINTER(C.c_uint64)]),
    ("ecg_migrate_update_parity", C.c_int, [vp, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint32, vp, C.c_uint64,
                                            C.c_uint64, C.c_int, C.c_int, C.c_uint64, vp, vp, vp, C.c_uint32,
                                            u32p, vp]),
    ("ecg_obj_ec_stripe_rec_nr", C.c_uint64, [C.c_uint32, C.c_uint64]),
    ("ecg_obj_ec_cell_bytes", C.c_uint64, [C.c_uint64, C.c_uint64]),
    ("ecg_obj_ec_tgt_of_recx_idx", C.c_uint32, [C.c_uint64, C.c_uint64, C.c_uint64]),
    ("ecg_obj_ec_idx_daos2vos", C.c_uint64, [C.c_uint64, C.c_uint64, C.c_uint64]),
    ("ecg_obj_ec_idx_vos2daos", C.c_uint64, [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32]),
    ("ecg_obj_ec_idx_parity2daos", C.c_uint64, [C.c_uint64, C.c_uint64, C.c_uint64]),
    ("ecg_obj_ec_shard_off_by_start", C.c_uint32, [C.c_uint32, C.c_uint32, C.c_uint32]),
    # chunked checksums (ecg_csum.h)
    ("ecg_csum_len", C.c_int, [C.c_int]),
    ("ecg_csum_record_chunksize", C.c_uint64, [C.c_uint64, C.c_uint64]),
    ("ecg_csum_chunk_count", C.c_uint32, [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64]),
    ("ecg_csum_extents", C.c_int, [vp, C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, vp, C.c_int64,
                                   C.c_uint32, vp, vp]),
    ("ecg_set_csum_launch", C.c_int, [vp, C.c_uint32]),
    ("ecg_set_fused_cols", C.c_int, [vp, C.c_uint32]),
    ("ecg_encode_csum", C.c_int, [vp, C.c_int, C.c_int, C.c_uint64, C.c_uint32, vp, C.c_int64, vp, C.c_int64,
                                  C.c_int64, C.c_int, C.c_uint64, C.c_uint64, vp, vp]),
    ("ecg_recover_csum", C.c_int, [vp, C.c_int, C.c_int, C.c_uint64, C.c_uint32, vp, C.c_int64, u32p, C.c_int,
                                   C.c_int, C.c_uint64, C.c_uint64, vp, vp]),
]

HASH_CRC16, HASH_CRC32, HASH_CRC64, HASH_ADLER32 = 1, 2, 3, 7
MULTI_ASYNC = 1

EXPORTED = [n for n, _, _ in _SIGS]


class Iov(C.Structure):
    """ecg_iov_t (d_iov_t: iov_buf, iov_buf_len, iov_len), device memory."""
    _fields_ = [("iov_buf", vp), ("iov_buf_len", C.c_uint64), ("iov_len", C.c_uint64)]


class EcRecx(C.Structure):
    """ecg_ec_recx_t (struct obj_ec_recx: oer_byte_off, oer_stripe_nr)."""
    _fields_ = [("byte_off", C.c_uint64), ("stripe_nr", C.c_uint32), ("pad", C.c_uint32)]


class Recx(C.Structure):
    """ecg_recx_t (daos_recx_t)."""
    _fields_ = [("rx_idx", C.c_uint64), ("rx_nr", C.c_uint64)]


class RecxEp(C.Structure):
    """ecg_recx_ep_t (struct daos_recx_ep)."""
    _fields_ = [("re_recx", Recx), ("re_ep", C.c_uint64), ("re_rec_size", C.c_uint32), ("re_type", C.c_uint8)]


class Sgl(C.Structure):
    """ecg_sgl_t (d_sg_list_t) over device iov buffers."""
    _fields_ = [("sg_nr", C.c_uint32), ("sg_nr_out", C.c_uint32), ("sg_iovs", C.POINTER(Iov))]


class RecovIod(C.Structure):
    """ecg_recov_iod_t: one iod of obj_ec_recov_data (device buffers)."""
    _fields_ = [("iod_size", C.c_uint64), ("singv", C.c_uint32), ("iod_nr", C.c_uint32),
                ("iod_recxs", C.POINTER(Recx)), ("sgl", C.POINTER(Sgl)), ("recov", C.POINTER(RecxEp)),
                ("recov_nr", C.c_uint32), ("stripe_nr", C.c_uint32), ("stripes", C.POINTER(RecxEp)),
                ("stripe_buf", vp)]


class MigratePiece(C.Structure):
    """ecg_migrate_piece_t: one piece of migrate_update_parity's walk."""
    _fields_ = [("recx", Recx), ("buf_off", C.c_uint64), ("buf_len", C.c_uint64), ("csum_off", C.c_uint64),
                ("nr_csums", C.c_uint32), ("parity", C.c_uint32)]


MAX_K, MAX_P = 64, 8


class RecovCodec(C.Structure):
    """struct ecg_obj_ec_recov_codec (include/ecg_daos.h), field for field."""
    _fields_ = [("er_gftbls", C.c_ubyte * (MAX_K * MAX_P * 32)), ("er_de_matrix", C.c_ubyte * (MAX_P * MAX_K)),
                ("er_dec_idx", C.c_uint32 * MAX_K), ("er_err_list", C.c_uint32 * MAX_P), ("er_nerrs", C.c_uint32),
                ("er_data_nerrs", C.c_uint32), ("k", C.c_int), ("p", C.c_int), ("reused_encode", C.c_int),
                ("er_builds", C.c_uint32)]


DRT_SHADOW = 2

_lib = None


class EcgError(RuntimeError):
    def __init__(self, rc: int, what: str):
        self.rc = rc
        super().__init__(f"{what}: rc={rc} ({lib().ecg_strerror().decode(errors='replace')})")


def lib():
    """Load libecg.so (built in-tree by __graft_entry__.build()).  Raises if absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = C.CDLL(LIB_PATH)
        for name, res, args in _SIGS:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _chk(rc: int, what: str):
    if rc != 0:
        raise EcgError(rc, what)


def _u8(a: np.ndarray):
    return a.ctypes.data_as(u8p)


def _u32(seq) -> C.Array:
    return (C.c_uint32 * max(1, len(seq)))(*seq)


def _i64(seq) -> C.Array:
    return (C.c_int64 * max(1, len(seq)))(*seq)


def device_count() -> int:
    return lib().ecg_device_count()


def last_kernel() -> str:
    return lib().ecg_last_kernel().decode()


def build_info() -> dict:
    """ecg_build_info() of the loaded library: src_sha256, hipcc, arch."""
    return dict(kv.split("=", 1) for kv in lib().ecg_build_info().decode().split(";"))


def source_hash() -> str:
    """sha256 (16 hex) over the library's sources as they are in this tree --
    the recipe of daos_amd/csrc/Makefile HASHED (paths relative to csrc,
    byte-sorted, contents concatenated).  Equal to build_info()["src_sha256"]
    iff the loaded libecg.so was built from exactly these sources."""
    import glob
    import hashlib

    csrc = os.path.join(_HERE, "csrc")
    pats = ("host/*.c", "host/*.h", "kernels/*.hip", "kernels/*.h", "*.h", "../../include/*.h")
    rel = {os.path.relpath(f, csrc) if not pat.startswith("..") else "../../include/" + os.path.basename(f)
           for pat in pats for f in glob.glob(os.path.join(csrc, pat))}
    rel |= {"Makefile", "exports.map"}
    h = hashlib.sha256()
    for r in sorted(rel, key=lambda x: x.encode()):
        with open(os.path.join(csrc, r), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def code_object_targets() -> list:
    """Offload targets of the GPU code objects bundled in the loaded
    libecg.so (from the clang offload bundle entry ids)."""
    import re

    with open(LIB_PATH, "rb") as f:
        blob = f.read()
    return sorted({m.decode() for m in re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", blob)})


def pci_bus_id(device: int) -> str:
    buf = C.create_string_buffer(64)
    _chk(lib().ecg_device_pci_bus_id(device, buf, 64), "pci_bus_id")
    return buf.value.decode()


def _host_array(a: np.ndarray, nbytes: int, what: str, write: bool = True) -> int:
    """Address of a host array the C side reads (or writes) `nbytes` of:
    uint8, C-contiguous, writeable when written, large enough -- anything
    else raises instead of letting native code run past it."""
    if not isinstance(a, np.ndarray) or a.dtype != np.uint8:
        raise ValueError(f"{what}: need a numpy uint8 array")
    if not a.flags["C_CONTIGUOUS"] or (write and not a.flags["WRITEABLE"]):
        raise ValueError(f"{what}: array must be C-contiguous" + (" and writeable" if write else ""))
    if a.nbytes < nbytes:
        raise ValueError(f"{what}: {a.nbytes} bytes < {nbytes} required")
    return a.ctypes.data


# ---------------------------------------------------------------- host math
def gf_mul(a: int, b: int) -> int:
    return lib().ecg_gf_mul(a, b)


def gf_inv(a: int) -> int:
    return lib().ecg_gf_inv(a)


def cauchy1(k: int, p: int) -> np.ndarray:
    m = np.zeros((k + p) * k, dtype=np.uint8)
    _chk(lib().ecg_gen_cauchy1(k, p, _u8(m)), "gen_cauchy1")
    return m.reshape(k + p, k)


def invert(mat: np.ndarray):
    n = mat.shape[0]
    a = np.ascontiguousarray(mat, dtype=np.uint8).copy()
    out = np.zeros((n, n), dtype=np.uint8)
    rc = lib().ecg_invert_matrix(_u8(a), _u8(out), n)
    return None if rc else out


def recov_matrix(k: int, p: int, err_list: Sequence[int]):
    """-> (rows [nerrs, k] in err_list order, dec_idx [k], reused_encode)."""
    en = cauchy1(k, p).reshape(-1).copy()
    rows = np.zeros(max(1, len(err_list)) * k, dtype=np.uint8)
    dec = (C.c_uint32 * k)()
    reused = C.c_int(0)
    _chk(lib().ecg_recov_matrix(k, p, _u8(en), _u32(err_list), len(err_list), _u8(rows), dec, C.byref(reused)),
         "recov_matrix")
    return rows.reshape(-1, k)[: len(err_list)], np.array(list(dec), dtype=np.uint32), bool(reused.value)


# ---------------------------------------------------------------- device side
class DeviceBuffer:
    def __init__(self, ctx: "Context", nbytes: int):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = vp()
        _chk(lib().ecg_dev_alloc(ctx.h, self.nbytes, C.byref(p)), "dev_alloc")
        self.ptr = p.value

    def upload(self, arr: np.ndarray, offset: int = 0, stream=None):
        a = np.ascontiguousarray(arr)
        assert offset + a.nbytes <= self.nbytes
        _chk(lib().ecg_memcpy(self.ctx.h, self.ptr + offset, a.ctypes.data, a.nbytes, 0, stream), "H2D")
        self.ctx.sync(stream)

    def download(self, nbytes: int | None = None, offset: int = 0, stream=None) -> np.ndarray:
        n = self.nbytes - offset if nbytes is None else nbytes
        out = np.empty(n, dtype=np.uint8)
        _chk(lib().ecg_memcpy(self.ctx.h, out.ctypes.data, self.ptr + offset, n, 1, stream), "D2H")
        self.ctx.sync(stream)
        return out

    def fill(self, value: int, stream=None):
        _chk(lib().ecg_memset(self.ctx.h, self.ptr, value, self.nbytes, stream), "memset")

    def free(self):
        if self.ptr:
            _chk(lib().ecg_dev_free(self.ctx.h, self.ptr), "dev_free")
            self.ptr = 0


class HostBuffer:
    """Pinned host memory exposed as a numpy uint8 array."""

    def __init__(self, ctx: "Context", nbytes: int):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = vp()
        _chk(lib().ecg_host_alloc(ctx.h, self.nbytes, C.byref(p)), "host_alloc")
        self.ptr = p.value
        self.array = np.ctypeslib.as_array((C.c_ubyte * self.nbytes).from_address(self.ptr))

    def free(self):
        if self.ptr:
            self.array = None
            _chk(lib().ecg_host_free(self.ctx.h, self.ptr), "host_free")
            self.ptr = 0


class Context:
    """One per device; mirrors ecg_ctx_t."""

    def __init__(self, device: int = 0, _handle: int | None = None):
        self.owned = _handle is None
        if _handle is None:
            h = vp()
            _chk(lib().ecg_ctx_create(device, C.byref(h)), f"ctx_create(device={device})")
            self.h = h.value
        else:
            self.h = _handle
        self.device = lib().ecg_ctx_device(self.h)

    def close(self):
        if self.h and self.owned:
            lib().ecg_ctx_destroy(self.h)
        self.h = None

    # plumbing
    def alloc(self, nbytes: int) -> DeviceBuffer:
        return DeviceBuffer(self, nbytes)

    def host_alloc(self, nbytes: int) -> HostBuffer:
        return HostBuffer(self, nbytes)

    def to_device(self, arr: np.ndarray) -> DeviceBuffer:
        a = np.ascontiguousarray(arr, dtype=np.uint8)
        b = DeviceBuffer(self, max(1, a.nbytes))
        b.upload(a)
        return b

    def sync(self, stream=None):
        _chk(lib().ecg_stream_sync(self.h, stream), "stream_sync")

    def stream(self):
        s = vp()
        _chk(lib().ecg_stream_create(self.h, C.byref(s)), "stream_create")
        return s.value

    def destroy_stream(self, s):
        _chk(lib().ecg_stream_destroy(self.h, s), "stream_destroy")

    def event(self):
        e = vp()
        _chk(lib().ecg_event_create(self.h, C.byref(e)), "event_create")
        return e.value

    def record(self, ev, stream=None):
        _chk(lib().ecg_event_record(self.h, ev, stream), "event_record")

    def elapsed_ms(self, a, b) -> float:
        ms = C.c_float()
        _chk(lib().ecg_event_elapsed_ms(self.h, a, b, C.byref(ms)), "event_elapsed")
        return ms.value

    def destroy_event(self, e):
        _chk(lib().ecg_event_destroy(self.h, e), "event_destroy")

    def set_launch(self, grid_x: int = 0, grid_y: int = 0, variant: int = 0):
        _chk(lib().ecg_set_launch(self.h, grid_x, grid_y, variant), "set_launch")

    def set_order(self, order: int = 0):
        _chk(lib().ecg_set_launch_order(self.h, order), "set_launch_order")

    def stats(self, reset: bool = False) -> dict:
        """Telemetry counters (include/ecg.h ecg_stats_t) as a dict."""
        buf = (C.c_uint64 * len(STATS_FIELDS))()
        _chk(lib().ecg_get_stats(self.h, C.cast(buf, vp), 1 if reset else 0), "get_stats")
        return dict(zip(STATS_FIELDS, buf))

    def set_wg_per_cu(self, wg_per_cu: int = 0):
        """Product-kernel blocks per CU: 0 per-shape default, 1..16 cap, 255 none."""
        _chk(lib().ecg_set_wg_per_cu(self.h, wg_per_cu), "set_wg_per_cu")

    def unaligned_ok(self) -> bool:
        """include/ecg.h ecg_ctx_unaligned_ok: misaligned dword accesses served."""
        r = lib().ecg_ctx_unaligned_ok(self.h)
        _chk(min(r, 0), "ctx_unaligned_ok")
        return r == 1

    def set_autotune(self, on: int = 1):
        """Launch tuner (include/ecg.h ecg_set_autotune): 0 off, 1 on, 2 on and forget decisions."""
        _chk(lib().ecg_set_autotune(self.h, on), "set_autotune")

    def tune_counters(self):
        """(probe cycles started, launches run inside a probe, shapes held) -- ecg_tune_counters."""
        cyc, lau, shp = C.c_uint64(), C.c_uint64(), C.c_uint32()
        _chk(lib().ecg_tune_counters(self.h, C.byref(cyc), C.byref(lau), C.byref(shp)), "tune_counters")
        return cyc.value, lau.value, shp.value

    def tune_state(self, k: int, rows: int, cell_bytes: int, nstripes: int, src_stride: int, dst_stride: int):
        """None while the shape is probing or unseen, else (cap, ms_uncapped, ms_capped);
        cap 255 = the tuner kept no cap.  Strides: encode k*C and the parity stripe
        stride; in-place recovery (k+p)*C for both."""
        cap, a, b = C.c_uint32(0), C.c_float(0), C.c_float(0)
        rc = lib().ecg_tune_state(self.h, k, rows, cell_bytes, nstripes, src_stride, dst_stride, C.byref(cap),
                                  C.byref(a), C.byref(b))
        if rc < 0:
            _chk(rc, "tune_state")
        return (cap.value, a.value, b.value) if rc == 1 else None

    def copy_kernel(self, dst: int, src: int, nbytes: int, mode: int = 0, stream=None):
        """mode 0 copy, 1 read-only, 2 write-only (HBM rate probes)."""
        _chk(lib().ecg_dev_copy_kernel(self.h, dst, src, nbytes, mode, stream), "copy_kernel")

    # codec
    def matmul(self, coef: np.ndarray, cell_bytes: int, nstripes: int, src: int, src_off, src_stride: int,
               dst: int, dst_off, dst_stride: int, flags: int = 0, stream=None):
        coef = np.ascontiguousarray(coef, dtype=np.uint8)
        rows, k = coef.shape
        _chk(lib().ecg_matmul(self.h, k, rows, _u8(coef), cell_bytes, nstripes, src, _i64(src_off), src_stride,
                              dst, _i64(dst_off), dst_stride, flags, stream), "matmul")

    def encode(self, k: int, p: int, cell_bytes: int, nstripes: int, data: int, data_stripe_stride: int,
               parity: int, parity_cell_stride: int, parity_stripe_stride: int, stream=None):
        _chk(lib().ecg_encode(self.h, k, p, cell_bytes, nstripes, data, data_stripe_stride, parity,
                              parity_cell_stride, parity_stripe_stride, stream), "encode")

    def recover(self, k: int, p: int, cell_bytes: int, nstripes: int, stripes: int, stripe_stride: int,
                err_list: Sequence[int], stream=None):
        _chk(lib().ecg_recover(self.h, k, p, cell_bytes, nstripes, stripes, stripe_stride, _u32(err_list),
                               len(err_list), stream), "recover")

    def update(self, k: int, p: int, cell_bytes: int, nstripes: int, cell_idx: Sequence[int], old: int, new: int,
               upd_stripe_stride: int, parity: int, parity_cell_stride: int, parity_stripe_stride: int,
               stream=None):
        _chk(lib().ecg_update(self.h, k, p, cell_bytes, nstripes, len(cell_idx), _u32(cell_idx), old, new,
                              upd_stripe_stride, parity, parity_cell_stride, parity_stripe_stride, stream),
             "update")

    def csum_extents(self, htype: int, chunksize: int, rec_size: int, rx_idx: int, rx_nr: int, buf: int,
                     ext_stride: int, n_ext: int, csums: int, stream=None):
        """Device checksums of n_ext extents (include/ecg_csum.h): csums[n_ext][nchunks]."""
        _chk(lib().ecg_csum_extents(self.h, htype, chunksize, rec_size, rx_idx, rx_nr, buf, ext_stride, n_ext,
                                    csums, stream), "csum_extents")

    def encode_csum(self, k: int, p: int, cell_bytes: int, nstripes: int, data: int, data_stripe_stride: int,
                    parity: int, parity_cell_stride: int, parity_stripe_stride: int, htype: int, chunksize: int,
                    rec_size: int, csums: int, stream=None):
        _chk(lib().ecg_encode_csum(self.h, k, p, cell_bytes, nstripes, data, data_stripe_stride, parity,
                                   parity_cell_stride, parity_stripe_stride, htype, chunksize, rec_size, csums,
                                   stream), "encode_csum")

    def recover_csum(self, k: int, p: int, cell_bytes: int, nstripes: int, stripes: int, stripe_stride: int,
                     err_list: Sequence[int], htype: int, chunksize: int, rec_size: int, csums: int, stream=None):
        _chk(lib().ecg_recover_csum(self.h, k, p, cell_bytes, nstripes, stripes, stripe_stride, _u32(err_list),
                                    len(err_list), htype, chunksize, rec_size, csums, stream), "recover_csum")

    def matmul_ptrs(self, k: int, rows: int, coef: np.ndarray, cell_bytes: int, nstripes: int,
                    cells: Sequence[int], stream=None):
        """cells[s*(k+rows)+j]: device addresses (inputs then outputs) per stripe."""
        co = np.ascontiguousarray(coef, dtype=np.uint8).reshape(-1)
        arr = (vp * len(cells))(*cells)
        _chk(lib().ecg_matmul_ptrs(self.h, k, rows, _u8(co), cell_bytes, nstripes, arr, stream), "matmul_ptrs")

    def update_ptrs(self, k: int, p: int, cell_bytes: int, reqs: Sequence, stream=None):
        """ecg_update_ptrs: reqs = [(vec_i, old_addr, new_addr, [parity_addr] * p)], device addresses;
        parity ^= coef[r][vec_i] * (old ^ new) for every request."""
        n = len(reqs)
        cells = (vp * max(1, n * (2 + p)))()
        vec = np.zeros(max(1, n), dtype=np.uint8)
        for i, (v, o, nw, par) in enumerate(reqs):
            vec[i] = v
            cells[i * (2 + p)] = o
            cells[i * (2 + p) + 1] = nw
            for r in range(p):
                cells[i * (2 + p) + 2 + r] = par[r]
        _chk(lib().ecg_update_ptrs(self.h, k, p, cell_bytes, n, cells, _u8(vec), stream), "update_ptrs")

    def encode_host(self, k: int, p: int, cell_bytes: int, nstripes: int, data: np.ndarray, parity: np.ndarray,
                    chunk: int = 0):
        dp = _host_array(data, nstripes * k * cell_bytes, "encode_host data", write=False)
        pp = _host_array(parity, nstripes * p * cell_bytes, "encode_host parity")
        _chk(lib().ecg_encode_host(self.h, k, p, cell_bytes, nstripes, dp, pp, chunk), "encode_host")

    def recover_host(self, k: int, p: int, cell_bytes: int, nstripes: int, stripes: np.ndarray,
                     err_list: Sequence[int], chunk: int = 0):
        sp = _host_array(stripes, nstripes * (k + p) * cell_bytes, "recover_host stripes")
        _chk(lib().ecg_recover_host(self.h, k, p, cell_bytes, nstripes, sp, _u32(err_list), len(err_list), chunk),
             "recover_host")

    def matmul_host(self, coef: np.ndarray, src: Sequence[np.ndarray], dst: Sequence[np.ndarray], flags: int = 0):
        coef = np.ascontiguousarray(coef, dtype=np.uint8)
        rows, k = coef.shape
        n = src[0].shape[0]
        sp = (u8p * k)(*[_u8(s) for s in src])
        dp = (u8p * rows)(*[_u8(d) for d in dst])
        _chk(lib().ecg_matmul_host(self.h, n, k, rows, _u8(coef), sp, dp, flags), "matmul_host")


class Multi:
    """ecg_multi_t: stripe ranges sharded over devices in one process, one
    host thread + context per shard (include/ecg_multi.h).  devices may
    repeat a device; None = $ECG_DEVICES or every device."""

    def __init__(self, devices: Sequence[int] | None = None):
        h = vp()
        arr = (C.c_int * len(devices))(*devices) if devices else None
        _chk(lib().ecg_multi_create(arr, len(devices) if devices else 0, C.byref(h)), "multi_create")
        self.h = h.value
        self.n = lib().ecg_multi_count(self.h)
        self.ctxs = [Context(_handle=lib().ecg_multi_ctx(self.h, i)) for i in range(self.n)]

    def numa_node(self, i: int) -> int:
        """NUMA node shard i's worker runs on (-1: not pinned)."""
        return lib().ecg_multi_numa_node(self.h, i)

    def range(self, nstripes: int, i: int):
        f, c = C.c_uint32(), C.c_uint32()
        _chk(lib().ecg_multi_range(self.h, nstripes, i, C.byref(f), C.byref(c)), "multi_range")
        return f.value, c.value

    def _shards(self, **seqs):
        """Every per-shard sequence must have one entry per shard: the C side
        reads n entries of each (a short nstripes would be read past its end,
        a short pointer list would hand a shard NULL)."""
        for name, v in seqs.items():
            if v is None or len(v) != self.n:
                raise ValueError(f"Multi: {name} has {0 if v is None else len(v)} entries, expected {self.n}")

    def encode(self, k: int, p: int, cell_bytes: int, nstripes: Sequence[int], data: Sequence[int],
               data_stripe_stride: int, parity: Sequence[int], parity_cell_stride: int, parity_stripe_stride: int,
               flags: int = 0):
        n = self.n
        self._shards(nstripes=nstripes, data=data, parity=parity)
        _chk(lib().ecg_multi_encode(self.h, k, p, cell_bytes, _u32(nstripes), (vp * n)(*data), data_stripe_stride,
                                    (vp * n)(*parity), parity_cell_stride, parity_stripe_stride, flags),
             "multi_encode")

    def recover(self, k: int, p: int, cell_bytes: int, nstripes: Sequence[int], stripes: Sequence[int],
                stripe_stride: int, err_list: Sequence[int], flags: int = 0):
        n = self.n
        self._shards(nstripes=nstripes, stripes=stripes)
        _chk(lib().ecg_multi_recover(self.h, k, p, cell_bytes, _u32(nstripes), (vp * n)(*stripes), stripe_stride,
                                     _u32(err_list), len(err_list), flags), "multi_recover")

    def sync(self):
        _chk(lib().ecg_multi_sync(self.h), "multi_sync")

    def encode_csum(self, k: int, p: int, cell_bytes: int, nstripes: Sequence[int], data: Sequence[int],
                    data_stripe_stride: int, parity: Sequence[int], parity_cell_stride: int,
                    parity_stripe_stride: int, htype: int, chunksize: int, rec_size: int, csums: Sequence[int],
                    flags: int = 0):
        n = self.n
        self._shards(nstripes=nstripes, data=data, parity=parity, csums=csums)
        _chk(lib().ecg_multi_encode_csum(self.h, k, p, cell_bytes, _u32(nstripes), (vp * n)(*data),
                                         data_stripe_stride, (vp * n)(*parity), parity_cell_stride,
                                         parity_stripe_stride, htype, chunksize, rec_size, (vp * n)(*csums), flags),
             "multi_encode_csum")

    def recover_csum(self, k: int, p: int, cell_bytes: int, nstripes: Sequence[int], stripes: Sequence[int],
                     stripe_stride: int, err_list: Sequence[int], htype: int, chunksize: int, rec_size: int,
                     csums: Sequence[int], flags: int = 0):
        n = self.n
        self._shards(nstripes=nstripes, stripes=stripes, csums=csums)
        _chk(lib().ecg_multi_recover_csum(self.h, k, p, cell_bytes, _u32(nstripes), (vp * n)(*stripes),
                                          stripe_stride, _u32(err_list), len(err_list), htype, chunksize, rec_size,
                                          (vp * n)(*csums), flags), "multi_recover_csum")

    def update(self, k: int, p: int, cell_bytes: int, nstripes: Sequence[int], cell_idx: Sequence[int],
               old: Sequence[int], new: Sequence[int], upd_stripe_stride: int, parity: Sequence[int],
               parity_cell_stride: int, parity_stripe_stride: int, flags: int = 0):
        n = self.n
        self._shards(nstripes=nstripes, old=old, new=new, parity=parity)
        _chk(lib().ecg_multi_update(self.h, k, p, cell_bytes, _u32(nstripes), len(cell_idx), _u32(cell_idx),
                                    (vp * n)(*old), (vp * n)(*new), upd_stripe_stride, (vp * n)(*parity),
                                    parity_cell_stride, parity_stripe_stride, flags), "multi_update")

    def migrate_range(self, oc_id: int, e_len: int, iod_size: int, offset: int, size: int, encode: bool, i: int):
        off, sz = C.c_uint64(), C.c_uint64()
        _chk(lib().ecg_multi_migrate_range(self.h, oc_id, e_len, iod_size, offset, size, int(encode), i,
                                           C.byref(off), C.byref(sz)), "multi_migrate_range")
        return off.value, sz.value

    def migrate_update_parity(self, oc_id: int, e_len: int, iod_size: int, shard: int, buffers: Sequence[int],
                              offset: int, size: int, encode: bool, csum_type: int, chunksize: int,
                              parity_out: Sequence[int], csums_out: Sequence[int], pieces_cap: int,
                              flags: int = 0):
        """Returns (pieces, shard_first): every piece in range order, shard i's
        at [shard_first[i], shard_first[i+1]) relative to its own buffers."""
        n = self.n
        self._shards(buffers=buffers, parity_out=parity_out, csums_out=csums_out)
        pieces = (MigratePiece * max(1, pieces_cap))()
        npc = C.c_uint32()
        first = (C.c_uint32 * (n + 1))()
        _chk(lib().ecg_multi_migrate_update_parity(self.h, oc_id, e_len, iod_size, shard, (vp * n)(*buffers), offset,
                                                   size, int(encode), csum_type, chunksize, (vp * n)(*parity_out),
                                                   (vp * n)(*csums_out), pieces, pieces_cap, C.byref(npc), first,
                                                   flags), "multi_migrate_update_parity")
        return list(pieces[:npc.value]), list(first)

    def encode_host(self, k: int, p: int, cell_bytes: int, nstripes: int, data: np.ndarray, parity: np.ndarray,
                    chunk: int = 0):
        dp = _host_array(data, nstripes * k * cell_bytes, "multi_encode_host data", write=False)
        pp = _host_array(parity, nstripes * p * cell_bytes, "multi_encode_host parity")
        _chk(lib().ecg_multi_encode_host(self.h, k, p, cell_bytes, nstripes, dp, pp, chunk), "multi_encode_host")

    def recover_host(self, k: int, p: int, cell_bytes: int, nstripes: int, stripes: np.ndarray,
                     err_list: Sequence[int], chunk: int = 0):
        sp = _host_array(stripes, nstripes * (k + p) * cell_bytes, "multi_recover_host stripes")
        _chk(lib().ecg_multi_recover_host(self.h, k, p, cell_bytes, nstripes, sp, _u32(err_list), len(err_list),
                                          chunk), "multi_recover_host")

    def close(self):
        if self.h:
            for c in self.ctxs:
                c.close()
            lib().ecg_multi_destroy(self.h)
            self.h = None


class QueueAttr(C.Structure):
    _fields_ = [("max_batch", C.c_uint32), ("max_wait_us", C.c_uint32), ("max_cell_bytes", C.c_uint64)]


DONE_CB = C.CFUNCTYPE(None, C.c_void_p, C.c_int)


class Queue:
    """ecg_queue_t: one-stripe requests from many threads -> batched launches.
    Completion is reported through a C callback; this wrapper records rc per
    request id (callbacks run on the queue's completion threads)."""

    def __init__(self, ctx, max_batch: int = 0, max_wait_us: int = 0, max_cell_bytes: int = 0):
        """ctx: a Context, a Multi (slots spread over its devices), or None
        (the CPU executor: host cells, no device)."""
        self.ctx = ctx
        h = vp()
        attr = QueueAttr(max_batch, max_wait_us, max_cell_bytes)
        if ctx is None:
            _chk(lib().ecg_queue_create(None, C.byref(attr), C.byref(h)), "queue_create(NULL)")
        elif isinstance(ctx, Multi):
            _chk(lib().ecg_queue_create_multi(ctx.h, C.byref(attr), C.byref(h)), "queue_create_multi")
        else:
            _chk(lib().ecg_queue_create(ctx.h, C.byref(attr), C.byref(h)), "queue_create")
        self.h = h.value
        self.done = {}
        self._keep = {}

        def _cb(arg, rc):          # arg = request id + 1 (a NULL void* would arrive as None)
            self.done[arg - 1] = rc

        self._cb = DONE_CB(_cb)

    def encode(self, rid: int, k: int, p: int, data, parity):
        C_ = data[0].shape[0]
        sp = (u8p * k)(*[_u8(d) for d in data])
        dp = (u8p * p)(*[_u8(d) for d in parity])
        self._keep[rid] = (data, parity)
        _chk(lib().ecg_queue_encode(self.h, k, p, C_, sp, dp, self._cb, rid + 1), "queue_encode")

    def encode_ptrs(self, rid: int, k: int, p: int, cell_bytes: int, data_ptrs, parity_ptrs):
        """ecg_queue_encode on cells given by address (device cells: batched
        into pointer-table launches in place)."""
        sp = (u8p * k)(*[C.cast(C.c_void_p(a), u8p) for a in data_ptrs])
        dp = (u8p * p)(*[C.cast(C.c_void_p(a), u8p) for a in parity_ptrs])
        _chk(lib().ecg_queue_encode(self.h, k, p, cell_bytes, sp, dp, self._cb, rid + 1), "queue_encode")

    def recover_ptr(self, rid: int, k: int, p: int, cell_bytes: int, stripe_ptr: int, err_list):
        """ecg_queue_recover on a [k+p][cell] stripe given by address."""
        _chk(lib().ecg_queue_recover(self.h, k, p, cell_bytes, C.cast(C.c_void_p(stripe_ptr), u8p),
                                     _u32(err_list), len(err_list), self._cb, rid + 1), "queue_recover")

    def recover(self, rid: int, k: int, p: int, stripe: np.ndarray, err_list):
        C_ = stripe.shape[-1]
        self._keep[rid] = stripe
        _chk(lib().ecg_queue_recover(self.h, k, p, C_, _u8(stripe), _u32(err_list), len(err_list), self._cb,
                                     rid + 1),
             "queue_recover")

    def update(self, rid: int, k: int, p: int, vec_i: int, old: np.ndarray, new: np.ndarray, parity):
        """parity[r] ^= coef[r][vec_i] * (old ^ new), in place at completion."""
        C_ = old.shape[0]
        dp = (u8p * p)(*[_u8(d) for d in parity])
        self._keep[rid] = (old, new, parity)
        _chk(lib().ecg_queue_update(self.h, k, p, C_, vec_i, _u8(old), _u8(new), dp, self._cb, rid + 1),
             "queue_update")

    def update_ptrs(self, rid: int, k: int, p: int, cell_bytes: int, vec_i: int, old: int, new: int, parity):
        """ecg_queue_update on cells given by address (device cells: batched
        into ecg_update_ptrs launches in place)."""
        dp = (u8p * p)(*[C.cast(C.c_void_p(a), u8p) for a in parity])
        _chk(lib().ecg_queue_update(self.h, k, p, cell_bytes, vec_i, C.cast(C.c_void_p(old), u8p),
                                    C.cast(C.c_void_p(new), u8p), dp, self._cb, rid + 1), "queue_update")

    def flush(self):
        _chk(lib().ecg_queue_flush(self.h), "queue_flush")
        self._keep.clear()

    def stats(self):
        r, b = C.c_uint64(), C.c_uint64()
        _chk(lib().ecg_queue_stats(self.h, C.byref(r), C.byref(b)), "queue_stats")
        return r.value, b.value

    def close(self):
        if self.h:
            lib().ecg_queue_destroy(self.h)
            self.h = None


# ---------------------------------------------------------------- ISA-L drop-in
def cpu_matmul(coef: np.ndarray, src: Sequence[np.ndarray], dst: Sequence[np.ndarray], flags: int = 0):
    """The product's CPU path (ecg_cpu_matmul) on host arrays."""
    coef = np.ascontiguousarray(coef, dtype=np.uint8)
    rows, k = coef.shape
    sp = (u8p * k)(*[_u8(a) for a in src])
    dp = (u8p * rows)(*[_u8(a) for a in dst])
    _chk(lib().ecg_cpu_matmul(src[0].shape[0], k, rows, _u8(coef), sp, dp, flags), "cpu_matmul")


def cpu_isa() -> str:
    return lib().ecg_cpu_isa().decode()


def cpu_set_isa(isa: str) -> int:
    return lib().ecg_cpu_set_isa(isa.encode())


def set_dropin_crossover(nbytes: int) -> None:
    lib().ecg_set_dropin_crossover(nbytes)


def dropin_crossover() -> int:
    return lib().ecg_dropin_crossover()


def isal_init_tables(coef: np.ndarray) -> np.ndarray:
    rows, k = coef.shape
    t = np.zeros(rows * k * 32, dtype=np.uint8)
    c = np.ascontiguousarray(coef, dtype=np.uint8)
    lib().ec_init_tables(k, rows, _u8(c), _u8(t))
    return t


def isal_encode_data(gftbls: np.ndarray, k: int, rows: int, data: Sequence[np.ndarray],
                     coding: Sequence[np.ndarray]):
    n = data[0].shape[0]
    sp = (u8p * k)(*[_u8(d) for d in data])
    dp = (u8p * rows)(*[_u8(c) for c in coding])
    lib().ec_encode_data(n, k, rows, _u8(gftbls), sp, dp)


def isal_encode_data_update(gftbls: np.ndarray, k: int, rows: int, vec_i: int, delta: np.ndarray,
                            coding: Sequence[np.ndarray]):
    dp = (u8p * rows)(*[_u8(c) for c in coding])
    lib().ec_encode_data_update(delta.shape[0], k, rows, vec_i, _u8(gftbls), _u8(delta), dp)


def isal_xor_gen(arrs: Sequence[np.ndarray]) -> int:
    v = (vp * len(arrs))(*[a.ctypes.data for a in arrs])
    return lib().xor_gen(len(arrs), arrs[0].shape[0], v)
