"""Minimal program for rocprofv3 counter passes of the standalone CRC kernels:
crc32 and crc64 over 1 GiB of device-resident 1 MiB cells in 32 KiB chunks
(the BENCH `crc*_32KiB_chunks_1GiB` rows), 5 launches each, and (with
`fused`) EC_8P2 encode with fused crc32 / crc64 checksums.  Run as
  rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE ... -- python3 tools/crc_pmc.py
Bench infrastructure (no oracle)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402
from tools.datagen import stripe_bytes  # noqa: E402


def main():
    ctx = ecg.Context(0)
    C, n = 1 << 20, 1024
    buf = ctx.alloc(C * n)
    blk = stripe_bytes(256 << 20, 9)
    for off in range(0, C * n, blk.size):
        buf.upload(blk[: min(blk.size, C * n - off)], offset=off)
    out = ctx.alloc(n * (C // 4096) * 8)
    for htype in (ecg.HASH_CRC32, ecg.HASH_CRC64):
        for _ in range(5):
            ctx.csum_extents(htype, 32768, 1, 0, C, buf.ptr, C, n, out.ptr)
        ctx.sync()
    if "fused" in sys.argv[1:]:
        k, p, S = 8, 2, 128                 # data k*S*C = 1 GiB = buf
        par = ctx.alloc(p * S * C)
        assert k * S * C <= buf.nbytes
        for _ in range(5):
            ctx.encode(k, p, C, S, buf.ptr, k * C, par.ptr, S * C, C)
        ctx.sync()
        for htype in (ecg.HASH_CRC32, ecg.HASH_CRC64):
            for _ in range(5):
                ctx.encode_csum(k, p, C, S, buf.ptr, k * C, par.ptr, S * C, C, htype, 32768, 1, out.ptr)
            ctx.sync()
        par.free()
    buf.free()
    out.free()
    ctx.close()
    print("crc_pmc done", flush=True)


if __name__ == "__main__":
    main()
