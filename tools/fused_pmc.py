"""Minimal program for rocprofv3 counter passes of the fused product +
checksum kernels against the plain product: EC_8P2 x 512 stripes of 1 MiB
cells (the bench row), data [S][k][C] -> parity [p][S][C] at the padded row
pitch, crc32 / crc64 over 32 KiB chunks, the three launches interleaved for
`rounds` rounds (default 12; the first few are the clock transient of
profiles/r02/fused_transient/, tools/pmc_summary.py --skip drops them).  Run as
  rocprofv3 --pmc SQ_WAVES ... -- python3 tools/fused_pmc.py [rounds] [--lib=path/libecg.so]
Bench infrastructure (no oracle)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402
from tools.datagen import stripe_bytes  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--lib=")]
    for a in sys.argv[1:]:
        if a.startswith("--lib="):        # an experimental build (tools/build_exp.sh)
            ecg.LIB_PATH = a.split("=", 1)[1]
    rounds = int(args[0]) if args else 12
    ctx = ecg.Context(0)
    k, p, C, S = 8, 2, 1 << 20, 512
    data = ctx.alloc(k * S * C)
    blk = stripe_bytes(256 << 20, 8)
    for off in range(0, data.nbytes, blk.size):
        data.upload(blk[: min(blk.size, data.nbytes - off)], offset=off)
    pitch = S * C + 4096
    par = ctx.alloc(p * pitch)
    out = ctx.alloc(p * S * (C // 32768) * 8)
    for _ in range(rounds):
        ctx.encode(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C)
        for htype in (ecg.HASH_CRC32, ecg.HASH_CRC64):
            ctx.encode_csum(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C, htype, 32768, 1, out.ptr)
    ctx.sync()
    data.free()
    par.free()
    out.free()
    ctx.close()
    print("fused_pmc done", flush=True)


if __name__ == "__main__":
    main()
