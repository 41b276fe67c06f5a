"""Minimal program for rocprofv3 FETCH_SIZE / WRITE_SIZE passes of one EC
product shape (the EC_8P2 decode and EC_16P2 rows), 5
launches after 2 warm-up launches, seeded random cells:
  dec_8p2     EC_8P2 1 MiB x 512, {d0,d1} regenerated in [S][k+p][C]
  enc_16p2    EC_16P2 128 KiB x 1024, data [S][k][C] -> parity [p][S][C] (padded pitch)
  dec_16p2    EC_16P2 128 KiB x 1024, {d0,d1} regenerated in [S][k+p][C]
  enc_4p2 / enc_8p2 / enc_16p2_cap2 (2 blocks per CU) / enc_16p2_x4096, and the
  streaming read / write kernels (4 GiB) as references for the memory-side counters,
  upd1_8p2    EC_8P2 1 MiB x 512, delta update of one cell per stripe (old, new
              [S][1][C], parity [p][S][C] read and written)
Run as  rocprofv3 --pmc FETCH_SIZE -- python3 tools/ec_pmc.py dec_8p2  and summarise
with tools/pmc_traffic.py (algorithmic bytes printed here) or tools/pmc_summary.py.
The launch tuner is off: every launch runs the geometry named.  Bench infrastructure."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from daos_amd import ecg  # noqa: E402
from tools.datagen import stripe_bytes  # noqa: E402

SHAPES = {"dec_8p2": (8, 2, 1 << 20, 512, "dec"), "enc_16p2": (16, 2, 128 << 10, 1024, "enc"),
          "dec_16p2": (16, 2, 128 << 10, 1024, "dec"), "enc_4p2": (4, 2, 1 << 20, 1024, "enc"),
          "enc_8p2": (8, 2, 1 << 20, 512, "enc"), "enc_16p2_cap2": (16, 2, 128 << 10, 1024, "enc"),
          "enc_16p2_x4096": (16, 2, 128 << 10, 4096, "enc"), "read": (0, 0, 0, 0, "read"),
          "write": (0, 0, 0, 0, "write"), "upd1_8p2": (8, 2, 1 << 20, 512, "upd")}


def stream(ctx, mode):
    """The box's streaming read (mode 1) / write (mode 2) kernel over 4 GiB,
    at the geometry bench.py measures its ceilings with."""
    n = 4 << 30
    a, b = ctx.alloc(n), ctx.alloc(n)
    a.fill(0x3C)
    ctx.set_launch(512 if mode == 1 else 0, 0, 0)
    for _ in range(7):
        ctx.copy_kernel(b.ptr, a.ptr, n, mode)
    ctx.sync()
    print(f"ec_pmc stream mode {mode} kernel {ecg.last_kernel()} bytes_per_launch {n}", flush=True)
    a.free()
    b.free()


def main():
    k, p, C, S, op = SHAPES[sys.argv[1]]
    ctx = ecg.Context(0)
    ctx.set_autotune(0)
    if op in ("read", "write"):
        stream(ctx, 1 if op == "read" else 2)
        ctx.close()
        return
    if sys.argv[1].endswith("_cap2"):
        ctx.set_wg_per_cu(2)
    st = (k + p) * C
    buf = ctx.alloc(S * st)
    blk = stripe_bytes(256 << 20, 5)
    for off in range(0, buf.nbytes, blk.size):
        buf.upload(blk[: min(blk.size, buf.nbytes - off)], offset=off)
    if op == "upd":
        # old / new cells in the first 2*S*C bytes of buf, parity rows after them
        pitch = S * C + 4096
        par = ctx.alloc(p * pitch)
        fn = lambda: ctx.update(k, p, C, S, [3], buf.ptr, buf.ptr + S * C, C, par.ptr, pitch, C)  # noqa: E731
        alg = (2 + 2 * p) * C * S
    elif op == "enc":
        pitch = S * C + 4096
        par = ctx.alloc(p * pitch)
        fn = lambda: ctx.encode(k, p, C, S, buf.ptr, k * C, par.ptr, pitch, C)  # noqa: E731
        alg = (k + p) * C * S
    else:
        par = None
        fn = lambda: ctx.recover(k, p, C, S, buf.ptr, st, [0, 1])  # noqa: E731
        alg = (k + 2) * C * S
    for _ in range(7):
        fn()
    ctx.sync()
    print(f"ec_pmc {sys.argv[1]} kernel {ecg.last_kernel()} alg_bytes_per_launch {alg}", flush=True)
    buf.free()
    if par is not None:
        par.free()
    ctx.close()


if __name__ == "__main__":
    main()
