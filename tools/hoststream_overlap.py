"""configs[4] rebuild stream: does overlapping the step's two host batches
fill the PCIe bubbles?  One step = one EC_8P2 1 MiB encode batch + one
{d0,d1} recovery batch of 64 stripes from pinned host memory
(ecg_encode_host / ecg_recover_host: chunks through 3 staging slots, each
call synchronous, so the link idles while a call drains its last chunk).
  serial   one context: encode then recover (bench.py's leg)
  overlap  two contexts on the same device, the encode and the recovery on
           two host threads at once (a rebuild of two objects in parallel)
GiB/s of user data and H2D GB/s per mode, then the raw pinned H2D rate.
Bench infrastructure; prints one JSON line."""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from daos_amd import ecg  # noqa: E402


def main(steps=10, warm=8):
    k, p, C, S = 8, 2, 1 << 20, 64
    if os.environ.get("HS_TORCH") == "1":       # as bench.py: torch's HIP runtime initialised first
        import torch

        torch.cuda.set_device(0)
        torch.cuda.synchronize()
    a, b = ecg.Context(0), ecg.Context(0)
    wl = bench.HostWorkload(a, k, p, C, S)
    out = {}

    def enc(ctx):
        ctx.encode_host(k, p, C, S, wl.data.array, wl.parity.array, chunk=wl.chunk)

    def rec(ctx):
        ctx.recover_host(k, p, C, S, wl.stripes.array, wl.err, chunk=wl.chunk)

    def serial():
        enc(a)
        rec(a)

    def overlap():
        t = threading.Thread(target=rec, args=(b,))
        t.start()
        enc(a)
        t.join()

    for name, fn in (("serial", serial), ("overlap", overlap), ("serial_again", serial), ("overlap_again", overlap)):
        for _ in range(warm):
            fn()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        dt = time.perf_counter() - t0
        out[name] = {"GiBps": round(wl.user_bytes_per_step() * steps / dt / bench.GIB, 2),
                     "h2d_GBps": round(wl.h2d_bytes_per_step() * steps / dt / 1e9, 2),
                     "ms_per_step": round(dt / steps * 1e3, 3)}
    out["verified"] = wl.verify()
    wl.free()
    out["pinned_GBps"] = bench.pinned_copy_rates(a)
    out["torch_initialised"] = os.environ.get("HS_TORCH") == "1"
    print(json.dumps(out), flush=True)
    a.close()
    b.close()


if __name__ == "__main__":
    main()
