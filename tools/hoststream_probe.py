"""Diagnostic: the configs[4] rebuild-stream rate in a fresh process, then
again after the device work the bench's headline and configs[3] leg do before
it (large allocations, launches), then after freeing them.  Bench
infrastructure; prints one JSON line per phase."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from daos_amd import ecg  # noqa: E402


def rate(ctx, label, steps=10, warm=2):
    wl = bench.HostWorkload(ctx, 8, 2, 1 << 20, 64)
    for _ in range(warm):
        wl.step()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        wl.step()
    ctx.sync()
    dt = time.perf_counter() - t0
    user = wl.user_bytes_per_step() * steps / dt / bench.GIB
    print(json.dumps({"phase": label, "GiBps": round(user, 2),
                      "h2d_GBps": round(wl.h2d_bytes_per_step() * steps / dt / 1e9, 2)}), flush=True)
    wl.free()


def main():
    ctx = ecg.Context(0)
    if "warm" in sys.argv[1:]:
        for w in (2, 4, 8, 16):
            rate(ctx, f"warm{w}_a", warm=w)
        ctx.close()
        return
    rate(ctx, "fresh")
    rate(ctx, "fresh_again")
    w = bench.Workload(ctx, 4, 2, 1 << 20, 1024)
    for _ in range(10):
        w.step()
    ctx.sync()
    rate(ctx, "with_headline_allocated")
    w.free()
    rate(ctx, "after_headline_freed")
    s = bench.Workload(ctx, 16, 2, 128 << 10, 8192, ops=("enc",), config_id=4)
    for _ in range(40):
        s.step()
    ctx.sync()
    s.free()
    rate(ctx, "after_strong_leg")
    ctx.close()


if __name__ == "__main__":
    main()
