"""Diagnostic: why bench.py's configs[4] leg (47-48 GiB/s) runs below the
same host stream in a fresh process (51 GiB/s, tools/hoststream_overlap.py).
Runs the rebuild-stream leg (bench.leg_stream) in phases: fresh, after the
headline workload, after the configs[3] legs, and once more; prints one JSON
line per phase.  Bench infrastructure."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from daos_amd import ecg  # noqa: E402


def leg(args, ctx, label):
    r = bench.leg_stream(args, ctx, 1, 0, 10, None)
    row = r["ranks"][0]
    print(json.dumps({"phase": label, "GiBps": r["value_GiBps"], "h2d_GBps": row["h2d_GBps"],
                      "frac": row["frac_of_h2d"], "pinned_cpus": row.get("pinned_cpus")}), flush=True)


def main():
    args = argparse.Namespace(rehearse=False, host_chunk=0)
    if os.environ.get("LP_TORCH") == "1":       # as bench.py: torch first, its HIP runtime
        import torch

        torch.cuda.set_device(0)
        torch.cuda.synchronize()
    ctx = ecg.Context(0)
    leg(args, ctx, "fresh")
    leg(args, ctx, "fresh_again")
    w = bench.Workload(ctx, 4, 2, 1 << 20, 1024)
    for _ in range(23):
        w.step()
    ctx.sync()
    w.free()
    leg(args, ctx, "after_headline")
    bench.leg_strong(args, ctx, 1, 0, 20)
    bench.leg_strong(args, ctx, 1, 0, 20, weak=True)
    leg(args, ctx, "after_config3_legs")
    leg(args, ctx, "again")
    ctx.close()


if __name__ == "__main__":
    main()
