"""Per-launch HBM traffic of a kernel from rocprofv3 --pmc CSVs.

Follows /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE come from separate --pmc passes (they do not fit one pass); both
are in KiB; on gfx950 FETCH_SIZE reports exactly half of the bytes of a wide
coalesced streaming read (16 B/lane global_load), so it is doubled.
WRITE_SIZE is exact for 16-B-per-lane streaming stores.

usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> <kernel-substring> <alg_bytes> <out.json>
"""
from __future__ import annotations

import csv
import glob
import json
import statistics
import sys


def per_launch(d: str, counter: str, needle: str) -> list[float]:
    vals = []
    for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row["Counter_Name"] == counter and needle in row["Kernel_Name"]:
                    vals.append(float(row["Counter_Value"]))
    return vals


def main() -> None:
    fetch_dir, write_dir, needle, alg, out = sys.argv[1:6]
    alg = int(alg)
    fetch = per_launch(fetch_dir, "FETCH_SIZE", needle)
    write = per_launch(write_dir, "WRITE_SIZE", needle)
    if not fetch or not write:
        raise SystemExit(f"no samples for {needle!r}: fetch={len(fetch)} write={len(write)}")
    f_kib = statistics.median(fetch)
    w_kib = statistics.median(write)
    read_bytes = 2.0 * f_kib * 1024          # gfx950 FETCH_SIZE under-count correction (x2)
    write_bytes = w_kib * 1024
    res = {
        "kernel": needle,
        "launches": {"fetch": len(fetch), "write": len(write)},
        "FETCH_SIZE_KiB_median": f_kib,
        "WRITE_SIZE_KiB_median": w_kib,
        "read_bytes_per_launch_corrected": int(read_bytes),
        "write_bytes_per_launch": int(write_bytes),
        "hbm_bytes_per_launch": int(read_bytes + write_bytes),
        "alg_bytes_per_launch": alg,
        "traffic_over_alg": round((read_bytes + write_bytes) / alg, 4),
        "correction": "FETCH_SIZE x2 (gfx950 wide-stream under-count), KiB -> bytes x1024",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
