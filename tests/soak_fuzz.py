"""Soak run of the seeded random-layout cases of test_gpu_fuzz.py over many
more seeds (not collected by pytest: run as  python tests/soak_fuzz.py N0 N1
on the GPU box).  Same checks: bytes vs the oracle, untouched bytes outside
the outputs, the lanes each launch ran vs the restated launch rules."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from daos_amd import ecg  # noqa: E402
from oracle import ref as oracle  # noqa: E402
import test_gpu_fuzz as fz  # noqa: E402


def main():
    n0, n1 = int(sys.argv[1]), int(sys.argv[2])
    ctx = ecg.Context(0)
    seen = {}
    for seed in range(n0, n1):
        got = fz.run_case(ctx, oracle, ecg, seed)
        seen[got] = seen.get(got, 0) + 1
        if (seed - n0) % 200 == 199:
            print(f"seeds {n0}..{seed}: {seen}", flush=True)
    print(f"soak OK: seeds {n0}..{n1 - 1}: {seen}", flush=True)


if __name__ == "__main__":
    main()
