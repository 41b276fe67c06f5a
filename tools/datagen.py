"""Seeded synthetic stripe bytes (bench/test infrastructure, not product).

BASELINE.md §3: splitmix64 -> xoshiro256**, seed 0xDA05EC00 + config_id.
Vectorised over L independent lanes (lane i seeded by splitmix64 of
seed + i); word w of the output is lane w % L, step w // L.
"""
from __future__ import annotations

import numpy as np

SEED_BASE = 0xDA05EC00
M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    x = x + np.uint64(0x9E3779B97F4A7C15)
    z = x
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x, z ^ (z >> np.uint64(31))


def _rotl(x: np.ndarray, k: int) -> np.ndarray:
    return (x << np.uint64(k)) | (x >> np.uint64(64 - k))


def stripe_bytes(nbytes: int, config_id: int = 0, lanes: int = 1 << 18) -> np.ndarray:
    """nbytes of deterministic pseudo-random data (uint8)."""
    nwords = (nbytes + 7) // 8
    lanes = max(1, min(lanes, nwords))
    with np.errstate(over="ignore"):
        x = np.uint64(SEED_BASE + config_id) + np.arange(lanes, dtype=np.uint64)
        s = []
        for _ in range(4):
            x, z = _splitmix64(x)
            s.append(z)
        s0, s1, s2, s3 = s
        steps = (nwords + lanes - 1) // lanes
        out = np.empty(steps * lanes, dtype=np.uint64)
        for i in range(steps):
            out[i * lanes:(i + 1) * lanes] = _rotl(s1 * np.uint64(5), 7) * np.uint64(9)
            t = s1 << np.uint64(17)
            s2 ^= s0
            s3 ^= s1
            s1 ^= s2
            s0 ^= s3
            s2 ^= t
            s3 = _rotl(s3, 45)
    return out.view(np.uint8)[:nbytes]
