"""Degraded-read scenarios shared by tests/test_sgl.py (CPU) and
tests/test_gpu_sgl.py (GPU): an array object of records, the iod recxs a
fetch asked for, the user's scatter-gather list, and the shadow recxs the
degraded fetch reports as to-be-recovered (ref:src/object/cli_ec.c:2313-2381,
2710-2812).  Recov recxs never span a gap between iod recxs (the reference
asserts on that, :2746)."""
from __future__ import annotations

import numpy as np

from oracle import sgl_py


def make_case(seed: int, k: int, e_len: int, iod_size: int, nstripes: int, n_iod: int, n_iov: int,
              n_recov: int, zero_iovs: int = 0, slack: int = 0):
    rng = np.random.default_rng(seed)
    srn = k * e_len
    nrec = nstripes * srn
    content = rng.integers(0, 256, nrec * iod_size, dtype=np.uint8)
    # iod recxs: sorted, disjoint; some touching (adjacent) so a recov recx may span two
    cuts = sorted(set(int(x) for x in rng.integers(1, nrec, 2 * n_iod)))
    pts = [0] + cuts + [nrec]
    iod = []
    for a, b in zip(pts[0::2], pts[1::2]):
        if b > a:
            iod.append((a, b - a))
    if len(iod) >= 2 and rng.random() < 0.7:       # make one adjacency
        a0, n0 = iod[0]
        a1, n1 = iod[1]
        iod[1] = (a0 + n0, a1 + n1 - (a0 + n0))
    total = sum(n for _, n in iod) * iod_size
    # user sgl: capacity = total (+ slack at the end), random split, some empty iovs
    cut = sorted(set(int(x) for x in rng.integers(1, max(2, total), max(0, n_iov - 1))))
    lens = np.diff([0] + cut + [total + slack]).tolist()
    for _ in range(zero_iovs):
        lens.insert(int(rng.integers(0, len(lens) + 1)), 0)
    # shadow recxs: inside one iod recx, or across two adjacent ones
    recov = []
    for _ in range(n_recov):
        j = int(rng.integers(0, len(iod)))
        a, n = iod[j]
        lo = a + int(rng.integers(0, n))
        hi_lim = a + n
        if j + 1 < len(iod) and iod[j + 1][0] == a + n and rng.random() < 0.5:
            hi_lim = iod[j + 1][0] + iod[j + 1][1]
        hi = lo + 1 + int(rng.integers(0, hi_lim - lo))
        recov.append({"idx": lo, "nr": hi - lo, "ep": int(rng.integers(1, 3)), "type": sgl_py.DRT_SHADOW})
    return dict(k=k, e_len=e_len, iod_size=iod_size, srn=srn, content=content, iod=iod, lens=lens,
                recov=recov)


def stripe_image(case, stripes, p, parity_fn=None):
    """[n][k+p][C] stripe buffer of the stripe list (stripe-list order), data
    cells from the object content; parity cells from parity_fn(data [k][C])
    or zero."""
    k, C, srn, isz = case["k"], case["e_len"] * case["iod_size"], case["srn"], case["iod_size"]
    blocks = []
    for s in stripes:
        for q in range(s["nr"] // srn):
            st = s["idx"] + q * srn
            data = case["content"][st * isz:(st + srn) * isz].reshape(k, C)
            par = parity_fn(data) if parity_fn else np.zeros((p, C), np.uint8)
            blocks.append(np.concatenate([data, par]).reshape(-1))
    return np.concatenate(blocks) if blocks else np.zeros(0, np.uint8)


def expected_user_bytes(case, fill=0xEE):
    """What the user's sgl should hold after fill-back: object bytes at the
    recovered records' iod offsets, `fill` elsewhere (as one flat array of
    iov capacities)."""
    isz = case["iod_size"]
    out = np.full(sum(case["lens"]), fill, np.uint8)
    off = 0
    for a, n in case["iod"]:
        for r in case["recov"]:
            lo, hi = max(a, r["idx"]), min(a + n, r["idx"] + r["nr"])
            if lo < hi:
                out[off + (lo - a) * isz: off + (hi - a) * isz] = case["content"][lo * isz: hi * isz]
        off += n * isz
    return out
