"""Pure-Python restatement of the degraded-read byte movement of the DAOS EC
client: the stripe list and the fill-back into the user's sgl.

TEST INFRASTRUCTURE ONLY (tests/ may import it; the product never does).

Follows, line by line in behaviour:
  obj_ec_stripe_list_add   ref:src/object/cli_ec.c:2252-2310
  obj_ec_stripe_list_init  ref:src/object/cli_ec.c:2313-2381 (array iods)
  daos_sgl_get_bytes / daos_sgl_processor (check_buf=true)
                           ref:src/common/misc.c:313-385
  oes_copy / obj_ec_sgl_copy
                           ref:src/object/cli_ec.c:2653-2707
  obj_ec_recov_fill_back   ref:src/object/cli_ec.c:2710-2812

Data model: a recx is (idx, nr); a recx_ep is a dict {idx, nr, ep, type};
an sgl is a list of numpy uint8 arrays (the iov buffers, iov_buf_len =
len(array)) plus a list of iov_len values and sg_nr_out.  Sizes here are
small (the tests run it on a few hundred KiB), so plain loops are fine.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

DRT_SHADOW = 2


def _overlap(a_idx, a_nr, b_idx, b_nr) -> bool:
    """DAOS_RECX_PTR_OVERLAP (ref:src/include/daos/common.h:1020-1022)."""
    return a_idx < b_idx + b_nr and b_idx < a_idx + a_nr


def stripe_list_add(lst: list, sr: dict) -> None:
    for e in lst:
        if not _overlap(e["idx"], e["nr"], sr["idx"], sr["nr"]):
            if e["ep"] != sr["ep"]:
                continue
            if e["idx"] + e["nr"] == sr["idx"]:
                e["nr"] += sr["nr"]
                return
            if sr["idx"] + sr["nr"] == e["idx"]:
                e["idx"] = sr["idx"]
                e["nr"] += sr["nr"]
                return
            continue
        if e["ep"] != sr["ep"]:
            e["ep"] = max(e["ep"], sr["ep"])
        start = min(e["idx"], sr["idx"])
        e["nr"] = max(e["idx"] + e["nr"], sr["idx"] + sr["nr"]) - start
        e["idx"] = start
        return
    lst.append(dict(sr))


def stripe_list_init(stripe_rec_nr: int, recxs: list) -> list:
    out: list = []
    for r in recxs:
        if r["type"] != DRT_SHADOW:
            continue
        start = (r["idx"] // stripe_rec_nr) * stripe_rec_nr
        end = -(-(r["idx"] + r["nr"]) // stripe_rec_nr) * stripe_rec_nr
        sr = dict(r)
        sr["idx"], sr["nr"] = start, end - start
        stripe_list_add(out, sr)
    return out


@dataclass
class Sgl:
    bufs: list                      # iov buffers (numpy uint8), iov_buf_len = len
    iov_len: list = field(default_factory=list)
    nr_out: int = 0

    def __post_init__(self):
        if not self.iov_len:
            self.iov_len = [0] * len(self.bufs)


def _get_bytes(sgl: Sgl, idx: list, req: int):
    """daos_sgl_get_bytes(check_buf=true): -> (iov, off, n) or None, end.
    A zero-capacity iov is stepped over (the reference asserts on it)."""
    if idx[0] >= len(sgl.bufs):
        return None, True
    cap = len(sgl.bufs[idx[0]])
    iov, off = idx[0], idx[1]
    n = min(req, cap - off)
    idx[1] += n
    if idx[1] == cap:
        idx[0] += 1
        idx[1] = 0
    return (iov, off, n), idx[0] == len(sgl.bufs)


def sgl_copy(sgl: Sgl, off: int, src: np.ndarray) -> None:
    """obj_ec_sgl_copy: skip `off` bytes, copy src into the sgl."""
    idx = [0, 0]
    req, end = off, False
    while req > 0 and not end:
        piece, end = _get_bytes(sgl, idx, req)
        if piece:
            req -= piece[2]
    req, end, copied = len(src), False, 0
    while req > 0 and not end:
        piece, end = _get_bytes(sgl, idx, req)
        if piece is None:
            continue
        iov, o, n = piece
        req -= n
        sgl.bufs[iov][o:o + n] = src[copied:copied + n]
        copied += n
        if idx[1] == 0:
            sgl.iov_len[idx[0] - 1] = len(sgl.bufs[idx[0] - 1])
        else:
            sgl.iov_len[idx[0]] = max(sgl.iov_len[idx[0]], idx[1])
    sgl.nr_out = idx[0] if idx[1] == 0 else idx[0] + 1


def recov_fill_back(iod_size: int, iod_recxs: list, sgl: Sgl, recov: list, stripes: list,
                    stripe_buf: np.ndarray, stripe_total_sz: int, stripe_rec_nr: int,
                    singv: bool = False) -> None:
    if singv:
        sgl_copy(sgl, 0, stripe_buf[:iod_size])
        return
    for r in recov:
        rr_idx, rr_nr = r["idx"], r["nr"]
        while True:
            rec_nr, hit = 0, None
            for i_idx, i_nr in iod_recxs:
                if not _overlap(rr_idx, rr_nr, i_idx, i_nr):
                    rec_nr += i_nr
                    continue
                assert rr_idx >= i_idx
                hit = (rr_idx, min(rr_idx + rr_nr, i_idx + i_nr) - rr_idx)
                rec_nr += rr_idx - i_idx
                break
            if hit is None:
                break
            o_idx, o_nr = hit
            iod_off = rec_nr * iod_size
            n_total = 0
            done = False
            for s in stripes:
                assert s["nr"] % stripe_rec_nr == 0
                s_idx = s["idx"]
                for _ in range(s["nr"] // stripe_rec_nr):
                    base = n_total * stripe_total_sz
                    if _overlap(o_idx, o_nr, s_idx, stripe_rec_nr):
                        assert o_idx >= s_idx
                        cnt = min(o_idx + o_nr, s_idx + stripe_rec_nr) - o_idx
                        a = base + iod_size * (o_idx - s_idx)
                        sgl_copy(sgl, iod_off, stripe_buf[a:a + cnt * iod_size])
                        iod_off += cnt * iod_size
                        o_idx += cnt
                        o_nr -= cnt
                        if o_nr == 0:
                            done = True
                            break
                    s_idx += stripe_rec_nr
                    n_total += 1
                if done:
                    break
            assert o_nr == 0
            if o_idx < rr_idx + rr_nr:
                rr_nr = rr_idx + rr_nr - o_idx
                rr_idx = o_idx
                continue
            break
