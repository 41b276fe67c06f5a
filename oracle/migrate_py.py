"""Pure-Python restatement of migrate_update_parity's walk
(ref:src/object/srv_obj_migrate.c:1096-1181) -- the rebuild of one EC parity
shard from a fetched record range.

TEST INFRASTRUCTURE ONLY (tests/ may import it; the product never does).

For each piece: the recx handed to vos_obj_update, where its bytes come
from, and (with a checksum type) its chunk checksums as the csummer computes
them (daos_csummer_calc_iods, :1156, via oracle.ref.csum_extents).  Parity
cells are ISA-L ec_encode_data of the full stripe, row `shard` of the
Cauchy1 matrix (obj_ec_encode_buf, ref:src/object/cli_ec.c:548-573; only
p_bufs[shard - k] is kept, :1141).
"""
from __future__ import annotations

import numpy as np

PARITY_BIT = 1 << 63


def idx_daos2vos(idx: int, stripe_rec_nr: int, e_len: int) -> int:
    """obj_ec_idx_daos2vos (ref:src/object/obj_ec.h:342-343)."""
    return (idx // stripe_rec_nr) * e_len + idx % e_len


def walk(k: int, e_len: int, offset: int, size: int, encode: bool):
    """-> [(rx_idx, rx_nr, parity?, record offset into the fetched range)]"""
    stride_nr, cell_nr = k * e_len, e_len
    split = stride_nr if encode else cell_nr
    out, done = [], 0
    while size > 0:
        if offset % split != 0:
            write_nr = min(-(-offset // split) * split - offset, size)
        else:
            write_nr = min(split, size)
        if write_nr == stride_nr:
            assert encode
            out.append((idx_daos2vos(offset, stride_nr, cell_nr) | PARITY_BIT, cell_nr, True, done))
        else:
            out.append((offset, write_nr, False, done))
        size -= write_nr
        offset += write_nr
        done += write_nr
    return out


def update_parity(ref, k: int, p: int, e_len: int, iod_size: int, shard: int, buffer: np.ndarray, offset: int,
                  size: int, encode: bool, csum_type: int = 0, chunksize: int = 0):
    """-> list of dicts {recx, parity, bytes, csums}: what each vos_obj_update
    of the reference receives."""
    en = ref.cauchy1(k, p)
    C = e_len * iod_size
    res = []
    for rx_idx, rx_nr, parity, roff in walk(k, e_len, offset, size, encode):
        if parity:
            cells = buffer[roff * iod_size: roff * iod_size + k * C].reshape(k, C)
            data = ref.encode_data(en[shard:shard + 1], cells)[0]
        else:
            data = buffer[roff * iod_size: (roff + rx_nr) * iod_size]
        cs = None
        if csum_type:
            cs = ref.csum_extents(csum_type, chunksize, iod_size, rx_idx, rx_nr, np.ascontiguousarray(data))[0]
        res.append({"recx": (rx_idx, rx_nr), "parity": parity, "bytes": np.ascontiguousarray(data), "csums": cs})
    return res
