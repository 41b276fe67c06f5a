"""The batching queue's CPU executor (ecg_queue_create(NULL, ...)): the same
slots, lock-free reservations and completion threads as the device queue,
with the batches computed by ecg_cpu_matmul -- so a GPU-less process can use
the facade, and the CPU suite (and the C driver under ThreadSanitizer,
tests/c/test_ecg_c.c queue_cpu_stress) exercises its state machine.

Reference pattern replaced: one aggregation / rebuild ULT per stripe on the
offload xstream, completion through an ABT_eventual
(ref:src/object/srv_ec_aggregate.c:701-734, ref:src/engine/ult.c:394-470).
Checked byte for byte against the oracle."""
import threading

import numpy as np
import pytest


def rand(shape, seed):
    return np.random.default_rng(seed).integers(0, 256, shape, dtype=np.uint8)


@pytest.fixture
def cpuq(ecglib):
    q = ecglib.Queue(None, max_batch=16, max_wait_us=100, max_cell_bytes=65536)
    yield q
    q.close()


@pytest.mark.parametrize("k,p,C_", [(2, 1, 4096), (4, 2, 4096 + 13), (8, 2, 65536), (16, 3, 8192)])
def test_cpu_queue_encode(cpuq, oracle, k, p, C_):
    S = 40
    data = rand((S, k, C_), k * 100 + p)
    par = [[np.zeros(C_, dtype=np.uint8) for _ in range(p)] for _ in range(S)]
    for s in range(S):
        cpuq.encode(s, k, p, list(data[s]), par[s])
    cpuq.flush()
    assert len(cpuq.done) == S and all(rc == 0 for rc in cpuq.done.values())
    en = oracle.cauchy1(k, p)
    for s in range(S):
        assert np.array_equal(np.stack(par[s]), oracle.encode_data(en[k:], data[s])), s


@pytest.mark.parametrize("k,p,err", [(4, 2, [1, 4]), (8, 2, [9, 0]), (8, 3, [2, 5, 7]), (2, 1, [0])])
def test_cpu_queue_recover(cpuq, oracle, k, p, err):
    S, C_ = 24, 8192 + 5
    data = rand((S, k, C_), 31 + k)
    en = oracle.cauchy1(k, p)
    full = np.stack([np.concatenate([data[s], oracle.encode_data(en[k:], data[s])]) for s in range(S)])
    work = full.copy()
    work[:, err] = 0
    for s in range(S):
        cpuq.recover(s, k, p, work[s], err)
    cpuq.flush()
    assert all(rc == 0 for rc in cpuq.done.values()) and len(cpuq.done) == S
    assert np.array_equal(work, full)


def test_cpu_queue_updates_many_threads(cpuq, oracle):
    """8 threads post per-cell updates of overlapping stripes (host cells):
    each stripe's final parity equals the oracle's agg_update_parity."""
    k, p, C_, S, T = 8, 2, 16384, 24, 8
    rng = np.random.default_rng(606)
    par0 = rand((S, p, C_), 41)
    upd = [(s, int(c)) for s in range(S) for c in rng.choice(k, int(rng.integers(1, 5)), replace=False)]
    rng.shuffle(upd)
    olds = rand((len(upd), C_), 42)
    news = rand((len(upd), C_), 43)
    par = par0.copy()

    def worker(t):
        for i in range(t, len(upd), T):
            s, c = upd[i]
            cpuq.update(i, k, p, c, olds[i], news[i], [par[s, r] for r in range(p)])

    th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    cpuq.flush()
    assert len(cpuq.done) == len(upd) and all(rc == 0 for rc in cpuq.done.values())
    for s in range(S):
        mine = sorted((c, i) for i, (ss, c) in enumerate(upd) if ss == s)
        bm = bytearray(2)
        for c, _ in mine:
            bm[c // 8] |= 1 << (c % 8)
        want = oracle.agg_update_parity(k, p, C_, 1, bytes(bm), np.stack([olds[i] for _, i in mine]),
                                        np.stack([news[i] for _, i in mine]), [(0, k * C_)], par0[s])
        assert np.array_equal(par[s], want), s


def test_cpu_queue_cells_in_place_large(cpuq, oracle):
    """Nothing is staged: cells bigger than the queue's max_cell_bytes (64 KiB
    here) and than one 256 KiB product chunk, ragged tails, k > 16 -- encode,
    recovery and updates straight from the callers' cells."""
    k, p, C_ = 20, 3, (256 << 10) * 2 + 77
    en = oracle.cauchy1(k, p)
    data = rand((3, k, C_), 77)
    par = [[np.zeros(C_, dtype=np.uint8) for _ in range(p)] for _ in range(3)]
    for s in range(3):
        cpuq.encode(s, k, p, list(data[s]), par[s])
    cpuq.flush()
    for s in range(3):
        assert np.array_equal(np.stack(par[s]), oracle.encode_data(en[k:], data[s])), s
    full = np.concatenate([data[0], np.stack(par[0])])
    work = full.copy()
    work[[3, 17, 21]] = 0
    cpuq.recover(100, k, p, work, [3, 17, 21])
    cpuq.flush()
    assert np.array_equal(work, full)
    k, p = 8, 2
    par0 = rand((p, C_), 78)
    old, new = rand((2, C_), 79)
    got = par0.copy()
    cpuq.update(200, k, p, 5, old, new, [got[0], got[1]])
    cpuq.flush()
    bm = bytes([1 << 5, 0])
    want = oracle.agg_update_parity(k, p, C_, 1, bm, old[None], new[None], [(0, k * C_)], par0)
    assert np.array_equal(got, want)
    assert all(rc == 0 for rc in cpuq.done.values())


def test_cpu_queue_batches_and_drain(ecglib, oracle):
    """Destroy drains: every callback runs before ecg_queue_destroy
    returns, the outputs complete."""
    k, p, C_ = 4, 2, 4096
    q = ecglib.Queue(None, max_batch=64, max_wait_us=1000000)
    data = rand((10, k, C_), 5)
    par = [[np.zeros(C_, dtype=np.uint8) for _ in range(p)] for _ in range(10)]
    for s in range(10):
        q.encode(s, k, p, list(data[s]), par[s])
    keep = q.done
    q.close()
    assert len(keep) == 10 and all(rc == 0 for rc in keep.values())
    en = oracle.cauchy1(k, p)
    for s in range(10):
        assert np.array_equal(np.stack(par[s]), oracle.encode_data(en[k:], data[s]))


def test_cpu_queue_lone_request_closes_at_once(ecglib, oracle):
    """A lone request does not wait max_wait_us (here 5 s) for company: with
    a completion thread free and no other work its batch closes at once."""
    import time

    k, p, C_ = 4, 2, 4096
    q = ecglib.Queue(None, max_batch=64, max_wait_us=5000000)
    try:
        data = rand((k, C_), 9)
        par = [np.zeros(C_, dtype=np.uint8) for _ in range(p)]
        t0 = time.perf_counter()
        q.encode(1, k, p, list(data), par)
        while 1 not in q.done and time.perf_counter() - t0 < 6.0:
            time.sleep(0.0005)
        assert q.done.get(1) == 0 and time.perf_counter() - t0 < 1.0
        assert np.array_equal(np.stack(par), oracle.encode_data(oracle.cauchy1(k, p)[k:], data))
    finally:
        q.close()


def test_cpu_queue_bad_arguments(cpuq, ecglib):
    L = ecglib.lib()
    assert L.ecg_queue_recover(cpuq.h, 4, 2, 4096, None, None, 0, None, None) == -ecglib.DER_INVAL
    err = ecglib._u32([0, 1, 2])
    buf = np.zeros(6 * 4096, dtype=np.uint8)
    assert L.ecg_queue_recover(cpuq.h, 4, 2, 4096, ecglib._u8(buf), err, 3, None, None) == -ecglib.DER_DATA_LOSS
