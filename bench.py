#!/usr/bin/env python3
"""EC encode+decode GiB/s with device-resident stripes (BASELINE.json metric).

Step (configs[1] of BASELINE.json, per GPU): EC_4P2, 1 MiB cells, 1024
stripes --
  * encode: client write layout, data [S][k][C] -> parity [p][S][C]
    (obj_ec_recx_encode's loop, ref:src/object/cli_ec.c:593-663), and
  * degraded decode: recovery layout [S][k+p][C], cells {d0,d1} lost,
    regenerated in place from the first k survivors
    (obj_ec_recov_data, ref:src/object/cli_ec.c:2814-2885).
value = user bytes through the codec (k*C*S per encode + k*C*S per decode,
summed over ranks) / wall time of K steps, GiB/s.

Multi-GPU: stripes are independent, so each GPU owns its own
batch (weak scaling; `enc_16p2_strong` splits a fixed 8192-stripe total) and
there is no data-path collective.
  * `--gpus N` with no WORLD_SIZE in the environment spawns N rank processes
    itself (one per device, before anything touches the GPU); under
    torch.distributed.run the launcher's ranks are used.  torch.distributed
    (gloo) only provides the barrier and the max-over-ranks of the elapsed
    time.  Ranks must land on distinct devices (--allow-shared-device to
    rehearse on fewer); n_gpus counts distinct PCI devices.
  * `--sharder lib` runs the N shards in ONE process through the library's
    own multi-device sharder (include/ecg_multi.h): one host thread +
    context per device.

roofline: the dominant kernel (ecg_mm_kernel<4,2>, which serves both the
encode and the 2-erasure decode) -- algorithmic bytes per launch
(k+rows)*C*S / mean launch duration from HIP events on its stream, against
the 8 TB/s HBM spec peak; `traffic` is copied from the committed rocprofv3
PMC pass of this command (`traffic_source` names the file), not measured in
the run.
cpu_baseline: the oracle's SIMD ISA-L-equivalent restatement (GFNI/AVX-512
+ OpenMP) on a bounded sample with a >= 1 GiB working set, rank 0 at N=1
only: every core of the process's affinity mask (3 repeats, median and
range) and 1 core, load average before/after, and per-config rows for
configs 1, 3 and the config-4 per-GPU shard beside the GPU detail rows.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)
PARITY_ROW_PAD = 4096
HBM_PEAK_GBS = 8000.0          # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md
ROUND = "r06"

# name -> (k, p, cell bytes, stripes, ops, strong scaling?)
WORKLOADS = {
    "enc_dec_4p2": (4, 2, 1 << 20, 1024, ("enc", "dec"), False),
    "dec_8p2": (8, 2, 1 << 20, 512, ("dec",), False),
    "enc_8p2": (8, 2, 1 << 20, 512, ("enc",), False),
    "enc_16p2_strong": (16, 2, 128 << 10, 8192, ("enc",), True),
    # configs[4]: stripes in pinned host memory, PCIe-inclusive (never the headline)
    "rebuild_stream_8p2": (8, 2, 1 << 20, 64, ("enc_host", "dec_host"), False),
}
HOST_CHUNK = 4          # stripes per staging chunk (profiles/r02/host_chunk_sweep/: 16 -> 4 = 0.92 -> 0.945 of H2D)
MARKER = 0x5A           # erased cells are overwritten with this before any decode runs


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="enc_dec_4p2", choices=sorted(WORKLOADS),
                    help="enc_dec_4p2 = BASELINE configs[1] (+ its decode); dec_8p2 = configs[2]; "
                         "enc_8p2 = the north-star EC_8P2 encode; "
                         "enc_16p2_strong = configs[3] (8192 stripes split across GPUs); "
                         "rebuild_stream_8p2 = configs[4] (host-resident, PCIe-inclusive)")
    ap.add_argument("--sharder", default="procs", choices=("procs", "lib"),
                    help="procs: one process per GPU; lib: one process, the library's ecg_multi sharder")
    ap.add_argument("--allow-shared-device", action="store_true",
                    help="permit more ranks/shards than visible devices (rehearsal on a small box)")
    ap.add_argument("--cpu-seconds", type=float, default=16.0, help="CPU baseline time budget (headline runs; the per-config rows take about as long again)")
    ap.add_argument("--no-detail", action="store_true", help="skip the extra per-config rows")
    ap.add_argument("--host-chunk", type=int, default=0,
                    help=f"stripes per staging chunk of the host-resident workloads (default {HOST_CHUNK})")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--wg-per-cu", type=int, default=0,
                    help="product-kernel blocks per CU (ecg_set_wg_per_cu): 0 per-shape default, 255 uncapped")
    ap.add_argument("--profile-only", action="store_true", help="just the timed loop (for rocprofv3)")
    ap.add_argument("--rehearse", action="store_true",
                    help="CPU-only rehearsal of launcher, barrier and aggregation: no GPU work, the "
                         "line carries rehearsal=true and its value is not a measurement")
    return ap.parse_args(argv)


def describe(name, k, p, C, S, ops, n_shards=1):
    parts = []
    if "enc" in ops:
        parts.append("encode (data [S][k][C] -> parity [p][S][C], row pitch S*C+4KiB)")
    if "dec" in ops:
        parts.append("degraded decode of cells d0,d1 in [S][k+p][C]")
    per = "per GPU" if not WORKLOADS[name][5] else f"per GPU ({WORKLOADS[name][3]} total, split {n_shards} ways)"
    return f"EC_{k}P{p} {C >> 10} KiB cells x {S} stripes {per}: " + " + ".join(parts)


# ------------------------------------------------------------------ launcher
def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args) -> int:
    """`--gpus N` without a launcher: start N rank processes (RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_* set) and wait.  This parent process
    never touches the GPU; rank 0 prints the JSON line.  If one rank fails the
    others are stopped (their exact PIDs), so nobody hangs in a barrier."""
    port = free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r if r > 0 else 128 - r
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def rank_numa(args):
    """A rank of an N-GPU run (N > 1) runs on the CPUs of its GPU's NUMA node:
    pinned here, from sysfs alone, before torch or libecg start the GPU
    runtime, so the runtime's threads and this rank's pinned staging inherit
    it (daos_amd/numa.py).  N = 1 only reports the node."""
    if args.rehearse:
        return None
    from daos_amd import numa

    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))
    nvis = len(numa.visible_gpus()) or 1
    if world > 1 and args.sharder == "procs":
        return numa.pin_to_device(local % nvis)
    return numa.placement(local % nvis)


def dist_init():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def max_over_ranks(world, x: float) -> float:
    if world == 1:
        return x
    import torch
    import torch.distributed as dist

    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather(world, obj):
    if world == 1:
        return [obj]
    import torch.distributed as dist

    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def finish_dist(world):
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


# ------------------------------------------------------------------ workloads
def fill_device(ctx, buf, nbytes, config_id, chunk=256 << 20):
    """Seeded random bytes; one generated chunk tiled over the buffer (the
    codec's cost does not depend on cross-chunk uniqueness).  Returns the
    chunk, from which the expected byte at any offset o is blk[o % blk.size]."""
    from tools.datagen import stripe_bytes

    blk = stripe_bytes(min(chunk, nbytes), config_id)
    off = 0
    while off < nbytes:
        n = min(blk.size, nbytes - off)
        buf.upload(blk[:n], offset=off)
        off += n
    return blk


def tiled(blk, off, n):
    """Bytes [off, off + n) of blk tiled without end."""
    import numpy as np

    idx = (np.arange(n, dtype=np.int64) + off) % blk.size
    return blk[idx]


class Workload:
    """One shard's EC batch on one device: encode (client layout) + decode
    (recovery layout).  The erased cells of the recovery image hold a marker
    until the first decode regenerates them, so verify() fails for a decode
    that wrote nothing."""

    def __init__(self, ctx, k, p, C, S, ops=("enc", "dec"), err=(0, 1), config_id=2):
        self.ctx, self.k, self.p, self.C, self.S, self.err = ctx, k, p, C, S, list(err)
        self.ops = tuple(ops)
        # Parity rows [p][S][C] at a pitch of S*C + 4 KiB: rows exactly a power
        # of two apart alias in HBM and cost EC_8P2 encode ~10 %
        # (profiles/r01/tune5_parity_row_aliasing.json, tune6_pitch.json).
        self.prow = S * C + PARITY_ROW_PAD
        self.data = ctx.alloc(max(1, S * k * C))
        self.parity = ctx.alloc(p * self.prow)
        # the recovery image only when this workload decodes
        self.stripes = ctx.alloc(max(1, S * (k + p) * C)) if "dec" in self.ops else None
        self.events = []        # per timed step: (start, stop) per op
        if S == 0:
            return
        fill_device(ctx, self.data, S * k * C, config_id)
        if "dec" in self.ops:
            # recovery buffer: a consistent [S][k+p][C] image (encode in place)
            self.img_blk = fill_device(ctx, self.stripes, S * (k + p) * C, config_id + 1)
            st = (k + p) * C
            ctx.encode(k, p, C, S, self.stripes.ptr, st, self.stripes.ptr + k * C, C, st)
            ctx.sync()
            from daos_amd import ecg

            for s in range(S):
                for e in self.err:
                    ecg._chk(ecg.lib().ecg_memset(ctx.h, self.stripes.ptr + s * st + e * C, MARKER, C, None),
                             "memset")
            ctx.sync()

    def enc_call(self):
        return (self.data.ptr, self.parity.ptr)

    def step(self, timed=False):
        c, k, p, C, S = self.ctx, self.k, self.p, self.C, self.S
        evs = []
        for op in self.ops:
            ev = (c.event(), c.event()) if timed else None
            if timed:
                c.record(ev[0])
            if op == "enc":
                c.encode(k, p, C, S, self.data.ptr, k * C, self.parity.ptr, self.prow, C)
            else:
                c.recover(k, p, C, S, self.stripes.ptr, (k + p) * C, self.err)
            if timed:
                c.record(ev[1])
                evs.append(ev)
        if timed:
            self.events.append(evs)

    def kernel_ms(self):
        """{op: [ms per timed step]}, read after the timed region."""
        out = {op: [] for op in self.ops}
        for evs in self.events:
            for op, (a, b) in zip(self.ops, evs):
                out[op].append(self.ctx.elapsed_ms(a, b))
                self.ctx.destroy_event(a)
                self.ctx.destroy_event(b)
        self.events = []
        return out

    def verify(self, nsample=3):
        """After the timed steps, on sampled stripes: the decode regenerated
        the erased cells (they held MARKER before) with the original bytes, and
        the timed encode's parity, put in a fresh stripe with d0/d1 erased,
        decodes back to its data.  The oracle checks live in tests/; this is
        the run's own consistency check."""
        import numpy as np

        if self.S == 0:
            return {}
        k, p, C, S = self.k, self.p, self.C, self.S
        st = (k + p) * C
        samples = sorted({0, S // 2, S - 1})[:nsample]
        out = {}
        if "dec" in self.ops:
            ok = True
            for s in samples:
                for e in self.err:
                    got = self.stripes.download(C, offset=s * st + e * C)
                    ok &= bool(np.array_equal(got, tiled(self.img_blk, s * st + e * C, C)))
            out["decode_regenerated_erased_cells"] = ok
        if "enc" in self.ops:
            ok = True
            probe = self.ctx.alloc(st)
            # one-stripe probes run the runtime-shaped kernel, so the
            # headline kernel's rocprofv3 statistics only count batch launches
            self.ctx.set_launch(0, 0, 1)
            for s in samples:
                cells = self.data.download(k * C, offset=s * k * C)
                par = np.stack([self.parity.download(C, offset=r * self.prow + s * C) for r in range(p)])
                img = np.concatenate([cells.reshape(k, C), par]).copy()
                img[self.err] = MARKER
                probe.upload(img)
                self.ctx.recover(k, p, C, 1, probe.ptr, st, self.err)
                self.ctx.sync()
                ok &= bool(np.array_equal(probe.download()[:k * C], cells))
            self.ctx.set_launch(0, 0, 0)
            probe.free()
            out["encode_parity_decodes_to_data"] = ok
        return out

    def user_bytes_per_step(self):
        return len(self.ops) * self.k * self.C * self.S

    def alg_bytes(self, op):
        # encode: read k, write p cells; decode: read k survivors, write nerrs
        return (self.k + (self.p if op == "enc" else len(self.err))) * self.C * self.S

    def free(self):
        for b in (self.data, self.parity, self.stripes):
            if b is not None:
                b.free()


class HostWorkload:
    """BASELINE configs[4], the rebuild stream: one rank's stripes live in
    pinned host memory (engine-side bio/NIC buffers); a step is one encode
    batch (data [S][k][C] -> parity [p][S][C]) and one 2-erasure recovery
    batch (in place in [S][k+p][C]), each streamed through device staging by
    ecg_encode_host / ecg_recover_host (H2D || kernel || D2H on 3 streams).
    PCIe-bound by construction."""

    def __init__(self, ctx, k, p, C, S, ops=("enc_host", "dec_host"), err=(0, 1), config_id=9, chunk=0):
        from tools.datagen import stripe_bytes

        self.ctx, self.k, self.p, self.C, self.S, self.err = ctx, k, p, C, S, list(err)
        self.chunk = chunk or HOST_CHUNK
        self.ops = tuple(ops)
        self.data = ctx.host_alloc(S * k * C)
        self.parity = ctx.host_alloc(S * p * C)
        self.stripes = ctx.host_alloc(S * (k + p) * C)
        blk = stripe_bytes(min(256 << 20, S * k * C), config_id)
        a = self.data.array
        for off in range(0, a.size, blk.size):
            n = min(blk.size, a.size - off)
            a[off:off + n] = blk[:n]
        ctx.encode_host(k, p, C, S, a, self.parity.array, chunk=self.chunk)
        img = self.stripes.array.reshape(S, k + p, C)
        img[:, :k] = a.reshape(S, k, C)
        img[:, k:] = self.parity.array.reshape(p, S, C).transpose(1, 0, 2)
        img[:, self.err] = MARKER           # the first recovery must regenerate them
        self.parity.array[:] = 0            # the first timed-region encode must write them
        self.events = []

    def step(self, timed=False):
        c, k, p, C, S = self.ctx, self.k, self.p, self.C, self.S
        if "enc_host" in self.ops:
            c.encode_host(k, p, C, S, self.data.array, self.parity.array, chunk=self.chunk)
        if "dec_host" in self.ops:
            c.recover_host(k, p, C, S, self.stripes.array, self.err, chunk=self.chunk)

    def kernel_ms(self):
        return {}

    def user_bytes_per_step(self):
        return len(self.ops) * self.k * self.C * self.S

    def h2d_bytes_per_step(self):
        # encode: k cells in; recovery: the k survivors in
        return len(self.ops) * self.k * self.C * self.S

    def d2h_bytes_per_step(self):
        n = 0
        if "enc_host" in self.ops:
            n += self.p * self.C * self.S
        if "dec_host" in self.ops:
            n += len(self.err) * self.C * self.S
        return n

    def verify(self):
        """Recovered cells (MARKER before the first step) equal the original
        data; and the timed encode's parity, copied into the image with d0/d1
        erased again, decodes back to the data."""
        import numpy as np

        S, k, p, C = self.S, self.k, self.p, self.C
        img = self.stripes.array.reshape(S, k + p, C)
        data = self.data.array.reshape(S, k, C)
        out = {"decode_regenerated_erased_cells": bool(np.array_equal(img[:, :k], data))}
        img[:, k:] = self.parity.array.reshape(p, S, C).transpose(1, 0, 2)
        img[:, self.err] = MARKER
        self.ctx.recover_host(k, p, C, S, self.stripes.array, self.err, chunk=self.chunk)
        out["encode_parity_decodes_to_data"] = bool(np.array_equal(img[:, :k], data))
        return out

    def free(self):
        for b in (self.data, self.parity, self.stripes):
            b.free()


class HostMultiWorkload(HostWorkload):
    """`--sharder lib` for configs[4]: ONE batch of S = stripes-per-GPU x N
    in pinned host memory, split by ecg_multi_encode_host /
    ecg_multi_recover_host into contiguous stripe ranges, each shard
    streaming its range through its own device's staging (include/ecg_multi.h)."""

    def __init__(self, m, k, p, C, S_per, ops, chunk=0):
        self.m = m
        super().__init__(m.ctxs[0], k, p, C, S_per * m.n, ops=ops, chunk=chunk)

    def step(self, timed=False):
        k, p, C, S = self.k, self.p, self.C, self.S
        if "enc_host" in self.ops:
            self.m.encode_host(k, p, C, S, self.data.array, self.parity.array, chunk=self.chunk)
        if "dec_host" in self.ops:
            self.m.recover_host(k, p, C, S, self.stripes.array, self.err, chunk=self.chunk)

    def sync(self):                 # the _host calls return with their outputs in host memory
        pass


class MultiWorkload:
    """`--sharder lib`: N shards in one process through ecg_multi (one host
    thread + context per device).  Each shard is a Workload on its own
    context; a step is one ecg_multi_encode + one ecg_multi_recover over all
    shards (asynchronous), the timed region ends with ecg_multi_sync."""

    def __init__(self, m, k, p, C, S_total, ops, strong):
        self.m, self.k, self.p, self.C = m, k, p, C
        self.ops = tuple(ops)
        self.shards = []
        for i, c in enumerate(m.ctxs):
            S = m.range(S_total, i)[1] if strong else S_total
            self.shards.append(Workload(c, k, p, C, S, ops=ops, config_id=2))
        self.err = self.shards[0].err
        self.S = self.shards[0].S

    def step(self, timed=False):
        from daos_amd import ecg

        k, p, C = self.k, self.p, self.C
        w0 = self.shards[0]
        ns = [w.S for w in self.shards]
        evs = []
        for op in self.ops:
            ev = (w0.ctx.event(), w0.ctx.event()) if timed else None
            if timed:
                w0.ctx.record(ev[0])
            if op == "enc":
                self.m.encode(k, p, C, ns, [w.data.ptr for w in self.shards], k * C,
                              [w.parity.ptr for w in self.shards], w0.prow, C, flags=ecg.MULTI_ASYNC)
            else:
                self.m.recover(k, p, C, ns, [w.stripes.ptr for w in self.shards], (k + p) * C, self.err,
                               flags=ecg.MULTI_ASYNC)
            if timed:
                w0.ctx.record(ev[1])
                evs.append(ev)
        if timed:
            w0.events.append(evs)

    def sync(self):
        self.m.sync()

    def kernel_ms(self):
        return self.shards[0].kernel_ms()

    def verify(self):
        out = {}
        for w in self.shards:
            for key, v in w.verify().items():
                out[key] = out.get(key, True) and v
        return out

    def user_bytes_per_step(self):
        return sum(w.user_bytes_per_step() for w in self.shards)

    def alg_bytes(self, op):
        return self.shards[0].alg_bytes(op)

    def free(self):
        for w in self.shards:
            w.free()


# ------------------------------------------------------------------ measurements
def pinned_copy_rates(ctx, n=1 << 30):
    """Raw pinned hipMemcpy H2D / D2H GB/s on this rank's device."""
    h = ctx.host_alloc(n)
    d = ctx.alloc(n)
    h.array[:] = 7
    from daos_amd import ecg

    out = {}
    for kind, name in ((0, "h2d"), (1, "d2h")):
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            if kind == 0:
                ecg._chk(ecg.lib().ecg_memcpy(ctx.h, d.ptr, h.ptr, n, 0, None), "h2d")
            else:
                ecg._chk(ecg.lib().ecg_memcpy(ctx.h, h.ptr, d.ptr, n, 1, None), "d2h")
            ctx.sync()
            ts.append(time.perf_counter() - t0)
        out[name] = round(n / sorted(ts)[1] / 1e9, 2)
    h.free()
    d.free()
    return out


def time_kernel(ctx, fn, iters, warm=3, blocks_out=None):
    """Median kernel time of `iters` timed blocks of launches issued back to
    back, as an engine streams batches: an event between consecutive blocks,
    all read after the last one (no host synchronisation -- and no idle GPU
    gap -- between launches).  A block is one launch, or several for launches
    shorter than ~1 ms (time_interleaved)."""
    return time_interleaved(ctx, [fn], iters, warm, blocks_out)[0]


# Launches per timed block: enough for ~1 ms of work.  An event recorded
# between two launches costs the stream ~5 us (the next launch waits for the
# event's completion signal): a 60 us EC_2P1 128 KiB x 1024 launch timed one
# per event pair read 65.4 us (0.77 of the HBM spec, BENCH_r05) where the kernel
# trace gives 59.7 us and blocks of back-to-back launches 60.4 us with no fixed
# per-launch cost in the batch-size fit (0.83-0.84, tools/short_launch.py,
# profiles/r06/short_launch/).  Launches of >= 0.5 ms keep one per block.
BLOCK_TARGET_MS = 1.0


def time_interleaved(ctx, fns, iters, warm=3, blocks_out=None):
    """Median kernel time of each of `fns`, launched in turn (one block of
    each per round): the box's clocks drift over a long run, so timing one
    configuration's block of launches after another's biases a ratio.  The
    launches go back to back with an event at every block boundary, read after
    the last launch (a host wait per launch would leave the GPU idle between
    launches, which short launches feel: EC_16P2 x 1024 ran 0.43 ms that way
    against 0.40 ms for the launch tuner's back-to-back arms, round 3).  Each
    fn's block holds B launches, B = BLOCK_TARGET_MS / its warm-up time per
    launch (1 for launches of >= 0.5 ms); blocks_out (a list) receives the Bs."""
    for _ in range(warm):           # warm-up rounds interleaved like the timed ones
        for fn in fns:
            fn()
    ctx.sync()
    # per-fn launch time from 4 back-to-back launches each -> launches per block
    nb = []
    e0, e1 = ctx.event(), ctx.event()
    for fn in fns:
        ctx.record(e0)
        for _ in range(4):
            fn()
        ctx.record(e1)
        ctx.sync()
        est = ctx.elapsed_ms(e0, e1) / 4
        nb.append(max(1, min(64, int(round(BLOCK_TARGET_MS / est)))) if est < BLOCK_TARGET_MS / 2 else 1)
    ctx.destroy_event(e0)
    ctx.destroy_event(e1)
    if blocks_out is not None:
        blocks_out[:] = nb
    evs = [ctx.event() for _ in range(iters * len(fns) + 1)]
    ctx.record(evs[0])
    n = 0
    for _ in range(iters):
        for fn, b in zip(fns, nb):
            for _ in range(b):
                fn()
            n += 1
            ctx.record(evs[n])
    ms = [[] for _ in fns]
    for i in range(n):
        ms[i % len(fns)].append(ctx.elapsed_ms(evs[i], evs[i + 1]) / nb[i % len(fns)])
    for e in evs:
        ctx.destroy_event(e)
    return [sorted(v)[len(v) // 2] for v in ms]


def measured_ceilings(ctx, iters=11):
    """This box's streaming rates (GB/s), each mode at its best measured
    geometry (profiles/r01/tune2*.json): reads with 512 persistent blocks,
    writes / copies with one 4 x 16 B slice per thread."""
    n = 2 << 30
    a, b = ctx.alloc(n), ctx.alloc(n)
    a.fill(0x3C)
    out = {}
    for mode, name, nbytes, blocks in ((0, "copy", 2 * n, 0), (1, "read", n, 512), (2, "write", n, 0)):
        ctx.set_launch(blocks, 0, 0)
        ms = time_kernel(ctx, lambda: ctx.copy_kernel(b.ptr, a.ptr, n, mode), iters)
        out[name] = round(nbytes / ms / 1e6, 1)
    ctx.set_launch(0, 0, 0)
    a.free()
    b.free()
    return out


def mix_ceiling(ceil, read_frac):
    """Time-weighted ceiling for a read/write mix from the measured rates."""
    return 1.0 / (read_frac / ceil["read"] + (1 - read_frac) / ceil["write"])


DETAIL_SHAPES = (("EC_8P2_1MiB_encode", 8, 2, 1 << 20, 512, "enc"),
                 ("EC_8P2_1MiB_decode_d0d1", 8, 2, 1 << 20, 512, "dec"),
                 ("EC_16P2_128KiB_encode", 16, 2, 128 << 10, 1024, "enc"),
                 ("EC_2P1_128KiB_encode", 2, 1, 128 << 10, 1024, "enc"))


def offset_rows(ctx, aligned, iters=11):
    """EC_8P2 1 MiB client-layout encode with operands at a byte offset of
    their allocation (DAOS rounds parity rows to 8 bytes only,
    ref:src/object/cli_ec.c:86; user cells carry no alignment,
    ref:src/object/cli_ec.c:510-536): parity rows at +8 or +4 run the
    dword-lane kernel, at +1 (and at +1 with rows misaligned by different
    amounts: row pitch +1) the same lanes with misaligned dword stores; data
    cells at +1 the funnel-shift kernel.  The byte kernel, which the launcher
    no longer picks (launch variant 2 forces it), is timed on 32 stripes for
    the record: it is ~8x slower.  Each 512-stripe row's `of_aligned` = the
    aligned row's ms / this ms."""
    from daos_amd import ecg

    k, p, C = 8, 2, 1 << 20
    rows = {}
    for what, off, S, warm in (("parity", 8, 512, 40), ("parity", 4, 512, 40), ("data", 1, 512, 40),
                               ("parity", 1, 512, 40), ("parity_unequal", 1, 512, 40),
                               ("parity_byte_kernel", 1, 32, 2)):
        data = ctx.alloc(S * k * C + 64)
        fill_device(ctx, data, S * k * C, 7)
        pitch = S * C + PARITY_ROW_PAD + (what == "parity_unequal")
        par = ctx.alloc(p * pitch + 64)
        doff, poff = (off, 0) if what == "data" else (0, off)
        ctx.set_launch(0, 0, 2 if what == "parity_byte_kernel" else 0)
        try:
            ms = time_kernel(ctx, lambda: ctx.encode(k, p, C, S, data.ptr + doff, k * C, par.ptr + poff, pitch,
                                                     C), iters, warm=warm)
        finally:
            ctx.set_launch(0, 0, 0)
        alg = (k + p) * C * S
        row = {f"{what}_offset_bytes": off, "stripes": S, "ms": round(ms, 4),
               "GiBps_user": round(k * C * S / (ms / 1e3) / GIB, 1), "alg_GBps": round(alg / ms / 1e6, 1),
               "roofline_frac": round(alg / ms / 1e6 / HBM_PEAK_GBS, 4), "kernel": ecg.last_kernel()}
        if aligned and S == 512:
            row["of_aligned"] = round(aligned["ms"] / ms, 4)
        rows[f"EC_8P2_1MiB_encode_{what}_off{off}"] = row
        data.free()
        par.free()
    return rows


def sgl_rows(ctx, aligned, iters=11):
    """The client's full-stripe encode over a device-resident sgl
    (ecg_obj_ec_recx_encode, restating obj_ec_recx_encode /
    obj_ec_stripe_encode, ref:src/object/cli_ec.c:476-546, 593-663): EC_8P2
    1 MiB x 512 stripes of one recx, parity into p separate buffers (the
    oer_pbufs layout, :75-97).  One iov: every cell used in place at an
    affine address, so the call runs the strided product kernel; 64 iovs of
    random lengths with gaps between them: cells cut across iovs are gathered
    into device scratch, the rest used in place, one pointer-table launch.
    Timed per call (host walk, table upload, gathers and product included);
    `of_aligned` = the plain encode row's ms / this ms."""
    import ctypes

    import numpy as np
    from daos_amd import ecg

    k, p, C, S = 8, 2, 1 << 20, 512
    total = S * k * C
    rng = np.random.default_rng(11)
    rows = {}
    L = ecg.lib()
    for name, n_iov in (("one_iov", 1), ("64_iovs", 64)):
        cuts = sorted(set(int(x) for x in rng.integers(1, total, n_iov - 1))) if n_iov > 1 else []
        lens = np.diff([0] + cuts + [total]).tolist()
        buf = ctx.alloc(total + 256 * n_iov)
        fill_device(ctx, buf, total + 256 * n_iov, 9)
        iovs, off = [], 0
        for ln in lens:
            iovs.append(ecg.Iov(buf.ptr + off, ln, ln))
            off += ln + (256 if n_iov > 1 else 0)
        iov_arr = (ecg.Iov * len(iovs))(*iovs)
        rx = (ecg.EcRecx * 1)(ecg.EcRecx(0, S, 0))
        pbufs = [ctx.alloc(S * C) for _ in range(p)]
        pb = (ctypes.c_void_p * p)(*[b.ptr for b in pbufs])
        oc = (37 << 24) | 1                         # OC_EC_8P2G1

        def fn():
            ecg._chk(L.ecg_obj_ec_recx_encode(ctx.h, oc, C, iov_arr, len(iovs), rx, 1, pb, None), "recx_encode")

        ms = time_kernel(ctx, fn, iters, warm=40)
        alg = (k + p) * C * S
        row = {"iovs": n_iov, "stripes": S, "ms": round(ms, 4), "GiBps_user": round(k * C * S / (ms / 1e3) / GIB, 1),
               "alg_GBps": round(alg / ms / 1e6, 1), "roofline_frac": round(alg / ms / 1e6 / HBM_PEAK_GBS, 4),
               "kernel": ecg.last_kernel()}
        if aligned:
            row["of_aligned"] = round(aligned["ms"] / ms, 4)
        rows[f"EC_8P2_1MiB_recx_encode_sgl_{name}"] = row
        buf.free()
        for b in pbufs:
            b.free()
    return rows


def update_rows(ctx, iters=11):
    """Aggregation's delta parity update (agg_update_parity: xor_gen of old and
    new, then ec_encode_data_update per updated cell,
    ref:src/object/srv_ec_aggregate.c:1062-1105) batched over stripes:
    parity[r] ^= sum_i coef[r][cell_i] * (old_i ^ new_i), one fused launch
    reading old, new and the parity and writing the parity -- (2n + 2p) * C
    algorithmic bytes per stripe for n updated cells."""
    from daos_amd import ecg

    k, p, C, S = 8, 2, 1 << 20, 512
    rows = {}
    for cells in ([3], [1, 6]):
        n = len(cells)
        old, new = ctx.alloc(S * n * C), ctx.alloc(S * n * C)
        fill_device(ctx, old, S * n * C, 12)
        fill_device(ctx, new, S * n * C, 13)
        pitch = S * C + PARITY_ROW_PAD
        par = ctx.alloc(p * pitch)
        fill_device(ctx, par, p * pitch, 14)
        ms = time_kernel(ctx, lambda: ctx.update(k, p, C, S, cells, old.ptr, new.ptr, n * C, par.ptr, pitch, C),
                         iters, warm=40)
        alg = (2 * n + 2 * p) * C * S
        rows[f"EC_8P2_1MiB_update_{n}cell"] = {
            "cells_per_stripe": n, "stripes": S, "ms": round(ms, 4),
            "GiBps_updated": round(n * C * S / (ms / 1e3) / GIB, 1), "alg_GBps": round(alg / ms / 1e6, 1),
            "roofline_frac": round(alg / ms / 1e6 / HBM_PEAK_GBS, 4), "kernel": ecg.last_kernel()}
        for b in (old, new, par):
            b.free()
    return rows


def layout_rows(ctx, iters=11):
    """The caller's parity layout, not the bench's: EC_4P2 1 MiB
    x 1024 (the headline's encode) and EC_8P2 1 MiB x 512, client-layout
    encode with the p parity rows
      padded   -- one buffer, rows S*C + 4 KiB apart (the headline's layout);
      unpadded -- one buffer, rows exactly S*C apart;
      separate -- p separate hipMalloc allocations of S*C bytes, as
                  obj_ec_pbufs_init allocates oer_pbufs (ref:src/object/
                  cli_ec.c:75-97), written through per-row cell offsets.
    Launches interleaved (one of each per round, so clock drift cannot bias
    the ratio); `of_padded` = the padded row's ms / this row's ms."""
    import numpy as np
    from daos_amd import ecg

    rows = {}
    for name, k, p, C, S in (("EC_4P2_1MiB_x1024", 4, 2, 1 << 20, 1024), ("EC_8P2_1MiB_x512", 8, 2, 1 << 20, 512)):
        data = ctx.alloc(S * k * C)
        fill_device(ctx, data, S * k * C, 10)
        padded = ctx.alloc(p * (S * C + PARITY_ROW_PAD))
        unpadded = ctx.alloc(p * S * C)
        sep = [ctx.alloc(S * C) for _ in range(p)]
        base = min(b.ptr for b in sep)
        soff = [j * C for j in range(k)]
        doff = [b.ptr - base for b in sep]
        coef = ecg.cauchy1(k, p)[k:]
        fns = {"padded": lambda: ctx.encode(k, p, C, S, data.ptr, k * C, padded.ptr, S * C + PARITY_ROW_PAD, C),
               "unpadded": lambda: ctx.encode(k, p, C, S, data.ptr, k * C, unpadded.ptr, S * C, C),
               "separate": lambda: ctx.matmul(coef, C, S, data.ptr, soff, k * C, base, doff, C)}
        ms = dict(zip(fns, time_interleaved(ctx, list(fns.values()), iters, warm=40)))
        kern = ecg.last_kernel()
        # the separate rows' bytes equal the padded rows' (same product, other addresses)
        ok = all(np.array_equal(sep[r].download(C, offset=s * C), padded.download(C, offset=r * (S * C + PARITY_ROW_PAD)
                                                                                 + s * C))
                 for r in range(p) for s in (0, S - 1))
        alg = (k + p) * C * S
        for lay, t in ms.items():
            rows[f"{name}_encode_parity_{lay}"] = {
                "layout": lay, "ms": round(t, 4), "GiBps_user": round(k * C * S / (t / 1e3) / GIB, 1),
                "alg_GBps": round(alg / t / 1e6, 1), "roofline_frac": round(alg / t / 1e6 / HBM_PEAK_GBS, 4),
                "of_padded": round(ms["padded"] / t, 4), "kernel": kern,
                **({"parity_row_addresses": [hex(b.ptr) for b in sep], "matches_padded": ok}
                   if lay == "separate" else {})}
        for b in [data, padded, unpadded] + sep:
            b.free()
    return rows


def detail_rows(ctx, ceil, iters=11, shapes=DETAIL_SHAPES, csum=True):
    """Extra device-resident rows (per GPU): the north-star EC_8P2 encode,
    EC_8P2 2-erasure decode, EC_16P2 128 KiB encode, EC_2P1 128 KiB encode.
    Encodes use the client write layout (data [S][k][C], parity [p][S][C] at
    the padded row pitch, as the headline); decodes the recovery layout
    [S][k+p][C].  Median kernel time over `iters` launches."""
    from daos_amd import ecg

    rows = {}
    for name, k, p, C, S, mode in shapes:
        st = (k + p) * C
        # encodes: the data cells alone, [S][k][C] (DAOS's client write buffer); decodes:
        # the whole recovery image [S][k+p][C]
        nb = S * (k * C if mode == "enc" else st)
        buf = ctx.alloc(nb)
        fill_device(ctx, buf, nb, 7)
        if mode == "enc":
            pitch = S * C + PARITY_ROW_PAD          # data [S][k][C] in buf, parity rows in buf2
            buf2 = ctx.alloc(p * pitch)
            par = buf2.ptr
            fn = (lambda buf=buf, k=k, p=p, C=C, S=S, par=par, pitch=pitch:
                  ctx.encode(k, p, C, S, buf.ptr, k * C, par, pitch, C))
            rd, wr = k, p
        else:
            buf2 = None
            ctx.encode(k, p, C, S, buf.ptr, st, buf.ptr + k * C, C, st)
            fn = (lambda buf=buf, k=k, p=p, C=C, S=S, st=st:
                  ctx.recover(k, p, C, S, buf.ptr, st, [0, 1]))
            rd, wr = k, 2
        # 80 warm-up launches: the launch tuner (include/ecg.h ecg_set_autotune) times its
        # two arms over the first 23 launches of a wide shape (its capped arm last, so a kept
        # cap needs no switch; the first ~10-20 launches after a switch to a cap run up to
        # 12 % slow: EC_16P2 cap 2 0.434 ms, then 0.38, tools/state_check3.py,
        # profiles/r03/tuner_check/); the timed launches run its choice in steady state
        nblk = []
        ms = time_kernel(ctx, fn, iters, warm=80, blocks_out=nblk)
        tuned = (ctx.tune_state(k, p, C, S, k * C, C) if mode == "enc"
                 else ctx.tune_state(k, 2, C, S, st, st))
        alg = (rd + wr) * C * S
        gbs = alg / ms / 1e6
        mix = mix_ceiling(ceil, rd / (rd + wr))
        rows[name] = {"GiBps_user": round(k * C * S / (ms / 1e3) / GIB, 1), "alg_GBps": round(gbs, 1),
                      "roofline_frac": round(gbs / HBM_PEAK_GBS, 4),
                      "read_frac": round(k * C * S / ms / 1e6 / HBM_PEAK_GBS, 4),
                      "measured_mix_ceiling_GBps": round(mix, 1), "frac_of_measured_mix": round(gbs / mix, 4),
                      "kernel": ecg.last_kernel(), "ms": round(ms, 4), "launches_per_timed_block": nblk[0],
                      "layout": "client [S][k][C] -> [p][S][C]" if mode == "enc" else "recovery [S][k+p][C]"}
        if tuned is not None:
            rows[name]["launch_tuner"] = {"wg_per_cu": None if tuned[0] == 255 else tuned[0],
                                          "uncapped_ms": round(tuned[1], 4), "capped_ms": round(tuned[2], 4)}
        buf.free()
        if buf2 is not None:
            buf2.free()
    rows.update(offset_rows(ctx, rows.get("EC_8P2_1MiB_encode"), iters))
    rows.update(sgl_rows(ctx, rows.get("EC_8P2_1MiB_encode"), iters))
    rows.update(update_rows(ctx, iters))
    rows.update(layout_rows(ctx, iters))
    if not csum:
        return rows
    # checksums of regenerated cells (include/ecg_csum.h): EC_8P2 encode with
    # crc32 over 32 KiB chunks of the parity, fused vs the product alone, and
    # the standalone checksum kernel over 1 GiB of 1 MiB cells
    k, p, C, S = 8, 2, 1 << 20, 512
    data = ctx.alloc(S * k * C)
    fill_device(ctx, data, S * k * C, 8)
    pitch = S * C + PARITY_ROW_PAD
    par = ctx.alloc(p * pitch)
    out = ctx.alloc(p * S * (C // 32768) * 8)
    hashes = (("crc32", ecg.HASH_CRC32), ("crc64", ecg.HASH_CRC64))
    kernels = {}

    def fused(htype):
        def fn():
            ctx.encode_csum(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C, htype, 32768, 1, out.ptr)
            kernels[htype] = ecg.last_kernel()
        return fn
    # the plain encode and both fused launches interleaved (their ratio is the row's point).
    # 15 warm-up rounds: when the VALU/LDS-dense fused kernels start after the memory-bound
    # encode the core clock dips and recovers over ~10 launches (the fused launches ran
    # 0.94 -> 1.26 -> 0.95 ms while the interleaved encode stayed at 0.82-0.85 ms,
    # profiles/r02/fused_transient/kernel_trace.csv); the rows report the steady state
    fns = [lambda: ctx.encode(k, p, C, S, data.ptr, k * C, par.ptr, pitch, C)] + [fused(h) for _, h in hashes]
    enc_i, *fus_i = time_interleaved(ctx, fns, iters, warm=15)
    # the same launches in back-to-back blocks, each configuration after 20 launches of
    # itself, forward then reverse order (the mean of the two medians cancels a linear
    # drift): the steady pattern of a rebuild stream, which launches encode_csum batch
    # after batch -- and how every other detail row is timed.  A fused launch that
    # follows a plain encode starts in the encode's clock state (the transient above)
    blk = [[] for _ in fns]
    for order in (list(range(len(fns))), list(reversed(range(len(fns))))):
        for i in order:
            blk[i].append(time_kernel(ctx, fns[i], iters, warm=20))
    enc, *fus_ms = [sum(v) / len(v) for v in blk]
    for (hname, htype), fus, fi in zip(hashes, fus_ms, fus_i):
        alg = (k + p) * C * S
        rows[f"EC_8P2_1MiB_encode_{hname}_32KiB_fused"] = {
            "GiBps_user": round(k * C * S / (fus / 1e3) / GIB, 1), "alg_GBps": round(alg / fus / 1e6, 1),
            "roofline_frac": round(alg / fus / 1e6 / HBM_PEAK_GBS, 4), "ms": round(fus, 4),
            "encode_only_ms": round(enc, 4), "checksum_overhead": round(fus / enc - 1, 4),
            "timing": "back-to-back blocks of each configuration (a rebuild stream's pattern)",
            "interleaved": {"ms": round(fi, 4), "encode_only_ms": round(enc_i, 4),
                            "checksum_overhead": round(fi / enc_i - 1, 4)},
            "kernel": kernels[htype]}
    # rebuild of parity shard p1 over the same 512 fetched stripes (migrate_update_parity,
    # include/ecg_daos.h): one output row + its crc32 chunks, (k + 1) cells of traffic per stripe
    import ctypes
    pieces = (ecg.MigratePiece * S)()
    npc = ctypes.c_uint32()

    def shard():
        ecg._chk(ecg.lib().ecg_migrate_update_parity(ctx.h, (37 << 24) | 1, C, 1, k + p - 1, data.ptr, 0, S * k * C,
                                                     1, ecg.HASH_CRC32, 32768, par.ptr, out.ptr, pieces, S,
                                                     ctypes.byref(npc), None), "migrate_update_parity")

    ms = time_kernel(ctx, shard, iters, warm=40)
    alg = (k + 1) * C * S
    rows["EC_8P2_1MiB_rebuild_parity_shard_crc32"] = {
        "GiBps_user": round(k * C * S / (ms / 1e3) / GIB, 1), "alg_GBps": round(alg / ms / 1e6, 1),
        "roofline_frac": round(alg / ms / 1e6 / HBM_PEAK_GBS, 4), "ms": round(ms, 4),
        "kernel": ecg.last_kernel()}
    n = 1024
    for hname, htype in (("crc32", ecg.HASH_CRC32), ("crc64", ecg.HASH_CRC64)):
        ms = time_kernel(ctx, lambda: ctx.csum_extents(htype, 32768, 1, 0, C, data.ptr, C, n, out.ptr), iters)
        rows[f"{hname}_32KiB_chunks_1GiB"] = {"alg_GBps": round(C * n / ms / 1e6, 1),
                                              "roofline_frac": round(C * n / ms / 1e6 / HBM_PEAK_GBS, 4),
                                              "ms": round(ms, 4), "kernel": ecg.last_kernel()}
    data.free(); par.free(); out.free()
    return rows


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share():
    """What this process may run on: the affinity mask, the machine's count,
    and the cgroup CPU quota if one is set (cpu.max, in CPUs)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"affinity": aff, "cpu_count": os.cpu_count(), "cgroup_quota_cpus": quota}


class CpuCase:
    """One CPU-baseline workload: the oracle's SIMD ISA-L-equivalent
    restatement (GFNI/AVX-512 + OpenMP over stripes) on >= 1 GiB of user data
    (so the 256 MB L3 of the box's EPYC cannot hold it), the same ops as the
    GPU row it sits beside.  ops: "enc" (data [S][k][C] -> parity [p][S][C])
    and/or "dec" ({d0,d1}, or {d0} at p = 1, in place in [S][k+p][C])."""

    def __init__(self, k, p, C, ops, config_id=2):
        import numpy as np

        from oracle import ref
        from tools.datagen import stripe_bytes

        self.ref, self.k, self.p, self.C, self.ops = ref, k, p, C, tuple(ops)
        self.S = S = max(32, -(-(1 << 30) // (k * C)))
        blk = stripe_bytes(min(256 << 20, S * k * C), config_id)
        self.data = np.resize(blk, S * k * C)
        self.stripes = np.empty(S * (k + p) * C, dtype=np.uint8)
        sv = self.stripes.reshape(S, k + p, C)
        sv[:, :k] = self.data.reshape(S, k, C)
        self.pout = np.empty(p * S * C, dtype=np.uint8)     # reused: no page faults in the timed loop
        ref.encode_batch(k, p, C, S, self.data, nthreads=8, simd=True, out=self.pout)
        sv[:, k:] = self.pout.reshape(p, S, C).transpose(1, 0, 2)
        self.err = [0, 1] if p >= 2 else [0]
        rc, _, self.dec, self.el, self.gt, _ = ref.recov_codec(k, p, self.err)
        assert rc == 0
        self.ws = S * ((k + p) * C * ("dec" in ops) + (k + p) * C * ("enc" in ops))

    def run(self, threads, secs):
        k, p, C, S, ref = self.k, self.p, self.C, self.S, self.ref
        user, n, t0 = 0, 0, time.perf_counter()
        while time.perf_counter() - t0 < secs or n == 0:
            if "enc" in self.ops:
                ref.encode_batch(k, p, C, S, self.data, nthreads=threads, simd=True, out=self.pout)
            if "dec" in self.ops:
                ref.recov_batch(k, len(self.err), self.gt, self.dec, self.el, C, (k + p) * C, S, self.stripes,
                                nthreads=threads, simd=True)
            user += len(self.ops) * k * C * S
            n += 1
        return user / (time.perf_counter() - t0) / GIB

    def row(self, threads, secs, repeats=3):
        """Median and range of `repeats` runs on `threads`, then one core."""
        many = sorted(self.run(threads, secs) for _ in range(repeats))
        one = self.run(1, secs)
        return {"value": round(many[len(many) // 2], 3), "unit": "GiB/s", "cores": threads,
                "runs": [round(x, 3) for x in many], "range": [round(many[0], 3), round(many[-1], 3)],
                "one_core": round(one, 3),
                "sample": f"EC_{self.k}P{self.p} {self.C >> 10} KiB cells, {self.S} stripes "
                          f"({self.S * self.k * self.C / GIB:.2f} GiB of data, {self.ws / GIB:.2f} GiB touched), "
                          f"{' + '.join(self.ops)}{' {d0,d1}' if 'dec' in self.ops else ''}"}


# per-config CPU rows beside the GPU detail rows (BASELINE.md §3 shapes, per GPU)
CPU_CONFIGS = (("EC_2P1_128KiB_encode", 2, 1, 128 << 10, ("enc",), 0),
               ("EC_8P2_1MiB_decode_d0d1", 8, 2, 1 << 20, ("dec",), 3),
               ("EC_16P2_128KiB_encode", 16, 2, 128 << 10, ("enc",), 4))


def cpu_baseline(k, p, C, budget_s, ops=("enc", "dec"), per_config=True):
    """The headline workload's CPU rate on every core of this process's
    affinity mask (3 repeats: median and range; plus one core), the load
    average before and after, and the same for configs 1, 3 and the config-4
    per-GPU shard.  Reported beside the GPU rows, never the target."""
    from oracle import ref

    share = cpu_share()
    # the CPUs this process is granted: its affinity mask, capped by the cgroup
    # quota when one is set (the GPU box's 256-CPU mask carries a 16-CPU quota:
    # 256 threads ran at 5 GiB/s there against 97 on 16, gpurun_out r03 bench)
    threads = share["affinity"]
    if share["cgroup_quota_cpus"]:
        threads = max(1, min(threads, int(share["cgroup_quota_cpus"])))
    load0 = [round(x, 2) for x in os.getloadavg()]
    t_all = time.perf_counter()
    head = CpuCase(k, p, C, ops, config_id=2)
    secs = budget_s / 8.0                      # 3 repeats + 1 core = 4 runs of the headline
    out = head.row(threads, secs)
    if threads < share["affinity"]:            # what the whole mask does under the quota (one short run)
        out["all_affinity_threads"] = {"threads": share["affinity"],
                                       "value": round(head.run(share["affinity"], secs / 2), 3)}
    del head
    out.update({"kind": "port", "cores_available": share, "cpu_model": cpu_model(),
                "variant": {0: "scalar", 1: "avx2-vpshufb", 2: "gfni-avx512"}[ref.simd_variant()],
                "what": "ISA-L-equivalent restatement (oracle/ec_simd.c), OpenMP over stripes"})
    if per_config:
        rows = {}
        for name, kk, pp, CC, oo, cid in CPU_CONFIGS:
            case = CpuCase(kk, pp, CC, oo, config_id=cid)
            rows[name] = case.row(threads, secs / 2)
            del case
        out["configs"] = rows
    out["load"] = {"before": load0, "after": [round(x, 2) for x in os.getloadavg()]}
    out["seconds"] = round(time.perf_counter() - t_all, 1)
    return out


def pmc_traffic():
    path = os.path.join(ROOT, "profiles", ROUND, "pmc_traffic.json")
    for older in ("r05", "r04", "r03", "r02", "r01"):    # the newest committed pass
        if not os.path.exists(path):
            path = os.path.join(ROOT, "profiles", older, "pmc_traffic.json")
    if os.path.exists(path):
        try:
            d = json.load(open(path))
            d["_path"] = os.path.relpath(path, ROOT)
            return d
        except (OSError, ValueError):
            return None
    return None


# ------------------------------------------------------------------ multi-GPU config legs
# BASELINE configs[3] and configs[4] are multi-GPU configurations; the driver's
# scaling run only invokes `bench.py --gpus N`, so every headline run (N = 1
# included, so the driver's N = 1, 2, 4, 8 runs give both legs a curve) runs
# them after the headline, each with its own barrier / max-over-ranks timing:
#   configs[3]: EC_16P2, 128 KiB cells, 8192 stripes in total, split over the
#     N ranks by contiguous stripe ranges (strong scaling; the reference's
#     per-stripe loop ref:src/object/cli_ec.c:627-659 is what the ranges cut),
#     and its weak form, 1024 stripes per rank;
#   configs[4]: the EC_8P2 rebuild stream -- per rank one encode batch and one
#     {d0,d1} recovery batch of 64 stripes, stripes in pinned host memory
#     allocated after the rank pinned itself to its GPU's NUMA node, so the
#     pages are node-local (weak scaling; the rebuild walk of
#     ref:src/object/srv_obj_migrate.c:1116-1177 is per object, so objects
#     partition across GPUs).
LEG_STRONG = "config3_EC_16P2_128KiB_x8192_strong"
LEG_WEAK = "config3_EC_16P2_128KiB_x1024_per_gpu_weak"
LEG_STREAM = "config4_EC_8P2_1MiB_rebuild_stream"
STRONG_TOTAL = 8192
WEAK_PER_GPU = 1024


def split_range(total, world, rank):
    """Contiguous stripe range [first, first + n) of `rank` (ecg_multi_range's cut)."""
    base, extra = divmod(total, world)
    n = base + (1 if rank < extra else 0)
    return rank * base + min(rank, extra), n


def timed_leg(world, steps, warm, step, sync, warm_s=0.0):
    """warm untimed steps (and at least warm_s seconds of them), then `steps`
    timed from a common barrier; returns (this rank's seconds, the max over
    ranks)."""
    t0 = time.perf_counter()
    n = 0
    while n < warm or time.perf_counter() - t0 < warm_s:
        step(False)
        n += 1
    sync()
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(steps):
        step(True)
    sync()
    mine = time.perf_counter() - t0
    barrier(world)
    return mine, max_over_ranks(world, mine)


def leg_strong(args, ctx, world, rank, steps, weak=False):
    """configs[3] on this rank's contiguous share of the 8192 stripes (weak:
    1024 stripes per rank, the per-GPU shard of the 8-GPU split, SURVEY §8(d)
    config 4's weak-scaling form)."""
    k, p, C = 16, 2, 128 << 10
    total = WEAK_PER_GPU * world if weak else STRONG_TOTAL
    first, S = split_range(total, world, rank)
    if args.rehearse:
        wl = None
        step, sync = (lambda timed: time.sleep(1e-4 * S / 1024)), (lambda: None)
    else:
        wl = Workload(ctx, k, p, C, S, ops=("enc",), config_id=4)
        step, sync = wl.step, ctx.sync
    # 40 warm-up launches: the launch tuner's probe of this shape (ecg_tune.c)
    mine, tmax = timed_leg(world, steps, 0 if args.rehearse else 40, step, sync)
    row = {"rank": rank, "first_stripe": first, "stripes": S, "ms_per_step": round(mine / steps * 1e3, 4)}
    if wl is not None:
        kms = wl.kernel_ms()["enc"]
        launch = sum(kms) / len(kms)
        alg = wl.alg_bytes("enc")
        row.update({"launch_ms": round(launch, 4), "alg_GBps": round(alg / launch / 1e6, 1),
                    "roofline_frac": round(alg / launch / 1e6 / HBM_PEAK_GBS, 4), "kernel": _last_kernel()})
        row["verified"] = all(wl.verify().values())      # after reading the timed launches' kernel
        wl.free()
    rows = gather(world, row)
    return {"config": f"EC_{k}P{p} {C >> 10} KiB cells, {total} stripes in total split over {world} "
                      "rank(s) by contiguous ranges, client-layout encode, device-resident",
            "value_GiBps": None if args.rehearse else round(total * k * C * steps / tmax / GIB, 2),
            "unit": "GiB/s", "scaling": "weak" if weak else "strong", "steps": steps,
            "ms_per_step": round(tmax / steps * 1e3, 4),
            "ranks": rows, "verified": all(r.get("verified", True) for r in rows),
            **({"rehearsal": True} if args.rehearse else {})}


def concurrent_copy_rates(world, ctx, host, nbytes, reps=3):
    """Pinned H2D / D2H copies with EVERY rank copying at once (barrier-aligned
    start of each copy), over `host` -- the leg's own pinned buffer -- and one
    device buffer of its size.  Returns this rank's own rate ("h2d"/"d2h") and
    the node aggregate: world x nbytes over the slowest rank's time
    ("node_h2d"/"node_d2h"), whose 1/world share is a rank's fair share of the
    host memory / PCIe the ranks contend for.  Without a context (CPU
    rehearsal) the "copy" is a host memcpy of the buffer."""
    import numpy as np

    dev = ctx.alloc(nbytes) if ctx is not None else None
    scratch = None if ctx is not None else np.empty_like(host)
    out = {}
    try:
        for name in ("h2d", "d2h"):
            ts, tmaxs = [], []
            for _ in range(reps):
                barrier(world)
                t0 = time.perf_counter()
                if ctx is None:
                    np.copyto(scratch, host) if name == "h2d" else np.copyto(host, scratch)
                else:
                    from daos_amd import ecg

                    src, dst = (host.ctypes.data, dev.ptr) if name == "h2d" else (dev.ptr, host.ctypes.data)
                    ecg._chk(ecg.lib().ecg_memcpy(ctx.h, dst, src, nbytes, 0 if name == "h2d" else 1, None),
                             name)
                    ctx.sync()
                t = time.perf_counter() - t0
                ts.append(t)
                tmaxs.append(max_over_ranks(world, t))
            out[name] = round(nbytes / sorted(ts)[len(ts) // 2] / 1e9, 2)
            out["node_" + name] = round(world * nbytes / sorted(tmaxs)[len(tmaxs) // 2] / 1e9, 2)
    finally:
        if dev is not None:
            dev.free()
        barrier(world)
    return out


def solo_copy_rates(world, rank, ctx, nbytes):
    """This rank's pinned copy rates with the other ranks idle (ranks take
    turns): the denominator a rank alone would see."""
    out = None
    for r in range(world):
        barrier(world)
        if r == rank and ctx is not None:
            out = pinned_copy_rates(ctx, n=nbytes)
    barrier(world)
    return out


def leg_stream(args, ctx, world, rank, steps, numa_info):
    """configs[4] per rank from node-local pinned buffers.  Its denominator is
    the rank's fair share of the node's concurrent pinned copy rate (every
    rank copying its leg buffer at once: N x bytes over the slowest rank's
    time, `node_concurrent_copy_ceiling`); each rank's own concurrent rate and
    its solo rate (ranks in turn) are reported beside it."""
    import numpy as np

    k, p, C, S = 8, 2, 1 << 20, 64
    saved = None
    if args.rehearse:
        wl = None
        step, sync = (lambda timed: time.sleep(2e-4)), (lambda: None)
    else:
        if not (numa_info or {}).get("pinned_cpus"):
            # N = 1 (or pinning off): the process was not pinned at start, so run the leg's
            # thread on its GPU's node while it allocates and first-touches the pinned stripes
            # and streams them -- "NUMA-local" must hold at every N, not only N > 1
            from daos_amd import ecg, numa

            node = ecg.lib().ecg_device_numa_node(ecg.lib().ecg_ctx_device(ctx.h))
            cpus = numa.node_cpus(node) & set(os.sched_getaffinity(0)) if node >= 0 else set()
            if cpus and os.environ.get("ECG_NUMA") != "0":
                saved = os.sched_getaffinity(0)
                os.sched_setaffinity(0, cpus)
                numa_info = dict(numa_info or {}, numa_node=node, pinned_cpus=len(cpus), pinned_for="leg")
        wl = HostWorkload(ctx, k, p, C, S, chunk=args.host_chunk)
        step, sync = wl.step, ctx.sync
    # >= 8 warm-up steps and >= 1 s of them: the first batches of a process's host pipeline ran 42
    # instead of 50 GiB/s after 2 warm-up steps (tools/hoststream_probe.py, profiles/r04/hoststream_probe/),
    # and right after the configs[3] legs' HBM-bound launches the first ~0.3 s of host streaming
    # ran 44-45 instead of 50.8 GiB/s whatever the context (tools/leg_probe.py, profiles/r05/leg_probe/)
    mine, tmax = timed_leg(world, steps, 0 if args.rehearse else 8, step, sync,
                           0.0 if args.rehearse else 1.0)
    row = {"rank": rank, "ms_per_step": round(mine / steps * 1e3, 4),
           "numa_node": (numa_info or {}).get("numa_node"), "pinned_cpus": (numa_info or {}).get("pinned_cpus")}
    user = 2 * k * C * S
    h2d_bytes = 2 * k * C * S if wl is None else wl.h2d_bytes_per_step()
    h2d = h2d_bytes * steps / mine / 1e9
    host = wl.data.array if wl is not None else np.ones(64 << 20, dtype=np.uint8)
    conc = concurrent_copy_rates(world, ctx if wl is not None else None, host, host.size)
    solo = solo_copy_rates(world, rank, ctx if wl is not None else None, 256 << 20)
    share = conc["node_h2d"] / world
    row.update({"h2d_GBps": round(h2d, 2),
                "concurrent_pinned_GBps": {"h2d": conc["h2d"], "d2h": conc["d2h"]},
                "fair_share_h2d_GBps": round(share, 2), "frac_of_fair_share_h2d": round(h2d / share, 4),
                "frac_of_own_concurrent_h2d": round(h2d / conc["h2d"], 4),
                "frac_of_h2d": None,
                "denominator": "frac_of_h2d: the rank's solo pinned H2D rate (ranks copying in turn; the "
                               "round-4 meaning); frac_of_fair_share_h2d: 1/N of the node's concurrent pinned "
                               "H2D rate (all ranks copying at once)"})
    if solo is not None:
        row.update({"measured_pinned_GBps": solo, "frac_of_h2d": round(h2d / solo["h2d"], 4)})
    if wl is not None:
        row.update({"d2h_GBps": round(wl.d2h_bytes_per_step() * steps / mine / 1e9, 2),
                    "verified": all(wl.verify().values())})
        wl.free()
    if saved is not None:
        os.sched_setaffinity(0, saved)
    rows = gather(world, row)
    node = {"h2d_GBps": conc["node_h2d"], "d2h_GBps": conc["node_d2h"],
            "what": "N x the pinned copy bytes of one rank over the slowest rank's time, every rank copying at "
                    "once: the node's host-memory / PCIe ceiling at this N"}
    return {"config": f"EC_{k}P{p} {C >> 20} MiB cells: per rank one encode batch + one {{d0,d1}} recovery "
                      f"batch of {S} stripes per step, stripes in NUMA-local pinned host memory, "
                      f"host<->device copies included ({args.host_chunk or HOST_CHUNK}-stripe staging chunks)",
            "value_GiBps": None if args.rehearse else round(world * user * steps / tmax / GIB, 2),
            "unit": "GiB/s", "scaling": "weak", "bound": "pcie", "steps": steps,
            "ms_per_step": round(tmax / steps * 1e3, 4), "ranks": rows,
            "node_concurrent_copy_ceiling": node,
            "frac_of_node_ceiling": None if args.rehearse else
            round(world * h2d_bytes * steps / tmax / 1e9 / node["h2d_GBps"], 4),
            "verified": all(r.get("verified", True) for r in rows),
            **({"rehearsal": True} if args.rehearse else {})}


def config_legs(args, ctx, world, rank, numa_info):
    steps = max(5, args.steps)
    return {LEG_STRONG: leg_strong(args, ctx, world, rank, steps),
            LEG_WEAK: leg_strong(args, ctx, world, rank, steps, weak=True),
            LEG_STREAM: leg_stream(args, ctx, world, rank, min(steps, 10), numa_info)}


def _last_kernel():
    from daos_amd import ecg

    return ecg.last_kernel()



# ------------------------------------------------------------------ reporting
def host_report(args, ctx, wl, world, rank, value, elapsed, ranks, nshard=1):
    """JSON line of the PCIe-inclusive rebuild stream (configs[4]).  The
    device kernels are not the bound here, the host links are: `roofline`
    is null and `pcie` sets the achieved H2D rate against this box's raw
    pinned copy rate (measured on rank 0 at N=1)."""
    k, p, C, S = wl.k, wl.p, wl.C, wl.S
    ver = wl.verify()
    allver = gather(world, ver)
    ok = all(all(v.values()) for v in allver)
    h2d = wl.h2d_bytes_per_step() * args.steps * world / elapsed / 1e9
    d2h = wl.d2h_bytes_per_step() * args.steps * world / elapsed / 1e9
    out = {
        "metric": "EC rebuild stream GiB/s (host-resident stripes, PCIe-inclusive)",
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": len({r["pci"] for r in ranks}),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: xoshiro256** stripes in pinned host memory",
        "config": {"workload": f"EC_{k}P{p} {C >> 10} KiB cells: per step one encode batch of {S // nshard} stripes "
                               f"+ one {{d0,d1}} recovery batch of {S // nshard} stripes per GPU, host<->device "
                               f"copies included ({wl.chunk}-stripe staging chunks)",
                   "name": args.workload, "k": k, "p": p, "cell_bytes": C, "stripes_per_gpu": S // nshard,
                   "erasures": wl.err,
                   "parallelism": (f"one {S}-stripe host batch split x{nshard} in one process (ecg_multi_*_host), "
                                   "no collective" if nshard > 1 or args.sharder == "lib"
                                   else f"stripe-sharded x{world}, no collective")},
        "roofline": None,
        "pcie": {"bound": "pcie", "h2d_GBps_all_ranks": round(h2d, 2), "d2h_GBps_all_ranks": round(d2h, 2)},
        "verified": ver,
        "ranks": ranks,
        "cpu_baseline": None,
    }
    wl.free()
    if rank == 0 and world == 1 and nshard == 1 and not args.no_detail:
        raw = pinned_copy_rates(ctx)
        out["pcie"]["measured_pinned_GBps"] = raw
        out["pcie"]["frac_of_h2d"] = round(h2d / raw["h2d"], 4)
    if rank == 0:
        print(json.dumps(out), flush=True)
    return ok


def rehearse(args, world, rank, local):
    """CPU-only rehearsal of the N-rank plumbing (launcher, env, barrier,
    max-over-ranks, gather): each rank 'steps' by sleeping 1 ms per step,
    then the configs[3] / configs[4] legs run their split, timing and
    aggregation with sleeps for the GPU work."""
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.001 * (1 + rank))
    elapsed = max_over_ranks(world, time.perf_counter() - t0)
    ranks = gather(world, {"rank": rank, "local_rank": local, "pid": os.getpid()})
    legs = config_legs(args, None, world, rank, None) if args.workload == "enc_dec_4p2" else {}
    if rank == 0:
        print(json.dumps({"metric": "rehearsal (no GPU work)", "rehearsal": True, "value": None, "n_ranks": world,
                          "steps": args.steps, "ms_per_step": round(elapsed / max(1, args.steps) * 1e3, 3),
                          "ranks": ranks, "detail": legs}), flush=True)
    finish_dist(world)


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1 and args.sharder == "procs":
        sys.exit(launch_ranks(args))          # parent: no GPU calls before or after
    numa_info = rank_numa(args)               # before anything starts the GPU runtime
    world, rank, local = dist_init()
    if "WORLD_SIZE" in os.environ and args.sharder == "procs" and world != args.gpus:
        raise SystemExit(f"bench.py: launched as {world} ranks but --gpus {args.gpus}")
    if args.sharder == "lib" and world > 1:
        raise SystemExit("bench.py: --sharder lib runs in one process (no WORLD_SIZE > 1)")
    if args.rehearse:
        rehearse(args, world, rank, local)
        return

    import torch  # noqa: F401  (shares libamdhip64 with libecg; sync per contract)

    from daos_amd import ecg

    ndev = ecg.device_count()
    if ndev < 1:
        raise SystemExit("bench.py: no gfx950 device visible")
    k, p, C, S, ops, strong = WORKLOADS[args.workload]
    host = ops[0].endswith("_host")
    nshard = args.gpus if args.sharder == "lib" else world
    if args.sharder == "lib":
        devices = list(range(args.gpus)) if args.gpus <= ndev else [i % ndev for i in range(args.gpus)]
        if args.gpus > ndev and not args.allow_shared_device:
            raise SystemExit(f"bench.py: {args.gpus} shards but {ndev} devices (--allow-shared-device to rehearse)")
        m = ecg.Multi(devices)
        ctx = m.ctxs[0]
        dev = devices[0]
        torch.cuda.set_device(dev)
        wl = (HostMultiWorkload(m, k, p, C, S, ops, chunk=args.host_chunk) if host
              else MultiWorkload(m, k, p, C, S, ops, strong))
        rank_devs = [{"shard": i, "device": d, "pci": ecg.pci_bus_id(d)} for i, d in enumerate(devices)]
        S = wl.S
    else:
        # LOCAL_RANK picks the device among those visible; a launcher that
        # gives each rank its own HIP_VISIBLE_DEVICES leaves one (index 0).
        # Sharing is judged on physical devices: the ranks' PCI bus ids,
        # checked collectively so every rank stops together.
        dev = local % ndev
        pcis = gather(world, ecg.pci_bus_id(dev))
        if len(set(pcis)) < world and not args.allow_shared_device:
            raise SystemExit(f"bench.py: {world} ranks on {len(set(pcis))} distinct devices {sorted(set(pcis))} "
                             "(--allow-shared-device to rehearse several ranks on one GPU)")
        torch.cuda.set_device(dev)
        ctx = ecg.Context(dev)
        ctx.set_wg_per_cu(args.wg_per_cu)
        m = None
        if strong:                      # configs[3]: a fixed stripe total split across ranks
            S = S // world + (1 if rank < S % world else 0)
        wl = (HostWorkload(ctx, k, p, C, S, ops=ops, chunk=args.host_chunk) if host
              else Workload(ctx, k, p, C, S, ops=ops))
        rank_devs = None

    for _ in range(args.warmup):
        wl.step()
    if m is not None:
        wl.sync()
    ctx.sync()

    barrier(world)
    torch.cuda.synchronize()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        wl.step(timed=True)
    if m is not None:
        wl.sync()
    ctx.sync()
    torch.cuda.synchronize()
    mine = time.perf_counter() - t0       # this rank's K steps, from the common start barrier
    barrier(world)
    elapsed = max_over_ranks(world, mine)  # the job took as long as its slowest rank

    if args.profile_only:
        wl.free()
        if m is not None:
            m.close()
        else:
            ctx.close()
        finish_dist(world)
        return

    if rank_devs is None:
        numa_rep = {"numa_node": numa_info["numa_node"], "pinned_cpus": numa_info["pinned_cpus"]} \
            if numa_info and "pinned_cpus" in numa_info else \
            {"numa_node": ecg.lib().ecg_device_numa_node(dev), "pinned_cpus": 0}
        rank_devs = gather(world, {"rank": rank, "device": dev, "pci": ecg.pci_bus_id(dev),
                                   "ms_per_step": round(mine / args.steps * 1e3, 3), **numa_rep})
    elif m is not None:
        for i, r in enumerate(rank_devs):
            r["numa_node"] = m.numa_node(i)
    n_gpus = len({r["pci"] for r in rank_devs})
    if strong:      # the fixed total, however it was split
        user = WORKLOADS[args.workload][3] * k * C * len(ops) * args.steps
    else:           # every rank processed the same batch
        user = wl.user_bytes_per_step() * args.steps * world
    value = user / elapsed / GIB
    if host:
        ok = host_report(args, ctx, wl, world, rank, value, elapsed, rank_devs, nshard)
        if m is not None:
            m.close()
        else:
            ctx.close()
        finish_dist(world)
        if not ok:
            raise SystemExit("bench.py: verification failed (see `verified`)")
        return
    kms = wl.kernel_ms()
    launches = [(op, ms) for op in ops for ms in kms[op]]
    mean_launch_ms = sum(ms for _, ms in launches) / len(launches)
    alg_per_launch = sum(wl.alg_bytes(op) for op, _ in launches) / len(launches)
    achieved = alg_per_launch / (mean_launch_ms / 1e3) / 1e9
    read_GBps = k * C * S / (mean_launch_ms / 1e3) / 1e9
    kernel_name = f"ecg_mm_kernel<{k},{p},0,0>"
    traffic, traffic_src = None, None
    pmc = pmc_traffic()
    if pmc and pmc.get("kernel", "").replace(" ", "") == f"ecg_mm_kernel<{k},{p}" and \
            pmc.get("alg_bytes_per_launch") == int(alg_per_launch):
        traffic = pmc.get("hbm_bytes_per_launch")
        traffic_src = (f"{pmc['_path']} (rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE passes of this "
                       "workload, FETCH x2 per the gfx950 correction; copied, not measured in this run)")
    ver = wl.verify()
    allver = gather(world, ver)
    ok = all(all(v.values()) for v in allver)

    par = (f"stripe-sharded x{nshard} in one process (ecg_multi), no collective" if m is not None
           else f"stripe-sharded x{world} (one process per GPU), no collective")
    out = {
        "metric": "EC encode+decode GiB/s (device-resident stripes)",
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: xoshiro256** stripes seeded 0xDA05EC00+id (BASELINE.md §3), device-resident",
        "config": {"workload": describe(args.workload, k, p, C, S, ops, nshard),
                   "name": args.workload, "k": k, "p": p, "cell_bytes": C, "stripes_per_gpu": S,
                   "erasures": wl.err if "dec" in ops else [],
                   "parallelism": par},
        "roofline": {"bound": "hbm", "kernel": kernel_name, "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     # north star's "fraction of HBM-read peak": the k input cells read per launch
                     "read_GBps": round(read_GBps, 1), "read_frac": round(read_GBps / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "alg_bytes_per_launch": int(alg_per_launch),
                     "mean_launch_ms": round(mean_launch_ms, 4),
                     **{f"{op}_ms_median": round(sorted(kms[op])[len(kms[op]) // 2], 4) for op in ops}},
        "verified": ver,
        "ranks": rank_devs,
        "cpu_baseline": None,
    }
    wl.free()
    legs = {}
    if args.workload == "enc_dec_4p2" and m is None and not args.no_detail:
        legs = config_legs(args, ctx, world, rank, numa_info)
        out["detail"] = dict(legs)
        ok = ok and all(v["verified"] for v in legs.values())
    if rank == 0 and world == 1 and not args.no_detail:
        ceil = measured_ceilings(ctx)
        mix = mix_ceiling(ceil, k / (k + p))      # enc (k in, p out) and dec (k in, 2 out) alike at p = 2
        out["roofline"]["measured_stream_GBps"] = ceil
        out["roofline"]["measured_mix_ceiling_GBps"] = round(mix, 1)
        out["roofline"]["frac_of_measured_mix"] = round(achieved / mix, 4)
        det = detail_rows(ctx, ceil)
        out["detail"] = {**det, **legs}
        e8 = det["EC_8P2_1MiB_encode"]
        out["roofline"]["north_star"] = {
            "target": ">= 70 % of per-GPU HBM-read roofline on EC_8P2 encode at 1 MiB cells, device-resident",
            "EC_8P2_1MiB_encode_frac": e8["roofline_frac"],
            "EC_8P2_1MiB_encode_read_frac": e8["read_frac"],
            "reading": "frac = (k+p)*C*S bytes (reads + writes) / t / 8 TB/s, the SURVEY §8(d) roofline; "
                       "read_frac = the k input cells alone / t / 8 TB/s.  The same launch must also write "
                       "p/k as many bytes, and this box's HBM streams 6.7-7.0 TB/s read-only, so read_frac "
                       "cannot reach 0.70 while parity is written (DESIGN.md §6)"}
    if rank == 0 and world == 1 and not args.no_cpu and m is None:
        out["cpu_baseline"] = cpu_baseline(k, p, C, args.cpu_seconds, ops)
        if "detail" in out:                   # CPU beside GPU, per config
            for name, row in out["cpu_baseline"].get("configs", {}).items():
                if name in out["detail"]:
                    out["detail"][name]["cpu_GiBps"] = row["value"]
                    out["detail"][name]["gpu_over_cpu"] = round(out["detail"][name]["GiBps_user"] / row["value"], 1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if m is not None:
        m.close()
    else:
        ctx.close()
    finish_dist(world)
    if not ok:
        raise SystemExit("bench.py: verification failed (see `verified`)")


if __name__ == "__main__":
    main()
