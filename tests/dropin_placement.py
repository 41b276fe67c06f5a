"""Subprocess helper of tests/test_gpu_dropin_placement.py: the ISA-L drop-in
(ec_encode_data, ec_encode_data_update, xor_gen) on cells of mixed placement
-- plain host, pinned host (ecg_host_alloc), device (ecg_dev_alloc) and
hipMallocManaged memory -- checked against the oracle.  Prints one JSON line
per case.  `python tests/dropin_placement.py past_end` instead makes one call
with a device cell running past its allocation: the library must abort with
a message naming the cell (run in a subprocess by the test)."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)

from daos_amd import ecg  # noqa: E402
from oracle import ref  # noqa: E402

hip = C.CDLL("libamdhip64.so")
hip.hipMallocManaged.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
hip.hipFree.argtypes = [C.c_void_p]


class Cells:
    """n cells of `length` bytes in one placement; .ptrs, .read(), .write()."""

    def __init__(self, ctx, kind, n, length, rng):
        self.kind, self.n, self.len = kind, n, length
        self.pitch = (length + 64 + 15) & ~15
        total = self.pitch * n + 64
        self.host = self.dev = self.man = None
        if kind == "host":
            self.host = np.zeros(total, dtype=np.uint8)
            base = self.host.ctypes.data
        elif kind == "pinned":
            self.pin = ctx.host_alloc(total)
            base = self.pin.ptr
        elif kind == "device":
            self.dev = ctx.alloc(total)
            base = self.dev.ptr
        elif kind == "managed":
            p = C.c_void_p()
            assert hip.hipMallocManaged(C.byref(p), total, 1) == 0, "hipMallocManaged"
            self.man = p.value
            base = p.value
        else:
            raise ValueError(kind)
        self.base = base
        self.ctx = ctx
        self.ptrs = [base + i * self.pitch + (i % 3) for i in range(n)]     # odd offsets too
        self.vals = rng.integers(0, 256, (n, length), dtype=np.uint8)
        for i in range(n):
            self.write(i, self.vals[i])

    def write(self, i, a):
        if self.kind == "device":
            ecg.lib().ecg_memcpy(self.ctx.h, self.ptrs[i], a.ctypes.data, a.nbytes, 0, None)
            self.ctx.sync()
        else:
            C.memmove(self.ptrs[i], a.ctypes.data, a.nbytes)

    def read(self, i):
        out = np.empty(self.len, dtype=np.uint8)
        if self.kind == "device":
            ecg.lib().ecg_memcpy(self.ctx.h, out.ctypes.data, self.ptrs[i], self.len, 1, None)
            self.ctx.sync()
        else:
            C.memmove(out.ctypes.data, self.ptrs[i], self.len)
        return out

    def free(self):
        if self.dev:
            self.dev.free()
        if self.kind == "pinned":
            self.pin.free()
        if self.man:
            hip.hipFree(self.man)


def u8pp(ptrs):
    return (ecg.u8p * len(ptrs))(*[C.cast(C.c_void_p(a), ecg.u8p) for a in ptrs])


def main():
    ctx = ecg.Context(0)
    rng = np.random.default_rng(0xD0)
    L = ecg.lib()
    k, p = 4, 2
    en = ref.cauchy1(k, p)
    tb = ecg.isal_init_tables(np.ascontiguousarray(en[k:]))
    kinds = ["host", "pinned", "device", "managed"]
    cases = []
    for length in (4096 + 7, 1 << 20):
        for sk in kinds:
            for dk in kinds:
                cases.append(("encode", length, sk, dk, None))
        # sources split over two placements (cell j on kinds[j % 2] of the pair)
        for a, b in (("host", "device"), ("device", "pinned"), ("managed", "device")):
            for dk in ("host", "device"):
                cases.append(("encode", length, a, dk, b))
        for sk in kinds:
            for dk in kinds:
                cases.append(("update", length, sk, dk, None))
        for a, b in (("host", "device"), ("pinned", "managed"), ("device", "device"), ("host", "host")):
            cases.append(("xor", length, a, b, None))
    for op, length, sk, dk, sk2 in cases:
        res = {"op": op, "len": length, "src": sk, "dst": dk, "src2": sk2}
        srcs = [Cells(ctx, sk, k, length, rng)]
        if sk2:
            srcs.append(Cells(ctx, sk2, k, length, rng))
        dst = Cells(ctx, dk, p if op != "xor" else 1, length, rng)
        try:
            if op == "encode":
                sp = [srcs[j % len(srcs)].ptrs[j] for j in range(k)]
                sv = np.stack([srcs[j % len(srcs)].vals[j] for j in range(k)])
                L.ec_encode_data(length, k, p, ecg._u8(tb), u8pp(sp), u8pp(dst.ptrs))
                want = ref.encode_data(en[k:], sv)
                got = np.stack([dst.read(r) for r in range(p)])
            elif op == "update":
                vec_i = 2
                L.ec_encode_data_update(length, k, p, vec_i, ecg._u8(tb), C.cast(C.c_void_p(srcs[0].ptrs[0]), ecg.u8p),
                                        u8pp(dst.ptrs))
                want = ref.encode_data_update(en[k:], vec_i, srcs[0].vals[0], dst.vals)
                got = np.stack([dst.read(r) for r in range(p)])
            else:
                arr = (C.c_void_p * 5)(*(srcs[0].ptrs[:4] + [dst.ptrs[0]]))
                assert L.xor_gen(5, length, arr) == 0
                want = np.bitwise_xor.reduce(srcs[0].vals[:4], axis=0)[None]
                got = dst.read(0)[None]
            res["kernel"] = ecg.last_kernel()
            res["equal"] = bool(np.array_equal(got, want))
        finally:
            for c in srcs + [dst]:
                c.free()
        print(json.dumps(res), flush=True)
    ctx.close()


def past_end():
    """A device output cell whose last 100 bytes lie past its allocation,
    with host sources: must abort naming the output, never touch memory."""
    ctx = ecg.Context(0)
    k, p, length = 4, 2, 4096
    en = ref.cauchy1(k, p)
    tb = ecg.isal_init_tables(np.ascontiguousarray(en[k:]))
    src = [np.zeros(length, dtype=np.uint8) for _ in range(k)]
    d = ctx.alloc(2 * length)
    dp = [d.ptr, d.ptr + length + 100]
    print("calling", flush=True)
    ecg.lib().ec_encode_data(length, k, p, ecg._u8(tb), u8pp([s.ctypes.data for s in src]), u8pp(dp))
    print("returned", flush=True)


if __name__ == "__main__":
    past_end() if sys.argv[1:] == ["past_end"] else main()
