"""Host NUMA placement without touching the GPU (sysfs only).

bench.py pins each rank process to the CPUs of its GPU's NUMA node BEFORE
anything initialises HIP, so the runtime's threads and the rank's pinned
staging inherit the placement (DAOS pins its engine xstreams per NUMA node,
ref:src/engine/ult.c:394-470).  The library does the same for its own
ecg_multi worker threads and queue staging (daos_amd/csrc/host/ecg_numa.c).

Device index -> PCI address follows the KFD topology: HIP enumerates the GPU
nodes of /sys/class/kfd/kfd/topology/nodes in node order, filtered by
ROCR_VISIBLE_DEVICES then HIP_VISIBLE_DEVICES.  `root` prefixes every path
(tests use a fake tree).
"""
from __future__ import annotations

import os


def _props(path: str) -> dict:
    out = {}
    try:
        with open(path) as f:
            for line in f:
                parts = line.split()
                if len(parts) == 2:
                    try:
                        out[parts[0]] = int(parts[1])
                    except ValueError:
                        pass
    except OSError:
        pass
    return out


def kfd_gpus(root: str = "") -> list:
    """PCI addresses ("dddd:bb:ss.f") of the KFD GPU nodes, in node order."""
    base = f"{root}/sys/class/kfd/kfd/topology/nodes"
    try:
        nodes = sorted(int(n) for n in os.listdir(base) if n.isdigit())
    except OSError:
        return []
    out = []
    for n in nodes:
        p = _props(f"{base}/{n}/properties")
        if p.get("simd_count", 0) == 0 or "location_id" not in p:
            continue                                    # a CPU node
        loc, dom = p["location_id"], p.get("domain", 0)
        out.append(f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7}")
    return out


def _filter(seq: list, spec: str | None) -> list:
    if not spec:
        return seq
    idx = []
    for tok in spec.split(","):
        tok = tok.strip()
        if tok.isdigit() and int(tok) < len(seq):
            idx.append(int(tok))
    return [seq[i] for i in idx]


def visible_gpus(root: str = "", env=None) -> list:
    env = os.environ if env is None else env
    g = _filter(kfd_gpus(root), env.get("ROCR_VISIBLE_DEVICES"))
    return _filter(g, env.get("HIP_VISIBLE_DEVICES") or env.get("CUDA_VISIBLE_DEVICES"))


def pci_numa_node(bdf: str, root: str = "") -> int:
    try:
        with open(f"{root}/sys/bus/pci/devices/{bdf.lower()}/numa_node") as f:
            n = int(f.read().strip())
        return n if n >= 0 else -1
    except (OSError, ValueError):
        return -1


def node_cpus(node: int, root: str = "") -> set:
    try:
        with open(f"{root}/sys/devices/system/node/node{node}/cpulist") as f:
            spec = f.read().strip()
    except OSError:
        return set()
    cpus = set()
    for part in filter(None, spec.split(",")):
        a, _, b = part.partition("-")
        cpus.update(range(int(a), int(b or a) + 1))
    return cpus


def placement(device: int, root: str = "", env=None) -> dict:
    """{"device", "pci", "numa_node", "node_cpus"} for a visible device index."""
    g = visible_gpus(root, env)
    if not g:
        return {"device": device, "pci": None, "numa_node": -1, "node_cpus": 0}
    bdf = g[device % len(g)]
    node = pci_numa_node(bdf, root)
    return {"device": device, "pci": bdf, "numa_node": node, "node_cpus": len(node_cpus(node, root)) if node >= 0 else 0}


def pin_to_device(device: int, root: str = "", env=None) -> dict:
    """Restrict this process (the calling thread and every thread it starts
    afterwards) to the CPUs of the device's NUMA node that it may use.  Call
    before the GPU runtime starts.  Returns placement() plus "pinned_cpus"
    (0 when nothing was changed)."""
    info = placement(device, root, env)
    info["pinned_cpus"] = 0
    env = os.environ if env is None else env
    if info["numa_node"] < 0 or env.get("ECG_NUMA") == "0":
        return info
    want = node_cpus(info["numa_node"], root) & set(os.sched_getaffinity(0))
    if want:
        os.sched_setaffinity(0, want)
        info["pinned_cpus"] = len(want)
    return info
