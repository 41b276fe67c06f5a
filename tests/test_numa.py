"""NUMA placement from sysfs (daos_amd/numa.py for bench ranks, before HIP
starts; ecg_pci_numa_node in libecg for the ecg_multi workers and queue
staging), over a fake sysfs tree of a 2-socket node with 4 GPUs: two behind
each socket, HIP order = KFD node order, visibility lists applied."""
import os

import pytest

from daos_amd import numa

GPUS = [  # KFD node, domain, bus, slot, fn, numa node
    (1, 0, 0x05, 0, 0, 0),
    (2, 0, 0x15, 0, 0, 0),
    (3, 0, 0x85, 0, 0, 1),
    (4, 1, 0x95, 0, 0, 1),
]


@pytest.fixture
def sysfs(tmp_path):
    root = str(tmp_path)
    kfd = os.path.join(root, "sys/class/kfd/kfd/topology/nodes")
    os.makedirs(os.path.join(kfd, "0"))
    with open(os.path.join(kfd, "0/properties"), "w") as f:      # the CPU node
        f.write("cpu_cores_count 64\nsimd_count 0\nlocation_id 0\n")
    for n, dom, bus, slot, fn, node in GPUS:
        os.makedirs(os.path.join(kfd, str(n)))
        with open(os.path.join(kfd, f"{n}/properties"), "w") as f:
            f.write(f"cpu_cores_count 0\nsimd_count 1024\nlocation_id {(bus << 8) | (slot << 3) | fn}\n"
                    f"domain {dom}\n")
        bdf = f"{dom:04x}:{bus:02x}:{slot:02x}.{fn}"
        os.makedirs(os.path.join(root, "sys/bus/pci/devices", bdf))
        with open(os.path.join(root, "sys/bus/pci/devices", bdf, "numa_node"), "w") as f:
            f.write(f"{node}\n")
    for node, cpus in ((0, "0-3,8-9"), (1, "4-7,10")):
        os.makedirs(os.path.join(root, f"sys/devices/system/node/node{node}"))
        with open(os.path.join(root, f"sys/devices/system/node/node{node}/cpulist"), "w") as f:
            f.write(cpus + "\n")
    return root


def test_kfd_order_and_nodes(sysfs):
    g = numa.kfd_gpus(sysfs)
    assert g == ["0000:05:00.0", "0000:15:00.0", "0000:85:00.0", "0001:95:00.0"]
    assert [numa.pci_numa_node(b, sysfs) for b in g] == [0, 0, 1, 1]
    assert numa.node_cpus(0, sysfs) == {0, 1, 2, 3, 8, 9}
    assert numa.node_cpus(1, sysfs) == {4, 5, 6, 7, 10}
    assert numa.pci_numa_node("0000:ff:00.0", sysfs) == -1


def test_visibility_lists(sysfs):
    assert numa.visible_gpus(sysfs, {"HIP_VISIBLE_DEVICES": "3,1"}) == ["0001:95:00.0", "0000:15:00.0"]
    assert numa.visible_gpus(sysfs, {"ROCR_VISIBLE_DEVICES": "2,3", "HIP_VISIBLE_DEVICES": "1"}) == ["0001:95:00.0"]
    p = numa.placement(0, sysfs, {"HIP_VISIBLE_DEVICES": "2"})
    assert p["pci"] == "0000:85:00.0" and p["numa_node"] == 1 and p["node_cpus"] == 5


def test_pin_restricts_to_node_cpus(sysfs):
    before = os.sched_getaffinity(0)
    try:
        info = numa.pin_to_device(2, sysfs, {})
        allowed = numa.node_cpus(1, sysfs) & before
        assert info["numa_node"] == 1
        if allowed:
            assert os.sched_getaffinity(0) == allowed and info["pinned_cpus"] == len(allowed)
        off = numa.pin_to_device(0, sysfs, {"ECG_NUMA": "0"})
        assert off["pinned_cpus"] == 0
    finally:
        os.sched_setaffinity(0, before)


def test_library_reads_the_same_node(sysfs, ecglib, monkeypatch):
    """libecg's ecg_pci_numa_node (the ecg_multi workers' placement) reads
    the same files: $ECG_SYSFS_ROOT points it at the fake tree."""
    monkeypatch.setenv("ECG_SYSFS_ROOT", sysfs)
    L = ecglib.lib()
    assert [L.ecg_pci_numa_node(b.upper().encode()) for b in numa.kfd_gpus(sysfs)] == [0, 0, 1, 1]
    assert L.ecg_pci_numa_node(b"0000:ff:00.0") == -1
