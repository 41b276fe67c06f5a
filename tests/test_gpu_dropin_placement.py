"""The ISA-L drop-in routes by the placement of EVERY pointer (VERDICT r05 weak
item 3: routing by src[0] alone sent a host-src / device-dst call to the CPU
path, which then stored through a device address -- SIGSEGV).

tests/dropin_placement.py runs in a subprocess (a crash there is a test
failure, not a dead pytest): ec_encode_data, ec_encode_data_update and
xor_gen over every pairing of plain host, pinned host, device and
hipMallocManaged cells, sources split over two placements too; every case
must return the oracle's bytes.  A device cell past its allocation must
abort with a message naming the output -- before any memory is touched.
Reference contract: ISA-L's void ec_encode_data (ref:src/object/cli_ec.c:540)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
HELPER = os.path.join(ROOT, "tests", "dropin_placement.py")


def test_dropin_mixed_placements_match_oracle():
    r = subprocess.run([sys.executable, "-u", HELPER], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.returncode, r.stdout[-3000:], r.stderr[-3000:])
    rows = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(rows) >= 80, len(rows)
    bad = [x for x in rows if not x["equal"]]
    assert not bad, bad
    for x in rows:
        cells = {x["src"], x["dst"]} | ({x["src2"]} if x["src2"] else set())
        if "device" in cells:          # any device cell: the GPU, never the CPU path
            assert not x["kernel"].startswith("cpu:"), x
        if cells == {"host"}:          # plain host memory only: the CPU path (default crossover)
            assert x["kernel"].startswith("cpu:"), x


def test_dropin_device_cell_past_end_aborts_with_message():
    r = subprocess.run([sys.executable, "-u", HELPER, "past_end"], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and r.returncode != -11, (r.returncode, r.stderr[-2000:])
    assert "returned" not in r.stdout
    assert "output 1" in r.stderr and "past the end" in r.stderr, r.stderr[-2000:]
