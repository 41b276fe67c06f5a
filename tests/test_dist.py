"""Multi-rank control path of bench.py on CPU (gloo, world_size 2).

The data path has no collective (stripes are independent); the
only cross-rank operations are the barrier and the max of the elapsed time.
"""
import os
import socket
import subprocess
import sys
import textwrap

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_gloo_barrier_and_max_two_ranks(tmp_path):
    script = tmp_path / "w.py"
    script.write_text(textwrap.dedent(f"""
        import os, sys, time
        sys.path.insert(0, {ROOT!r})
        import bench
        world, rank, local = bench.dist_init()
        assert world == 2 and local == rank
        bench.barrier(world)
        t = 0.25 if rank == 1 else 0.1
        m = bench.max_over_ranks(world, t)
        assert abs(m - 0.25) < 1e-12, m
        bench.barrier(world)
        print("rank", rank, "ok", m)
    """))
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = [p.communicate(timeout=300)[0] for p in procs]
    for r, (p, o) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, o
        assert f"rank {r} ok" in o


def test_weak_scaling_accounting():
    """value counts every rank's stripes: N x per-GPU user bytes / max time."""
    sys.path.insert(0, ROOT)
    import bench

    class FakeCtx:
        pass

    wl = bench.Workload.__new__(bench.Workload)
    wl.k, wl.p, wl.C, wl.S, wl.err, wl.ops = 4, 2, 1 << 20, 1024, [0, 1], ("enc", "dec")
    assert wl.user_bytes_per_step() == 2 * 4 * (1 << 20) * 1024
    assert wl.alg_bytes("enc") == wl.alg_bytes("dec") == 6 * (1 << 20) * 1024
    wl.k, wl.p, wl.ops = 16, 2, ("enc",)
    assert wl.user_bytes_per_step() == 16 * (1 << 20) * 1024
    assert set(bench.WORKLOADS) == {"enc_dec_4p2", "dec_8p2", "enc_8p2", "enc_16p2_strong", "rebuild_stream_8p2"}
    assert bench.WORKLOADS["enc_dec_4p2"][:4] == (4, 2, 1 << 20, 1024)      # BASELINE configs[1]


def test_host_stream_accounting():
    """configs[4] (rebuild stream): user bytes = k cells per stripe per batch,
    H2D = the k inputs (encode) / k survivors (recovery), D2H = p parity cells
    + the erased cells."""
    sys.path.insert(0, ROOT)
    import bench

    wl = bench.HostWorkload.__new__(bench.HostWorkload)
    wl.k, wl.p, wl.C, wl.S, wl.err, wl.ops = 8, 2, 1 << 20, 64, [0, 1], ("enc_host", "dec_host")
    assert wl.user_bytes_per_step() == 2 * 8 * (1 << 20) * 64
    assert wl.h2d_bytes_per_step() == 2 * 8 * (1 << 20) * 64
    assert wl.d2h_bytes_per_step() == (2 + 2) * (1 << 20) * 64
    assert bench.WORKLOADS["rebuild_stream_8p2"][:2] == (8, 2)


def _bench_env():
    env = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    return env


def test_bench_gpus_n_spawns_ranks():
    """`bench.py --gpus 2` with no launcher in the environment starts two
    rank processes itself (gloo rendezvous on 127.0.0.1) and rank 0 prints
    ONE aggregated line: max-over-ranks time (rank 1 sleeps twice as long)
    and both ranks listed.  --rehearse replaces the GPU work with sleeps."""
    import json

    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "20",
                        "--rehearse"], env=_bench_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["rehearsal"] is True and d["value"] is None
    assert d["n_ranks"] == 2
    assert sorted(x["rank"] for x in d["ranks"]) == [0, 1]
    assert len({x["pid"] for x in d["ranks"]}) == 2
    assert d["ms_per_step"] >= 2.0          # the slower rank (2 ms steps) sets the time
    # the configs[3] / configs[4] legs ran on both ranks (split, timing, aggregation)
    strong = d["detail"]["config3_EC_16P2_128KiB_x8192_strong"]
    assert strong["scaling"] == "strong" and len(strong["ranks"]) == 2
    assert sorted((r["first_stripe"], r["stripes"]) for r in strong["ranks"]) == [(0, 4096), (4096, 4096)]
    weak = d["detail"]["config3_EC_16P2_128KiB_x1024_per_gpu_weak"]
    assert weak["scaling"] == "weak" and sorted(r["stripes"] for r in weak["ranks"]) == [1024, 1024]
    stream = d["detail"]["config4_EC_8P2_1MiB_rebuild_stream"]
    assert stream["scaling"] == "weak" and sorted(r["rank"] for r in stream["ranks"]) == [0, 1]
    # its denominator: the node's pinned copy rate with both ranks copying at once (N x bytes over the
    # slowest rank's time), a rank's fair share of it, and each rank's own concurrent rate beside
    # (solo denominators gave fractions > 1 at N = 8)
    node = stream["node_concurrent_copy_ceiling"]
    assert node["h2d_GBps"] > 0 and node["d2h_GBps"] > 0
    for r in stream["ranks"]:
        assert set(r["concurrent_pinned_GBps"]) == {"h2d", "d2h"} and r["concurrent_pinned_GBps"]["h2d"] > 0
        assert abs(r["fair_share_h2d_GBps"] - node["h2d_GBps"] / 2) < 0.02
        assert abs(r["frac_of_fair_share_h2d"] / (r["h2d_GBps"] / r["fair_share_h2d_GBps"]) - 1) < 1e-2   # rounding
        if r.get("measured_pinned_GBps"):
            assert abs(r["frac_of_h2d"] / (r["h2d_GBps"] / r["measured_pinned_GBps"]["h2d"]) - 1) < 1e-2

def test_strong_split_ranges():
    """configs[3]'s 8192 stripes cut into contiguous ranges that cover the
    total exactly once for every world size, the first ranks one longer."""
    sys.path.insert(0, ROOT)
    import bench

    for world in range(1, 17):
        rs = [bench.split_range(8192 + 5, world, r) for r in range(world)]
        assert rs[0][0] == 0 and sum(n for _, n in rs) == 8197
        assert all(a + n == b for (a, n), (b, _) in zip(rs, rs[1:]))
        assert max(n for _, n in rs) - min(n for _, n in rs) <= 1


def test_bench_world_mismatch_refused():
    """Under an external launcher, --gpus must equal WORLD_SIZE (a driver
    that launches N ranks reports N, never silently 1)."""
    env = dict(_bench_env(), WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rehearse"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "--gpus 2" in (r.stderr + r.stdout)
