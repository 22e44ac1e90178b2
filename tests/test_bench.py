"""bench.py's multi-rank harness on the CPU (gloo): the launcher, rendezvous, rank count, max-over-ranks
timing and the JSON line, without a GPU (--workload selftest times a trivial CPU step under the same
harness the GPU workloads use; tools/bench_harness.py)."""
import json
import os
import subprocess
import sys

import pytest

from tools import bench_harness as bh

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None, timeout=240):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=e, cwd=ROOT)


def _lines(stdout):
    return [json.loads(ln) for ln in stdout.splitlines() if ln.startswith("{")]


@pytest.mark.parametrize("scaling", ["weak", "strong"])
def test_launcher_two_ranks_one_json_line(scaling):
    r = _run(["--gpus", "2", "--workload", "selftest", "--steps", "3", "--warmup", "1", "--settle-s", "0",
              "--pairs", "1000", "--scaling", scaling])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _lines(r.stdout)
    assert len(lines) == 1, r.stdout
    d = lines[0]
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2 and len(d["rank_ms_per_step"]) == 2
    assert d["scaling"] == scaling and d["steps"] == 3
    # value = every unit processed by all ranks / the slowest rank's time
    total = (1000 * 2 if scaling == "weak" else 1000) * 3
    assert abs(d["value"] * d["ms_per_step"] * 3 / 1e3 - total) <= 1e-6 * total
    assert abs(d["ms_per_step"] - max(d["rank_ms_per_step"])) <= 1e-9 * d["ms_per_step"] + 1e-12


@pytest.mark.parametrize("graph", ["on", "off"])
def test_strong_scaling_two_ranks_graph_flag(graph):
    """--scaling strong on 2 ranks with the graph-replay timing the evalpdf workload uses for short kernels: both
    figures reported, value from the graph-timed one, exactly K steps timed as K/R replays of R launches."""
    r = _run(["--gpus", "2", "--workload", "selftest", "--steps", "12", "--warmup", "1", "--settle-s", "0",
              "--pairs", "2000", "--scaling", "strong", "--graph", graph])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _lines(r.stdout)[0]
    assert d["ranks_seen"] == 2 and d["scaling"] == "strong"
    t = d["timing"]
    assert "launch_timed" in t and len(t["launch_timed"]["rank_ms_per_step"]) == 2
    if graph == "on":
        g = t["graph_timed"]
        assert t["value_from"] == "graph_timed" and g["launches_per_replay"] * g["replays"] == 12
        assert g["launches_per_replay"] == bh.graph_reps(12) == 12
        assert abs(d["ms_per_step"] - max(g["rank_ms_per_step"])) <= 1e-9 * d["ms_per_step"] + 1e-12
    else:
        assert t["value_from"] == "launch_timed" and "graph_timed" not in t
    assert abs(d["value"] * d["ms_per_step"] * 12 / 1e3 - 2000 * 12) <= 1e-6 * 2000 * 12


def test_graph_reps_divides_steps():
    for k in (1, 7, 12, 20, 50, 97, 100):
        r = bh.graph_reps(k)
        assert k % r == 0 and 1 <= r <= 20


def test_launcher_single_rank_default():
    r = _run(["--workload", "selftest", "--steps", "2", "--warmup", "0", "--settle-s", "0", "--pairs", "10"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _lines(r.stdout)[0]
    assert d["n_gpus"] == 1 and d["ranks_seen"] == 1


def test_gpus_must_match_launcher_world_size():
    r = _run(["--gpus", "4", "--workload", "selftest", "--steps", "1", "--warmup", "0"],
             env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in (r.stderr + r.stdout)


def test_shard_ranges_cover_the_batch():
    for world in (1, 2, 3, 8):
        # weak: every rank owns per_rank units of [0, world * per_rank)
        spans = [bh.shard(100, r, world, "weak") for r in range(world)]
        assert spans == [(100 * r, 100) for r in range(world)]
        # strong: a fixed total split into contiguous, disjoint, covering ranges
        spans = [bh.shard(1001, r, world, "strong") for r in range(world)]
        assert spans[0][0] == 0 and sum(c for _, c in spans) == 1001
        assert all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(world - 1))
        assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def test_cpu_topology_is_consistent():
    threads, phys, smt, quota, _ = bh.cpu_topology()
    assert threads == len(os.sched_getaffinity(0)) and 1 <= phys <= threads and smt >= 1
    assert quota is None or quota > 0


def test_pmc_summary_keeps_to_the_longest_matching_kernel(tmp_path):
    """tools/pmc_summary.py: a pattern that also matches a short companion kernel (k_check -> k_check_final) must not
    mix the companion's dispatches into the medians -- the summary is the longest matching kernel's."""
    from tools import pmc_summary
    rows = ["Kernel_Name,Dispatch_Id,Counter_Name,Counter_Value,Start_Timestamp,End_Timestamp"]
    for d in range(3):
        rows.append(f'"void k_check<M, 0>(CheckArgs)",{2 * d},SQ_INSTS_VALU,{1000 + d},0,{2_000_000 + d}')
        rows.append(f'"k_check_final(double const*, int, double*)",{2 * d + 1},SQ_INSTS_VALU,7,0,5000')
    p = tmp_path / "pass1" / "run"
    p.mkdir(parents=True)
    (p / "x_counter_collection.csv").write_text("\n".join(rows) + "\n")
    s = pmc_summary.summarise(str(tmp_path), "k_check")
    assert s["SQ_INSTS_VALU"] == 1001 and s["dispatches"] == 3 and s["dispatch_ns"] == 2_000_001
    both = pmc_summary.summarise(str(tmp_path), "k_check", by_kernel=True)
    assert len(both) == 2
