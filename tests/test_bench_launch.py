"""bench.py's multi-GPU launch contract (CPU): `bench.py --gpus N` alone spawns
N rank processes (one per GPU, rendezvous on 127.0.0.1) before anything
touches the GPU; under torch.distributed.run the ranks come from the launcher
and WORLD_SIZE must equal --gpus.  Space placement is the reference's
dispatcher placing spaces on game processes (DispatcherService.go:529-540)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_single_gpu_runs_in_process():
    assert bench.launch_plan(1, {}) is None


def test_gpus_n_spawns_n_ranks():
    plan = bench.launch_plan(4, {"PATH": "/bin"})
    assert len(plan) == 4
    assert [e["RANK"] for e in plan] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in plan] == ["0", "1", "2", "3"]
    assert {e["WORLD_SIZE"] for e in plan} == {"4"}
    assert {e["MASTER_ADDR"] for e in plan} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in plan}) == 1
    assert all(e["PATH"] == "/bin" for e in plan)


def test_outside_launcher_must_match():
    assert bench.launch_plan(2, {"WORLD_SIZE": "2", "RANK": "1"}) is None
    with pytest.raises(ValueError):
        bench.launch_plan(8, {"WORLD_SIZE": "2"})
    with pytest.raises(ValueError):
        bench.launch_plan(0, {})


def test_mismatch_exits_nonzero_before_gpu_work():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=3" in r.stderr


def test_spawn_propagates_rank_failure(monkeypatch, tmp_path):
    """spawn_ranks re-runs this script per rank; a failing rank fails the job."""
    script = tmp_path / "fake.py"
    script.write_text("import os, sys\nsys.exit(3 if os.environ['RANK'] == '1' else 0)\n")
    monkeypatch.setattr(bench, "__file__", str(script))
    monkeypatch.setattr(sys, "argv", [str(script)])
    assert bench.spawn_ranks(bench.launch_plan(2, dict(os.environ))) == 3
    script.write_text("import sys\nsys.exit(0)\n")
    assert bench.spawn_ranks(bench.launch_plan(3, dict(os.environ))) == 0


def test_line_summary_is_last_and_compact():
    """The headline numbers of every leg close the JSON line (a stdout tail keeps them)."""
    out = {"ms_per_step": 0.21, "p99_tick_ms": 0.23, "roofline": {"avg_launch_ms": 0.07, "frac": 0.08},
           "host_to_host_tick": {"ms_per_step": 0.35, "p50_tick_ms": 0.6, "p99_tick_ms": 0.7,
                                 "serial_p99_tick_ms": 0.69},
           "small_flush": {"1": {"device": {"p50_ms": 0.05}}, "note": "x"},
           "cfg5_strips": {"error": "cfg5 child job: exit timeout"}, "cpu_baseline": None}
    s = bench.line_summary(out)
    assert s["host_to_host_p99_ms"] == 0.7 and s["combined_ms"] == 0.07
    assert s["small_flush_p50_ms"] == {"1": 0.05}
    assert s["cfg5_error"].startswith("cfg5 child job") and s["cpu_grid_ms_per_tick"] is None
    assert len(__import__("json").dumps(s)) < 1200


def test_cpu_core_counts_bounded_by_affinity():
    c = bench.cpu_core_counts()
    assert 1 <= c["used"] <= c["affinity"]
    assert c["cgroup_quota"] is None or c["used"] <= c["cgroup_quota"]
