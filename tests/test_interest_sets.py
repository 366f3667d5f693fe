"""CPU test of the replay's per-entity interest sets (tools/interest_sets.hpp):
the host-side InterestedIn / InterestedBy of Entity.go:236-246 that the C++
tick bench (tools/tick_bench.cpp) replays the flush's events into, checked
against std::set over random add / delete streams."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_interest_sets_match_std_set(tmp_path):
    exe = tmp_path / "interest_sets_test"
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-o", str(exe),
                    os.path.join(ROOT, "tests", "cpp", "interest_sets_test.cpp")], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok")
