"""C++ host mirror of the AOIManager interface (include/gwaoi_aoi.hpp):
builds against the in-tree libgwaoi.so here; on the GPU its test program
(tests/cpp/aoi_manager_test.cpp) runs KATs and a random churn stream checked
against the closed form, with In == By."""
import os
import subprocess

import pytest

from goworld_amd import build


def test_cpp_mirror_builds_and_links():
    exe = build.build_cpp_tests()
    assert os.access(exe, os.X_OK)
    out = subprocess.run(["nm", "-D", "--undefined-only", exe], capture_output=True, text=True, check=True).stdout
    for sym in ("gwaoi_world_create", "gwaoi_tick", "gwaoi_moved_batch", "gwaoi_enter_batch", "gwaoi_leave_batch"):
        assert sym in out


@pytest.mark.gpu
def test_cpp_mirror_on_gpu():
    exe = build.build_cpp_tests()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "ok"
