"""The C-ABI library loads without a GPU and exports every function that
include/gwaoi.h declares (no compute calls here)."""
import ctypes as C
import os
import re

import pytest

from goworld_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions(name="gwaoi.h"):
    src = open(os.path.join(ROOT, "include", name)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gwaoi_[a-z_0-9]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from goworld_amd import build
    build.build()
    return _lib.load()


def test_header_lists_match_binding():
    assert header_functions() == sorted(_lib.EXPORTS)
    assert header_functions("gwaoi_strips.h") == sorted(_lib.STRIP_EXPORTS)
    assert header_functions("gwaoi_sync.h") == sorted(_lib.SYNC_EXPORTS)
    assert header_functions("gwaoi_wire.h") == sorted(_lib.WIRE_EXPORTS)


def test_library_exports_every_declared_symbol(lib):
    for name in (header_functions() + header_functions("gwaoi_strips.h") + header_functions("gwaoi_sync.h") +
                 header_functions("gwaoi_wire.h")):
        assert hasattr(lib, name), name
        assert C.cast(getattr(lib, name), C.c_void_p).value


def test_pure_host_entry_points(lib):
    assert lib.gwaoi_abi_version() == 6
    assert lib.gwaoi_strerror(0) == b"ok"
    assert b"state" in lib.gwaoi_strerror(-3)
    # null-argument handling never touches the device
    assert lib.gwaoi_world_create(None, None) == -1
    assert lib.gwaoi_tick(None, None) == -1
    # the flush end (one entry point, mode bits) and its host readers validate the handle first
    assert lib.gwaoi_tick_finish(None, 0, None, None) == -1
    assert lib.gwaoi_tick_finish(None, 7, None, None) == -1
    assert lib.gwaoi_events_host(None, None) == -1
    assert lib.gwaoi_pairs_host(None, None) == -1
    assert lib.gwaoi_world_destroy(None) == -1
    # entity-sync entry points validate before any device work
    assert lib.gwaoi_entity_bind(None, 0, None) == -1
    assert lib.gwaoi_sync_from_clients(None, None, 0) == -1
    assert lib.gwaoi_collect_sync_infos(None, None) == -1
    assert lib.gwaoi_collect_client_events(None, None, None) == -1
    # wire regroups validate the handle first
    assert lib.gwaoi_wire_create(0, None) == -1
    assert lib.gwaoi_wire_gate_from_clients(None, None, 0, 4, None) == -1
    assert lib.gwaoi_wire_gate_to_clients(None, None, 0, None) == -1
    assert lib.gwaoi_wire_set_clients(None, None, None, 0) == -1


def test_library_is_gfx950_code_object():
    path = _lib.LIB_PATH
    data = open(path, "rb").read()
    assert b"gfx950" in data
    assert b"amdgcn-amd-amdhsa" in data


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(ImportError):
        _lib.load()
