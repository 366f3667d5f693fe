"""ctypes binding of libgwaoi.so (include/gwaoi.h).

The shared library is built in-tree (goworld_amd/lib/libgwaoi.so) by
``goworld_amd.build``.  There is no fallback: if the library is missing,
``load()`` raises.  PyTorch, when installed, is imported first so that the
process holds exactly one HIP runtime (torch bundles its own libamdhip64, and
libgwaoi then binds to that copy by soname).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# GWAOI_LIB: an alternative in-tree build (tools/variants.sh, A/B tuning runs)
LIB_PATH = os.environ.get("GWAOI_LIB") or os.path.join(HERE, "lib", "libgwaoi.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "gwaoi.h")

GWAOI_F_TIMING = 1
GWAOI_F_NO_SPARSE = 2  # never the sparse flush (include/gwaoi.h)
GWAOI_F_BATCH_READY = 4  # accepted and ignored since ABI 5
GWAOI_F_UNIQUE_MOVES = 8  # a flush's Moved batches never repeat a slot: no last-op claims (checked on device)
# test and diagnostics flags (include/gwaoi.h): a slower or failing path, to compare with the default one
GWAOI_F_TEST_FORCE_RADIX = 0x100
GWAOI_F_TEST_FORCE_COPY = 0x200
GWAOI_F_TEST_BUCKETED = 0x400
GWAOI_F_TEST_REGROW_FAIL = 0x800
GWAOI_F_TEST_SPARSE_SEQUENCE = 0x1000
GWAOI_F_TEST_SPARSE_SCR2 = 0x2000
GWAOI_F_TEST_CHECK_STAGES = 0x4000

STATUS = {
    0: "GWAOI_OK", -1: "GWAOI_EINVAL", -2: "GWAOI_EBADSLOT", -3: "GWAOI_ESTATE", -4: "GWAOI_ENOMEM",
    -5: "GWAOI_EDEVICE", -6: "GWAOI_ENONFINITE", -7: "GWAOI_EBADSPACE", -8: "GWAOI_EBUSY",
    -9: "GWAOI_ECAPACITY",
}

# every function include/gwaoi.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "gwaoi_world_create", "gwaoi_world_destroy", "gwaoi_space_create", "gwaoi_space_destroy",
    "gwaoi_enter", "gwaoi_leave", "gwaoi_moved", "gwaoi_enter_batch", "gwaoi_leave_batch",
    "gwaoi_moved_batch", "gwaoi_moved_batch_device", "gwaoi_tick", "gwaoi_tick_device",
    "gwaoi_events_device", "gwaoi_neighbors", "gwaoi_world_info", "gwaoi_stage_times",
    "gwaoi_reset_stage_times", "gwaoi_set_stage_timing", "gwaoi_sync", "gwaoi_stream", "gwaoi_stream_after", "gwaoi_stream_before", "gwaoi_strerror", "gwaoi_last_error",
    "gwaoi_abi_version", "gwaoi_enter_seq", "gwaoi_moved_seq", "gwaoi_moved_batch_device_seq",
    "gwaoi_snapshot", "gwaoi_restore", "gwaoi_debug_counters", "gwaoi_tick_begin", "gwaoi_tick_finish",
    "gwaoi_events_csr", "gwaoi_events_csr_device",
    "gwaoi_enter_batch_device", "gwaoi_leave_batch_device", "gwaoi_moved_batch_stage",
    "gwaoi_moved_batch_commit", "gwaoi_moved_batch_pinned", "gwaoi_pinned_alloc", "gwaoi_pinned_free",
    "gwaoi_events_host", "gwaoi_pairs_host",
]

# gwaoi_tick_finish modes
GWAOI_END_NEXT, GWAOI_END_HOST, GWAOI_END_PAIRS = 1, 2, 4

# every function include/gwaoi_strips.h declares
STRIP_EXPORTS = [
    "gwaoi_strips_create", "gwaoi_strips_destroy", "gwaoi_strips_halo", "gwaoi_strips_route",
    "gwaoi_strips_route_scatter", "gwaoi_strips_tick", "gwaoi_strips_events_device", "gwaoi_strips_events",
    "gwaoi_strips_last_error", "gwaoi_strips_route_kinds", "gwaoi_strips_tick_async", "gwaoi_strips_wait",
    "gwaoi_strips_host_waits", "gwaoi_strips_route_row_words", "gwaoi_strips_route_begin", "gwaoi_strips_route_end",
]

# every function include/gwaoi_sync.h declares
SYNC_EXPORTS = [
    "gwaoi_entity_bind", "gwaoi_entity_bind_batch", "gwaoi_entity_unbind", "gwaoi_entity_set_client",
    "gwaoi_entity_set_syncing", "gwaoi_entity_set_position_yaw", "gwaoi_set_position_yaw",
    "gwaoi_sync_from_clients", "gwaoi_sync_from_clients_device", "gwaoi_collect_sync_infos",
    "gwaoi_collect_sync_infos_device", "gwaoi_collect_client_events", "gwaoi_entity_enter_plain",
    "gwaoi_entity_leave_plain",
]

# every function include/gwaoi_wire.h declares
WIRE_EXPORTS = [
    "gwaoi_wire_create", "gwaoi_wire_destroy", "gwaoi_wire_last_error", "gwaoi_wire_set_entity_games",
    "gwaoi_wire_remove_entities", "gwaoi_wire_set_clients", "gwaoi_wire_remove_clients",
    "gwaoi_wire_gate_from_clients", "gwaoi_wire_gate_from_clients_device", "gwaoi_wire_dispatcher_to_games",
    "gwaoi_wire_dispatcher_to_games_device", "gwaoi_wire_gate_to_clients", "gwaoi_wire_gate_to_clients_device",
]

SYNC_OUT_REC = 48  # ClientID[16] + EntityID[16] + x,y,z,yaw float32 (Entity.go:1233-1251)
DESTROY_REC = 32   # ClientID[16] + EntityID[16]
SIF_OWN_CLIENT, SIF_NEIGHBOR_CLIENTS = 1, 2


class Config(C.Structure):
    _fields_ = [("max_slots", C.c_uint32), ("max_spaces", C.c_uint32), ("device", C.c_int32),
                ("flags", C.c_uint32), ("event_capacity", C.c_uint64), ("cells_per_dist", C.c_float)]


class Events(C.Structure):
    _fields_ = [("n_enter", C.c_uint64), ("n_leave", C.c_uint64),
                ("enter", C.POINTER(C.c_uint32)), ("leave", C.POINTER(C.c_uint32))]


class Info(C.Structure):
    _fields_ = [("ticks", C.c_uint64), ("next_seq", C.c_uint64), ("live", C.c_uint32),
                ("spaces", C.c_uint32), ("total_cells", C.c_uint32), ("pending_ops", C.c_uint32),
                ("event_capacity", C.c_uint64), ("max_slots", C.c_uint32), ("max_spaces", C.c_uint32)]


class StripsConfig(C.Structure):
    _fields_ = [("n_strips", C.c_uint32), ("rank", C.c_uint32), ("edges", C.c_void_p),
                ("aoi_distance", C.c_float), ("teleport", C.c_float)]


class GateRecords(C.Structure):
    _fields_ = [("n_gates", C.c_uint32), ("gate_ids", C.POINTER(C.c_uint16)),
                ("offsets", C.POINTER(C.c_uint64)), ("records", C.c_void_p)]


class WireGroups(C.Structure):
    _fields_ = [("n_groups", C.c_uint32), ("keys", C.POINTER(C.c_uint32)), ("offsets", C.POINTER(C.c_uint64)),
                ("records", C.c_void_p), ("rec_bytes", C.c_uint32), ("n_dropped", C.c_uint64)]


class Debug(C.Structure):
    _fields_ = [("flushes", C.c_uint64), ("combined_replays", C.c_uint64), ("combined_queue_drains", C.c_uint64),
                ("special_global", C.c_uint64), ("event_regrows", C.c_uint64), ("speculative_launches", C.c_uint64),
                ("cell_size_switches", C.c_uint64), ("cells_per_dist", C.c_uint32), ("pad", C.c_uint32),
                ("incremental_sorts", C.c_uint64), ("sparse_flushes", C.c_uint64), ("sparse_declined", C.c_uint64),
                ("premarked_runs", C.c_uint64), ("sparse_unfused", C.c_uint64),
                ("unique_flushes", C.c_uint64), ("overlapped_flushes", C.c_uint64)]


class StageTime(C.Structure):
    _fields_ = [("name", C.c_char * 32), ("ms", C.c_double), ("calls", C.c_uint64)]


class GwaoiError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{STATUS.get(code, code)}: {msg}")
        self.code = code
        self.events = None  # tick(): the committed flush's (enter, leave) pairs, still to replay


_lib = None


def load():
    """Load libgwaoi.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
    try:  # one HIP runtime per process: bind to torch's copy when torch is present
        import torch  # noqa: F401
    except Exception:
        pass
    L = C.CDLL(LIB_PATH)
    vp, u32, u64, f, sz = C.c_void_p, C.c_uint32, C.c_uint64, C.c_float, C.c_size_t
    P = C.POINTER
    sigs = {
        "gwaoi_world_create": ([P(Config), P(vp)], C.c_int),
        "gwaoi_world_destroy": ([vp], C.c_int),
        "gwaoi_space_create": ([vp, f, P(u32)], C.c_int),
        "gwaoi_space_destroy": ([vp, u32], C.c_int),
        "gwaoi_enter": ([vp, u32, u32, f, f], C.c_int),
        "gwaoi_leave": ([vp, u32], C.c_int),
        "gwaoi_moved": ([vp, u32, f, f], C.c_int),
        "gwaoi_enter_batch": ([vp, u32, vp, vp, vp, sz], C.c_int),
        "gwaoi_leave_batch": ([vp, vp, sz], C.c_int),
        "gwaoi_moved_batch": ([vp, vp, vp, vp, sz], C.c_int),
        "gwaoi_moved_batch_device": ([vp, vp, vp, vp, sz], C.c_int),
        "gwaoi_tick": ([vp, P(Events)], C.c_int),
        "gwaoi_tick_device": ([vp, P(u64), P(u64)], C.c_int),
        "gwaoi_tick_begin": ([vp], C.c_int),
        "gwaoi_events_csr": ([vp, P(vp), P(vp), P(u64)], C.c_int),
        "gwaoi_events_csr_device": ([vp, P(vp), P(vp), P(u64)], C.c_int),
        "gwaoi_tick_finish": ([vp, C.c_uint32, P(u64), P(u64)], C.c_int),
        "gwaoi_events_host": ([vp, P(Events)], C.c_int),
        "gwaoi_pairs_host": ([vp, P(Events)], C.c_int),
        "gwaoi_moved_batch_stage": ([vp, sz, P(vp), P(vp), P(vp)], C.c_int),
        "gwaoi_moved_batch_commit": ([vp, sz], C.c_int),
        "gwaoi_moved_batch_pinned": ([vp, vp, vp, vp, sz], C.c_int),
        "gwaoi_pinned_alloc": ([vp, sz, P(vp)], C.c_int),
        "gwaoi_pinned_free": ([vp, vp], C.c_int),
        "gwaoi_events_device": ([vp, P(vp), P(vp)], C.c_int),
        "gwaoi_neighbors": ([vp, u32, vp, sz, P(sz)], C.c_int),
        "gwaoi_world_info": ([vp, P(Info)], C.c_int),
        "gwaoi_debug_counters": ([vp, P(Debug)], C.c_int),
        "gwaoi_stage_times": ([vp, P(StageTime), sz, P(sz)], C.c_int),
        "gwaoi_reset_stage_times": ([vp], C.c_int),
        "gwaoi_set_stage_timing": ([vp, C.c_uint32], C.c_int),
        "gwaoi_sync": ([vp], C.c_int),
        "gwaoi_stream": ([vp], vp),
        "gwaoi_stream_after": ([vp, vp], C.c_int),
        "gwaoi_stream_before": ([vp, vp], C.c_int),
        "gwaoi_strerror": ([C.c_int], C.c_char_p),
        "gwaoi_last_error": ([vp], C.c_char_p),
        "gwaoi_abi_version": ([], C.c_int),
        "gwaoi_enter_seq": ([vp, u32, u32, f, f, u64], C.c_int),
        "gwaoi_moved_seq": ([vp, u32, f, f, u64], C.c_int),
        "gwaoi_moved_batch_device_seq": ([vp, vp, vp, vp, vp, sz], C.c_int),
        "gwaoi_enter_batch_device": ([vp, u32, vp, vp, vp, vp, sz, vp], C.c_int),
        "gwaoi_leave_batch_device": ([vp, u32, vp, sz], C.c_int),
        "gwaoi_strips_create": ([vp, u32, P(StripsConfig), P(vp)], C.c_int),
        "gwaoi_strips_destroy": ([vp], C.c_int),
        "gwaoi_strips_halo": ([vp, P(f)], C.c_int),
        "gwaoi_strips_route": ([vp, vp, sz, P(u64)], C.c_int),
        "gwaoi_strips_route_row_words": ([vp, P(u32)], C.c_int),
        "gwaoi_strips_route_begin": ([vp, vp, sz, vp], C.c_int),
        "gwaoi_strips_route_end": ([vp, vp, P(vp), P(u64)], C.c_int),
        "gwaoi_strips_route_scatter": ([vp, vp, vp], C.c_int),
        "gwaoi_strips_tick": ([vp, vp, sz, vp, sz, vp, sz, P(u64), P(u64)], C.c_int),
        "gwaoi_strips_route_kinds": ([vp, vp, vp, vp], C.c_int),
        "gwaoi_strips_tick_async": ([vp, vp, sz, vp, sz, vp, sz, u64, u64, vp], C.c_int),
        "gwaoi_strips_wait": ([vp, P(u64), P(u64)], C.c_int),
        "gwaoi_strips_host_waits": ([vp, P(u64)], C.c_int),
        "gwaoi_strips_events_device": ([vp, P(vp), P(vp)], C.c_int),
        "gwaoi_strips_events": ([vp, P(Events)], C.c_int),
        "gwaoi_strips_last_error": ([vp], C.c_char_p),
        "gwaoi_snapshot": ([vp, vp, vp, vp, vp, vp, sz, P(sz)], C.c_int),
        "gwaoi_restore": ([vp, vp, vp, vp, vp, vp, sz], C.c_int),
        "gwaoi_entity_bind": ([vp, u32, vp], C.c_int),
        "gwaoi_entity_bind_batch": ([vp, vp, vp, sz], C.c_int),
        "gwaoi_entity_unbind": ([vp, u32], C.c_int),
        "gwaoi_entity_set_client": ([vp, u32, C.c_uint16, vp], C.c_int),
        "gwaoi_entity_set_syncing": ([vp, u32, C.c_int], C.c_int),
        "gwaoi_entity_set_position_yaw": ([vp, u32, f, f, f, f], C.c_int),
        "gwaoi_set_position_yaw": ([vp, u32, f, f, f, f], C.c_int),
        "gwaoi_entity_enter_plain": ([vp, u32, f, f, f], C.c_int),
        "gwaoi_entity_leave_plain": ([vp, u32], C.c_int),
        "gwaoi_sync_from_clients": ([vp, vp, sz], C.c_int),
        "gwaoi_sync_from_clients_device": ([vp, vp, sz], C.c_int),
        "gwaoi_collect_sync_infos": ([vp, P(GateRecords)], C.c_int),
        "gwaoi_collect_sync_infos_device": ([vp, P(GateRecords)], C.c_int),
        "gwaoi_collect_client_events": ([vp, P(GateRecords), P(GateRecords)], C.c_int),
        "gwaoi_wire_create": ([C.c_int, P(vp)], C.c_int),
        "gwaoi_wire_destroy": ([vp], None),
        "gwaoi_wire_last_error": ([vp], C.c_char_p),
        "gwaoi_wire_set_entity_games": ([vp, vp, vp, sz], C.c_int),
        "gwaoi_wire_remove_entities": ([vp, vp, sz], C.c_int),
        "gwaoi_wire_set_clients": ([vp, vp, vp, sz], C.c_int),
        "gwaoi_wire_remove_clients": ([vp, vp, sz], C.c_int),
        "gwaoi_wire_gate_from_clients": ([vp, vp, sz, u32, P(WireGroups)], C.c_int),
        "gwaoi_wire_gate_from_clients_device": ([vp, vp, sz, u32, P(WireGroups)], C.c_int),
        "gwaoi_wire_dispatcher_to_games": ([vp, vp, sz, P(WireGroups)], C.c_int),
        "gwaoi_wire_dispatcher_to_games_device": ([vp, vp, sz, P(WireGroups)], C.c_int),
        "gwaoi_wire_gate_to_clients": ([vp, vp, sz, P(WireGroups)], C.c_int),
        "gwaoi_wire_gate_to_clients_device": ([vp, vp, sz, P(WireGroups)], C.c_int),
    }
    for name, (args, res) in sigs.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class World:
    """One GPU AOI world: many spaces, one HIP stream (include/gwaoi.h)."""

    def __init__(self, max_slots: int, max_spaces: int = 1, device: int = -1, timing: bool = False,
                 event_capacity: int = 0, cells_per_dist: float = 0.0, sparse: bool = True,
                 unique_moves: bool = False, test_flags: int = 0):
        """test_flags: an OR of GWAOI_F_TEST_* (tests comparing a slower path with the default one)."""
        self._L = load()
        flags = ((GWAOI_F_TIMING if timing else 0) | (0 if sparse else GWAOI_F_NO_SPARSE) |
                 (GWAOI_F_UNIQUE_MOVES if unique_moves else 0) | int(test_flags))
        cfg = Config(max_slots, max_spaces, device, flags, event_capacity, cells_per_dist)
        h = C.c_void_p()
        self._check(self._L.gwaoi_world_create(C.byref(cfg), C.byref(h)), world=False)
        self._w = h
        self.max_slots = max_slots

    def close(self):
        if getattr(self, "_w", None):
            self._L.gwaoi_world_destroy(self._w)
            self._w = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc, world=True):
        if rc != 0:
            msg = self._L.gwaoi_strerror(rc).decode()
            if world and getattr(self, "_w", None):
                last = self._L.gwaoi_last_error(self._w).decode()
                if last:
                    msg += f" ({last})"
            raise GwaoiError(rc, msg)
        return rc

    # ---- spaces / AOIManager calls
    def space_create(self, aoi_distance) -> int:
        s = C.c_uint32()
        self._check(self._L.gwaoi_space_create(self._w, C.c_float(aoi_distance), C.byref(s)))
        return s.value

    def space_destroy(self, space):
        self._check(self._L.gwaoi_space_destroy(self._w, space))

    def enter(self, space, slot, x, z, seq=None):
        if seq is None:
            self._check(self._L.gwaoi_enter(self._w, space, slot, C.c_float(x), C.c_float(z)))
        else:
            self._check(self._L.gwaoi_enter_seq(self._w, space, slot, C.c_float(x), C.c_float(z), int(seq)))

    def leave(self, slot):
        self._check(self._L.gwaoi_leave(self._w, slot))

    def moved(self, slot, x, z, seq=None):
        if seq is None:
            self._check(self._L.gwaoi_moved(self._w, slot, C.c_float(x), C.c_float(z)))
        else:
            self._check(self._L.gwaoi_moved_seq(self._w, slot, C.c_float(x), C.c_float(z), int(seq)))

    def enter_batch(self, space, slots, x, z):
        s = np.ascontiguousarray(slots, np.uint32)
        x = np.ascontiguousarray(x, np.float32)
        z = np.ascontiguousarray(z, np.float32)
        self._check(self._L.gwaoi_enter_batch(self._w, space, _p(s), _p(x), _p(z), s.size))

    def leave_batch(self, slots):
        s = np.ascontiguousarray(slots, np.uint32)
        self._check(self._L.gwaoi_leave_batch(self._w, _p(s), s.size))

    def moved_batch(self, slots, x, z):
        s = np.ascontiguousarray(slots, np.uint32)
        x = np.ascontiguousarray(x, np.float32)
        z = np.ascontiguousarray(z, np.float32)
        self._check(self._L.gwaoi_moved_batch(self._w, _p(s), _p(x), _p(z), s.size))

    def stage_moves(self, n: int):
        """gwaoi_moved_batch_stage: (slots, x, z) numpy views of n moves in the world's pinned
        staging memory, to be filled by the caller and queued with commit_moves(k)."""
        ps, px, pz = C.c_void_p(), C.c_void_p(), C.c_void_p()
        self._check(self._L.gwaoi_moved_batch_stage(self._w, n, C.byref(ps), C.byref(px), C.byref(pz)))
        u32, f32 = C.POINTER(C.c_uint32), C.POINTER(C.c_float)
        return (np.ctypeslib.as_array(C.cast(ps, u32), shape=(n,)), np.ctypeslib.as_array(C.cast(px, f32), shape=(n,)),
                np.ctypeslib.as_array(C.cast(pz, f32), shape=(n,)))

    def commit_moves(self, k: int):
        """gwaoi_moved_batch_commit: queue the first k staged moves (one H2D, checked on the device)."""
        self._check(self._L.gwaoi_moved_batch_commit(self._w, k))

    def pinned_batch(self, n: int):
        """A move batch buffer in pinned host memory (gwaoi_pinned_alloc): (slots, x, z) numpy
        arrays of n moves; free with free_pinned_batch.  Queue a filled prefix with moved_batch_pinned."""
        p = C.c_void_p()
        self._check(self._L.gwaoi_pinned_alloc(self._w, 12 * n, C.byref(p)))
        buf = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint32)), shape=(3 * n,))
        return p.value, (buf[:n], buf[n:2 * n].view(np.float32), buf[2 * n:].view(np.float32))

    def free_pinned_batch(self, ptr: int):
        self._check(self._L.gwaoi_pinned_free(self._w, C.c_void_p(ptr)))

    def moved_batch_pinned(self, views, k: int):
        """gwaoi_moved_batch_pinned: the first k moves of a pinned_batch (read in place by the H2D)."""
        s, x, z = views
        self._check(self._L.gwaoi_moved_batch_pinned(self._w, _p(s), _p(x), _p(z), k))

    def moved_batch_device(self, d_slots: int, d_x: int, d_z: int, n: int, d_seq: int | None = None):
        if d_seq is None:
            self._check(self._L.gwaoi_moved_batch_device(self._w, C.c_void_p(d_slots), C.c_void_p(d_x),
                                                         C.c_void_p(d_z), n))
        else:
            self._check(self._L.gwaoi_moved_batch_device_seq(self._w, C.c_void_p(d_slots), C.c_void_p(d_x),
                                                             C.c_void_p(d_z), C.c_void_p(d_seq), n))

    def enter_batch_device(self, space, d_slots: int, d_x: int, d_z: int, n: int, d_seq: int | None = None,
                           box=None):
        """gwaoi_enter_batch_device: Enter calls whose arrays live in device memory (slots
        not live; box = (x0, z0, x1, z1) around the positions, or None)."""
        b = np.ascontiguousarray(box, np.float32) if box is not None else None
        self._check(self._L.gwaoi_enter_batch_device(self._w, space, C.c_void_p(d_slots), C.c_void_p(d_x),
                                                     C.c_void_p(d_z), C.c_void_p(d_seq) if d_seq else None, n,
                                                     _p(b) if b is not None else None))

    def leave_batch_device(self, space, d_slots: int, n: int):
        self._check(self._L.gwaoi_leave_batch_device(self._w, space, C.c_void_p(d_slots), n))

    # ---- flush
    def tick(self, copy: bool = True):
        """Flush; returns (enter_pairs, leave_pairs) as (n,2) uint32 arrays [a, b].

        When the flush committed but the device reported a problem in the queued
        ops (a dropped move: ESTATE / ENONFINITE / EINVAL), the GwaoiError carries
        the flush's events as ``.events``: they must still be replayed.
        copy=False: views of the world's pinned buffer, valid until the next flush."""
        ev = Events()
        return self._events(self._L.gwaoi_tick(self._w, C.byref(ev)), ev, copy)

    def tick_begin(self):
        """Start the flush (gwaoi_tick_begin); AOIManager calls made before tick_end
        are queued for the next flush."""
        self._check(self._L.gwaoi_tick_begin(self._w))

    def finish(self, mode: int = 0):
        """gwaoi_tick_finish(mode): commit the flush in flight; mode is an OR of GWAOI_END_NEXT
        (begin the next flush), GWAOI_END_HOST (events to host memory: events_host) and
        GWAOI_END_PAIRS (one event per mirrored pair: pairs_host).  Returns the finished flush's
        (n_enter, n_leave); on a committed flush with a device-reported problem the GwaoiError
        carries them as ``.counts``."""
        ne, nl = C.c_uint64(), C.c_uint64()
        rc = self._L.gwaoi_tick_finish(self._w, mode, C.byref(ne), C.byref(nl))
        if rc != 0:
            try:
                self._check(rc)
            except GwaoiError as e:
                e.counts = (ne.value, nl.value)
                raise
        return ne.value, nl.value

    def _finish_events(self, mode, copy):
        # the flush's host events with its status: a committed flush with a device-reported
        # problem raises with them as ``.events`` (events_host describes the copy this call made,
        # empty when the flush did not commit)
        err = None
        try:
            self.finish(mode)
        except GwaoiError as e:
            err = e
        ev = Events()
        ok = self._L.gwaoi_events_host(self._w, C.byref(ev)) == 0
        ent, lev = self._events(0, ev, copy) if ok else (None, None)
        if err is not None:
            err.events = (ent, lev) if ok else None
            raise err
        return ent, lev

    def tick_end(self, copy: bool = True):
        """Finish the flush started by tick_begin: (enter_pairs, leave_pairs) as tick()
        (gwaoi_tick_finish(GWAOI_END_HOST))."""
        return self._finish_events(GWAOI_END_HOST, copy)

    def tick_end_device(self):
        """gwaoi_tick_finish(0): events stay in HBM."""
        return self.finish(0)

    def tick_end_begin_device(self):
        """gwaoi_tick_finish(GWAOI_END_NEXT): finish the flush in flight and begin the next one
        (queued on the GPU before this one's commit when only device Moved batches were
        queued).  Returns the finished flush's (n_enter, n_leave); its events stay
        readable through events_device() while the next flush runs."""
        return self.finish(GWAOI_END_NEXT)

    def tick_end_begin(self, copy: bool = True):
        """gwaoi_tick_finish(GWAOI_END_NEXT | GWAOI_END_HOST) + events_host: finish the flush in
        flight (its events copied to host memory beside the next flush) and begin the next one."""
        return self._finish_events(GWAOI_END_NEXT | GWAOI_END_HOST, copy)

    def tick_end_begin_async(self):
        """gwaoi_tick_finish(GWAOI_END_NEXT | GWAOI_END_HOST): the events' copy to host memory is
        left running; returns (n_enter, n_leave).  events_host() waits for it."""
        return self.finish(GWAOI_END_NEXT | GWAOI_END_HOST)

    def tick_end_begin_pairs_async(self):
        """gwaoi_tick_finish(GWAOI_END_NEXT | GWAOI_END_PAIRS): one event per mirrored pair copied
        out; returns the directed (n_enter, n_leave).  pairs_host() waits for them."""
        return self.finish(GWAOI_END_NEXT | GWAOI_END_PAIRS)

    def pairs_host(self, copy: bool = True):
        """gwaoi_pairs_host: (enter pairs, leave pairs) as (n,2) arrays; (a,b) stands for (a,b) and (b,a)."""
        ev = Events()
        return self._events(self._L.gwaoi_pairs_host(self._w, C.byref(ev)), ev, copy)

    def events_host(self, copy: bool = True):
        """gwaoi_events_host: the events of the last tick_end_begin_async in host memory."""
        ev = Events()
        return self._events(self._L.gwaoi_events_host(self._w, C.byref(ev)), ev, copy)

    def _events(self, rc, ev, copy):
        ne, nl = ev.n_enter, ev.n_leave
        cp = (lambda a: a.copy()) if copy else (lambda a: a)
        ent = cp(np.ctypeslib.as_array(ev.enter, shape=(2 * ne,)).reshape(ne, 2)) if ne else np.empty((0, 2), np.uint32)
        lev = cp(np.ctypeslib.as_array(ev.leave, shape=(2 * nl,)).reshape(nl, 2)) if nl else np.empty((0, 2), np.uint32)
        if rc != 0:
            try:
                self._check(rc)
            except GwaoiError as e:
                e.events = (ent, lev) if (ev.enter or ev.leave) else None
                raise
        return ent, lev

    def tick_device(self):
        """Flush; events stay in HBM.  Returns (n_enter, n_leave); on a committed flush
        with a device-reported problem the GwaoiError carries them as ``.counts``."""
        ne, nl = C.c_uint64(), C.c_uint64()
        rc = self._L.gwaoi_tick_device(self._w, C.byref(ne), C.byref(nl))
        if rc != 0:
            try:
                self._check(rc)
            except GwaoiError as e:
                e.counts = (ne.value, nl.value)
                raise
        return ne.value, nl.value

    def events_csr(self):
        """The last flush's events by entity (gwaoi_events_csr): (offsets[max_slots+1], items)
        uint32 copies; item = b | 0x80000000 for an enter (s, b), b for a leave."""
        o, it, n = C.c_void_p(), C.c_void_p(), C.c_uint64()
        self._check(self._L.gwaoi_events_csr(self._w, C.byref(o), C.byref(it), C.byref(n)))
        off = np.ctypeslib.as_array(C.cast(o, C.POINTER(C.c_uint32)), shape=(self.max_slots + 1,)).copy()
        items = (np.ctypeslib.as_array(C.cast(it, C.POINTER(C.c_uint32)), shape=(n.value,)).copy() if n.value
                 else np.empty(0, np.uint32))
        return off, items

    def events_device(self):
        e, l = C.c_void_p(), C.c_void_p()
        self._check(self._L.gwaoi_events_device(self._w, C.byref(e), C.byref(l)))
        return e.value, l.value

    # ---- queries
    def neighbors(self, slot, cap=4096):
        while True:
            out = np.empty(cap, np.uint32)
            n = C.c_size_t()
            self._check(self._L.gwaoi_neighbors(self._w, slot, _p(out), cap, C.byref(n)))
            if n.value <= cap:
                return np.sort(out[:n.value])
            cap = n.value

    def info(self) -> dict:
        i = Info()
        self._check(self._L.gwaoi_world_info(self._w, C.byref(i)))
        return {k: getattr(i, k) for k, _ in Info._fields_}

    def debug_counters(self) -> dict:
        """Rare-path counters summed over flushes (gwaoi_debug_counters)."""
        d = Debug()
        self._check(self._L.gwaoi_debug_counters(self._w, C.byref(d)))
        return {k: getattr(d, k) for k, _ in Debug._fields_}

    def stage_times(self) -> dict:
        arr = (StageTime * 32)()
        n = C.c_size_t()
        self._check(self._L.gwaoi_stage_times(self._w, arr, 32, C.byref(n)))
        return {arr[i].name.decode(): (arr[i].ms, arr[i].calls) for i in range(min(n.value, 32))}

    def stage_names(self) -> list:
        arr = (StageTime * 32)()
        n = C.c_size_t()
        self._check(self._L.gwaoi_stage_times(self._w, arr, 32, C.byref(n)))
        return [arr[i].name.decode() for i in range(min(n.value, 32))]

    def set_stage_timing(self, stages=None):
        """Time the named stages with HIP events (None = all, [] = none)."""
        names = getattr(self, "_stage_names", None) or self.stage_names()
        self._stage_names = names
        mask = (1 << len(names)) - 1 if stages is None else sum(1 << names.index(s) for s in stages)
        self._check(self._L.gwaoi_set_stage_timing(self._w, mask))

    def reset_stage_times(self):
        self._check(self._L.gwaoi_reset_stage_times(self._w))

    def sync(self):
        self._check(self._L.gwaoi_sync(self._w))

    def stream(self) -> int:
        return self._L.gwaoi_stream(self._w) or 0

    def stream_after(self, other: int):
        """The world's stream runs what it is given next after everything queued on `other` (a hipStream_t)."""
        self._check(self._L.gwaoi_stream_after(self._w, C.c_void_p(other)))

    def stream_before(self, other: int):
        """`other` runs what it is given next after everything queued on the world's stream."""
        self._check(self._L.gwaoi_stream_before(self._w, C.c_void_p(other)))

    # ---- freeze / restore
    def snapshot(self) -> dict:
        """AOI state of the last flush in frame order: slot, space, x, z, seq arrays."""
        n = C.c_size_t()
        self._check(self._L.gwaoi_snapshot(self._w, None, None, None, None, None, 0, C.byref(n)))
        k = n.value
        out = {"slot": np.empty(k, np.uint32), "space": np.empty(k, np.uint32), "x": np.empty(k, np.float32),
               "z": np.empty(k, np.float32), "seq": np.empty(k, np.uint64)}
        if k:
            self._check(self._L.gwaoi_snapshot(self._w, _p(out["slot"]), _p(out["space"]), _p(out["x"]),
                                               _p(out["z"]), _p(out["seq"]), k, C.byref(n)))
        return out

    def restore(self, snap: dict):
        a = {k: np.ascontiguousarray(snap[k], t) for k, t in
             (("slot", np.uint32), ("space", np.uint32), ("x", np.float32), ("z", np.float32), ("seq", np.uint64))}
        self._check(self._L.gwaoi_restore(self._w, _p(a["slot"]), _p(a["space"]), _p(a["x"]), _p(a["z"]),
                                          _p(a["seq"]), a["slot"].size))

    # ---- entity position sync (include/gwaoi_sync.h)
    def entity_bind(self, slots, eids):
        """Bind slots to 16-byte entity ids: eids is (n,16) uint8 or a list of 16-byte bytes."""
        s = np.ascontiguousarray(np.atleast_1d(slots), np.uint32)
        e = _ids(eids, s.size)
        self._check(self._L.gwaoi_entity_bind_batch(self._w, _p(s), _p(e), s.size))

    def entity_unbind(self, slot):
        self._check(self._L.gwaoi_entity_unbind(self._w, slot))

    def entity_set_client(self, slot, gate_id=0, clientid=None):
        if clientid is None:
            self._check(self._L.gwaoi_entity_set_client(self._w, slot, 0, None))
        else:
            c = _ids([clientid], 1)
            self._check(self._L.gwaoi_entity_set_client(self._w, slot, gate_id, _p(c)))

    def entity_set_syncing(self, slot, syncing=True):
        self._check(self._L.gwaoi_entity_set_syncing(self._w, slot, 1 if syncing else 0))

    def entity_set_position_yaw(self, slot, x, y, z, yaw):
        self._check(self._L.gwaoi_entity_set_position_yaw(self._w, slot, C.c_float(x), C.c_float(y),
                                                          C.c_float(z), C.c_float(yaw)))

    def entity_enter_plain(self, slot, x, y, z):
        """Space.enter of a space without AOI (or an entity type without AOI)."""
        self._check(self._L.gwaoi_entity_enter_plain(self._w, slot, C.c_float(x), C.c_float(y), C.c_float(z)))

    def entity_leave_plain(self, slot):
        self._check(self._L.gwaoi_entity_leave_plain(self._w, slot))

    def set_position_yaw(self, slot, x, y, z, yaw):
        self._check(self._L.gwaoi_set_position_yaw(self._w, slot, C.c_float(x), C.c_float(y), C.c_float(z),
                                                   C.c_float(yaw)))

    def sync_from_clients(self, payload):
        """Decode a HandleSyncPositionYawFromClient payload (bytes / uint8 array, 32 B per record)."""
        b = np.frombuffer(bytes(payload), np.uint8) if not isinstance(payload, np.ndarray) else \
            np.ascontiguousarray(payload, np.uint8).reshape(-1)
        if b.size % 32:
            raise ValueError("payload is not a whole number of 32-byte records")
        self._check(self._L.gwaoi_sync_from_clients(self._w, _p(b), b.size // 32))

    def sync_from_clients_device(self, d_payload: int, n_rec: int):
        self._check(self._L.gwaoi_sync_from_clients_device(self._w, C.c_void_p(d_payload), n_rec))

    def collect_sync_infos(self) -> dict:
        """CollectEntitySyncInfos: {gate_id: (n,48) uint8 records}."""
        g = GateRecords()
        self._check(self._L.gwaoi_collect_sync_infos(self._w, C.byref(g)))
        return _gate_dict(g, SYNC_OUT_REC)

    def collect_sync_infos_device(self):
        """Records stay in HBM: (gate_ids, offsets (records), device pointer)."""
        g = GateRecords()
        self._check(self._L.gwaoi_collect_sync_infos_device(self._w, C.byref(g)))
        ids = [g.gate_ids[i] for i in range(g.n_gates)]
        off = [g.offsets[i] for i in range(g.n_gates + 1)] if g.n_gates else [0]
        return ids, off, g.records or 0

    def collect_client_events(self):
        """Events routed to clients: ({gate: (n,48) create records}, {gate: (n,32) destroy records})."""
        c, d = GateRecords(), GateRecords()
        self._check(self._L.gwaoi_collect_client_events(self._w, C.byref(c), C.byref(d)))
        return _gate_dict(c, SYNC_OUT_REC), _gate_dict(d, DESTROY_REC)


def _ids(ids, n) -> np.ndarray:
    if isinstance(ids, np.ndarray):
        a = np.ascontiguousarray(ids, np.uint8).reshape(-1, 16)
    else:
        a = np.frombuffer(b"".join(bytes(i) for i in ids), np.uint8).reshape(-1, 16)
    if a.shape[0] != n:
        raise ValueError(f"expected {n} ids of 16 bytes")
    return np.ascontiguousarray(a)


def _gate_dict(g: GateRecords, rec: int) -> dict:
    out = {}
    if not g.n_gates:
        return out
    total = g.offsets[g.n_gates]
    buf = np.ctypeslib.as_array(C.cast(g.records, C.POINTER(C.c_uint8)), shape=(total * rec,)).copy() \
        if total else np.empty(0, np.uint8)
    for i in range(g.n_gates):
        a, b = g.offsets[i], g.offsets[i + 1]
        out[g.gate_ids[i]] = buf[a * rec:b * rec].reshape(-1, rec)
    return out


def pair_keys(pairs: np.ndarray) -> np.ndarray:
    """(n,2) uint32 pairs -> sorted uint64 keys a<<32|b."""
    if pairs.size == 0:
        return np.empty(0, np.uint64)
    k = (pairs[:, 0].astype(np.uint64) << np.uint64(32)) | pairs[:, 1].astype(np.uint64)
    return np.sort(k)


class Wire:
    """The position-sync wire regroups of a gate or a dispatcher on the GPU
    (include/gwaoi_wire.h): GateService.handleSyncPositionYawFromClient +
    tryFlushPendingSyncPackets, DispatcherService.handleSyncPositionYawFromClient
    + sendEntitySyncInfosToGames, GateService.handleSyncPositionYawOnClients.
    Each regroup returns ``{destination key: bytes}`` (host) in key order."""

    def __init__(self, device: int = 0):
        self._L = load()
        h = C.c_void_p()
        rc = self._L.gwaoi_wire_create(device, C.byref(h))
        if rc != 0:
            raise GwaoiError(rc, self._L.gwaoi_strerror(rc).decode())
        self._w = h

    def close(self):
        if getattr(self, "_w", None):
            self._L.gwaoi_wire_destroy(self._w)
            self._w = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        self.close()

    def _check(self, rc):
        if rc != 0:
            raise GwaoiError(rc, self._L.gwaoi_strerror(rc).decode() + " (" +
                             self._L.gwaoi_wire_last_error(self._w).decode() + ")")

    @staticmethod
    def _ids(ids) -> np.ndarray:
        a = np.ascontiguousarray(np.frombuffer(b"".join(ids), np.uint8) if isinstance(ids, (list, tuple))
                                 else np.asarray(ids, np.uint8))
        assert a.size % 16 == 0
        return a

    def set_entity_games(self, ids, games):
        a, g = self._ids(ids), np.ascontiguousarray(games, np.uint16)
        if a.size // 16 != g.size:
            raise ValueError(f"{a.size // 16} ids but {g.size} games")
        self._check(self._L.gwaoi_wire_set_entity_games(self._w, _p(a), _p(g), g.size))

    def remove_entities(self, ids):
        a = self._ids(ids)
        self._check(self._L.gwaoi_wire_remove_entities(self._w, _p(a), a.size // 16))

    def set_clients(self, ids, index):
        a, x = self._ids(ids), np.ascontiguousarray(index, np.uint32)
        if a.size // 16 != x.size:
            raise ValueError(f"{a.size // 16} ids but {x.size} client indices")
        self._check(self._L.gwaoi_wire_set_clients(self._w, _p(a), _p(x), x.size))

    def remove_clients(self, ids):
        a = self._ids(ids)
        self._check(self._L.gwaoi_wire_remove_clients(self._w, _p(a), a.size // 16))

    @staticmethod
    def _groups(g: WireGroups, on_device: bool):
        n = g.n_groups
        keys = np.ctypeslib.as_array(g.keys, shape=(n,)).copy() if n else np.empty(0, np.uint32)
        off = np.ctypeslib.as_array(g.offsets, shape=(n + 1,)).copy()
        if on_device:
            return keys, off, g.records, int(g.n_dropped)
        total = int(off[-1]) * g.rec_bytes
        buf = C.string_at(g.records, total) if total else b""
        return {int(k): buf[int(off[i]) * g.rec_bytes:int(off[i + 1]) * g.rec_bytes] for i, k in enumerate(keys)}, \
            int(g.n_dropped)

    def _call(self, fn, data, *extra, rec=32):
        buf = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else np.ascontiguousarray(data)
        assert buf.size % rec == 0
        g = WireGroups()
        self._check(fn(self._w, _p(buf) if buf.size else None, buf.size // rec, *extra, C.byref(g)))
        return self._groups(g, False)

    def gate_from_clients(self, records: bytes, n_dispatchers: int):
        return self._call(self._L.gwaoi_wire_gate_from_clients, records, n_dispatchers)

    def dispatcher_to_games(self, records: bytes):
        return self._call(self._L.gwaoi_wire_dispatcher_to_games, records)

    def gate_to_clients(self, records: bytes):
        return self._call(self._L.gwaoi_wire_gate_to_clients, records, rec=48)

    def _call_device(self, fn, d_ptr: int, n: int, *extra):
        g = WireGroups()
        self._check(fn(self._w, C.c_void_p(d_ptr) if n else None, n, *extra, C.byref(g)))
        return self._groups(g, True)

    def gate_from_clients_device(self, d_ptr: int, n: int, n_dispatchers: int):
        """(keys, offsets, device records pointer, n_dropped)."""
        return self._call_device(self._L.gwaoi_wire_gate_from_clients_device, d_ptr, n, n_dispatchers)

    def dispatcher_to_games_device(self, d_ptr: int, n: int):
        return self._call_device(self._L.gwaoi_wire_dispatcher_to_games_device, d_ptr, n)

    def gate_to_clients_device(self, d_ptr: int, n: int):
        return self._call_device(self._L.gwaoi_wire_gate_to_clients_device, d_ptr, n)
