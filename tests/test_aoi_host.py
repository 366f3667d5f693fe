"""Host logic of the AOIManager mirror (goworld_amd/aoi.py) on CPU, with a
stub in place of the GPU world: call-order batching, slot lifetime across
Leave/flush, callback replay order, and the misuse errors where go-aoi
panics."""
import numpy as np
import pytest

from goworld_amd import aoi as A


class StubWorld:
    def __init__(self, max_slots, max_spaces=1, device=-1, **kw):
        self.calls = []
        self.next_space = 0
        self.result = (np.empty((0, 2), np.uint32), np.empty((0, 2), np.uint32))

    def space_create(self, d):
        self.next_space += 1
        return self.next_space - 1

    def space_destroy(self, s):
        self.calls.append(("space_destroy", s))

    def enter_batch(self, sp, slots, x, z):
        self.calls.append(("enter", sp, slots.tolist(), x.tolist(), z.tolist()))

    def leave_batch(self, slots):
        self.calls.append(("leave", slots.tolist()))

    def moved_batch(self, slots, x, z):
        self.calls.append(("moved", slots.tolist(), x.tolist(), z.tolist()))

    def tick(self):
        self.calls.append(("tick",))
        return self.result

    def close(self):
        pass


@pytest.fixture
def world(monkeypatch):
    monkeypatch.setattr(A, "World", StubWorld)
    return A.AOIWorld(8, max_spaces=2)


class Rec:
    def __init__(self, log, name):
        self.log, self.name = log, name

    def on_enter_aoi(self, other):
        self.log.append(("enter", self.name, other.data))

    def on_leave_aoi(self, other):
        self.log.append(("leave", self.name, other.data))


def mk(log, name):
    a = A.AOI()
    A.init_aoi(a, 100.0, name, Rec(log, name))
    return a


def test_calls_are_batched_in_call_order(world):
    log = []
    m0 = world.new_xzlist_aoi_manager(100.0)
    m1 = world.new_xzlist_aoi_manager(50.0)
    a, b, c = mk(log, "a"), mk(log, "b"), mk(log, "c")
    m0.enter(a, 1, 2)
    m0.enter(b, 3, 4)
    m1.enter(c, 5, 6)  # other space: new run
    m0.moved(a, 7, 8)
    m0.moved(b, 9, 10)
    m0.leave(a)
    m1.moved(c, 11, 12)
    sa, sb, sc = a.slot, b.slot, c.slot
    world.flush()
    calls = world.world.calls
    assert calls[0] == ("enter", 0, [sa, sb], [1.0, 3.0], [2.0, 4.0])
    assert calls[1] == ("enter", 1, [sc], [5.0], [6.0])
    assert calls[2] == ("moved", [sa, sb], [7.0, 9.0], [8.0, 10.0])
    assert a.slot == -1  # left and flushed: slot released
    assert calls[3][0] == "leave" and calls[4][0] == "moved" and calls[5] == ("tick",)


def test_replay_leaves_then_enters_pairwise(world):
    log = []
    m = world.new_xzlist_aoi_manager(100.0)
    a, b, c = mk(log, "a"), mk(log, "b"), mk(log, "c")
    for e in (a, b, c):
        m.enter(e, 0, 0)
    sa, sb, sc = a.slot, b.slot, c.slot
    world.world.result = (np.array([[sa, sb], [sb, sa]], np.uint32), np.array([[sa, sc], [sc, sa]], np.uint32))
    assert world.flush() == (2, 2)
    assert log == [("leave", "a", "c"), ("leave", "c", "a"), ("enter", "a", "b"), ("enter", "b", "a")]


def test_slot_kept_until_flush_and_reused_after(world):
    log = []
    m = world.new_xzlist_aoi_manager(100.0)
    a = mk(log, "a")
    m.enter(a, 0, 0)
    s = a.slot
    m.leave(a)
    assert a.slot == s  # leave events of this flush still name it
    m.enter(a, 1, 1)  # re-enter before the flush keeps the slot
    assert a.slot == s
    world.flush()
    assert a.slot == s and world._by_slot[s] is a
    m.leave(a)
    world.flush()
    assert a.slot == -1 and world._by_slot[s] is None and s in world._free


def test_misuse_raises_like_reference_panics(world):
    log = []
    m0 = world.new_xzlist_aoi_manager(100.0)
    m1 = world.new_xzlist_aoi_manager(100.0)
    a = mk(log, "a")
    with pytest.raises(A.AOIError):
        m0.moved(a, 1, 1)  # never entered
    with pytest.raises(A.AOIError):
        m0.leave(a)
    m0.enter(a, 0, 0)
    with pytest.raises(A.AOIError):
        m0.enter(a, 0, 0)  # twice
    with pytest.raises(A.AOIError):
        m1.moved(a, 0, 0)  # wrong space
    with pytest.raises(A.AOIError):
        m0.moved(a, float("nan"), 0)
    with pytest.raises(A.AOIError):
        world.new_xzlist_aoi_manager(0.0)  # EnableAOI: d > 0 (Space.go:92)


def test_slot_exhaustion(world):
    log = []
    m = world.new_xzlist_aoi_manager(100.0)
    for i in range(8):
        m.enter(mk(log, str(i)), i, i)
    with pytest.raises(A.AOIError):
        m.enter(mk(log, "x"), 0, 0)


def test_entity_interest_symmetry_rules():
    e1, e2 = A.EntityInterest(1, 100.0), A.EntityInterest(2, 100.0)
    e1.on_enter_aoi(e2.aoi)
    e2.on_enter_aoi(e1.aoi)
    assert e1.interested_in == {e2} and e2.interested_by == {e1} and e1.interested_by == {e2}
    e1.on_leave_aoi(e2.aoi)
    e2.on_leave_aoi(e1.aoi)
    assert not (e1.interested_in or e1.interested_by or e2.interested_in or e2.interested_by)


def test_restore_and_snapshot_validate_without_a_gpu():
    """Null-argument paths of the freeze/restore ABI never touch the device."""
    from goworld_amd import _lib
    L = _lib.load()
    assert L.gwaoi_snapshot(None, None, None, None, None, None, 0, None) == -1
    assert L.gwaoi_restore(None, None, None, None, None, None, 0) == -1
