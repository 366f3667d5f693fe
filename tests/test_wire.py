"""Position-sync wire path between gate, dispatcher and game:
the GPU regroups of include/gwaoi_wire.h against the CPU restatement
oracle/wire.py (GateService.go:346-371, 398-425; DispatcherService.go:786-825).

CPU tests pin the restatement on hand-derived cases read off the Go source
(the reference holds no test or fixture for these handlers: parity for this
row is against the restatement).  GPU tests compare the
libgwaoi regroups with the restatement byte for byte, per destination.
"""
import struct

import numpy as np
import pytest

from oracle import wire as W


def _id(k: int) -> bytes:
    return struct.pack("<QQ", 0x1234_5678_0000_0000 + k, 0xABCD_0000_0000_0000 ^ (k * 0x9E3779B97F4A7C15 & (2**64 - 1)))


def _rec(eid: bytes, x=1.0, y=2.0, z=3.0, yaw=0.5) -> bytes:
    return eid + struct.pack("<4f", x, y, z, yaw)


# ---------------------------------------------------------------- CPU oracle --

def test_dispatcher_of_uses_last_two_id_bytes():
    eid = bytes(14) + bytes([0x01, 0x02])  # hash = 1*256 + 2 = 258
    assert W.dispatcher_of(eid, 1) == 1
    assert W.dispatcher_of(eid, 4) == 258 % 4 + 1 == 3
    assert W.dispatcher_of(eid, 300) == 259
    assert W.dispatcher_of(bytes(16), 7) == 1


def test_gate_from_clients_keeps_arrival_order_per_dispatcher():
    a, b, c = bytes(15) + b"\x00", bytes(15) + b"\x01", bytes(15) + b"\x02"
    pay = _rec(a, 1) + _rec(b, 2) + _rec(c, 3) + _rec(a, 4)
    out = W.gate_from_clients(pay, 2)
    assert out == {1: _rec(a, 1) + _rec(c, 3) + _rec(a, 4), 2: _rec(b, 2)}
    assert W.gate_from_clients(b"", 3) == {}


def test_dispatcher_drops_entities_without_dispatch_info():
    e1, e2, e3 = _id(1), _id(2), _id(3)
    pay = _rec(e1, 1) + _rec(e3, 2) + _rec(e2, 3) + _rec(e1, 4)
    out = W.dispatcher_to_games(pay, {e1: 7, e2: 2})
    assert out == {7: _rec(e1, 1) + _rec(e1, 4), 2: _rec(e2, 3)}


def test_gate_to_clients_strips_client_id_and_drops_unknown_clients():
    c1, c2, c3 = _id(100), _id(101), _id(102)
    e1, e2 = _id(1), _id(2)
    pay = c1 + _rec(e1, 1) + c2 + _rec(e2, 2) + c3 + _rec(e1, 3) + c1 + _rec(e2, 4)
    out = W.gate_to_clients(pay, {c1: 10, c2: 11})
    assert out == {10: _rec(e1, 1) + _rec(e2, 4), 11: _rec(e2, 2)}


def test_wire_library_loads_and_rejects_null_handles():
    from goworld_amd import _lib
    L = _lib.load()
    assert L.gwaoi_wire_dispatcher_to_games(None, None, 0, None) == -1
    assert L.gwaoi_wire_remove_entities(None, None, 0) == -1


# ----------------------------------------------------------------- GPU parity --

def _d2h(ptr: int, nbytes: int) -> bytes:
    """Copy device memory to host through the HIP runtime this process already
    loaded (torch's copy, found by path: dlopen of the same file adds no second runtime)."""
    import ctypes
    path = next(line.split()[-1] for line in open("/proc/self/maps") if "libamdhip64.so" in line)
    hip = ctypes.CDLL(path)
    out = ctypes.create_string_buffer(max(nbytes, 1))
    assert hip.hipMemcpy(out, ctypes.c_void_p(ptr), ctypes.c_size_t(nbytes), 2) == 0  # hipMemcpyDeviceToHost
    return out.raw[:nbytes]


def _payload(rng, ids, n, prefix=None):
    pick = rng.integers(0, len(ids), n)
    vals = rng.standard_normal((n, 4)).astype(np.float32)
    parts = []
    for i in range(n):
        r = ids[pick[i]] + vals[i].tobytes()
        parts.append((prefix[i] if prefix is not None else b"") + r)
    return b"".join(parts)


@pytest.mark.gpu
def test_gpu_gate_from_clients_matches_oracle():
    from goworld_amd import Wire
    rng = np.random.default_rng(11)
    ids = [rng.bytes(16) for _ in range(5000)]
    pay = _payload(rng, ids, 60_000)
    with Wire(0) as w:
        for nd in (1, 3, 16, 1000):
            got, dropped = w.gate_from_clients(pay, nd)
            assert dropped == 0
            assert got == W.gate_from_clients(pay, nd), nd
        assert w.gate_from_clients(b"", 4) == ({}, 0)


@pytest.mark.gpu
def test_gpu_dispatcher_to_games_matches_oracle():
    from goworld_amd import Wire
    rng = np.random.default_rng(12)
    ids = [rng.bytes(16) for _ in range(6000)]
    games = {e: int(rng.integers(1, 40)) for e in ids[:5000]}  # 1000 entities have no dispatch info
    pay = _payload(rng, ids, 50_000)
    with Wire(0) as w:
        keys = list(games)
        w.set_entity_games(keys, [games[k] for k in keys])  # > 1024 ids: the table grows
        got, dropped = w.dispatcher_to_games(pay)
        want = W.dispatcher_to_games(pay, games)
        assert got == want
        assert dropped == 50_000 - sum(len(v) for v in want.values()) // 32 > 0
        # migrations and destroyed entities between ticks
        moved = keys[:700]
        for k in moved:
            games[k] = 99
        w.set_entity_games(moved, [99] * len(moved))
        gone = keys[700:1200]
        for k in gone:
            del games[k]
        w.remove_entities(gone)
        got, _ = w.dispatcher_to_games(pay)
        assert got == W.dispatcher_to_games(pay, games)


@pytest.mark.gpu
def test_gpu_gate_to_clients_matches_oracle_host_and_device():
    torch = pytest.importorskip("torch")
    from goworld_amd import Wire
    rng = np.random.default_rng(13)
    eids = [rng.bytes(16) for _ in range(3000)]
    cids = [rng.bytes(16) for _ in range(2500)]
    connected = {c: int(i) for i, c in zip(rng.permutation(100_000)[:2000], cids[:2000])}  # 500 disconnected
    n = 40_000
    pick = rng.integers(0, len(cids), n)
    pay = _payload(rng, eids, n, prefix=[cids[k] for k in pick])
    want = W.gate_to_clients(pay, connected)
    with Wire(0) as w:
        w.set_clients(list(connected), list(connected.values()))
        got, dropped = w.gate_to_clients(pay)
        assert got == want
        assert dropped == int(sum(1 for k in pick if cids[k] not in connected))
        # device-resident input (the game's collect output stays in HBM)
        d = torch.from_numpy(np.frombuffer(pay, np.uint8).copy()).to("cuda:0")
        torch.cuda.synchronize()
        keys, off, dptr, dropped2 = w.gate_to_clients_device(d.data_ptr(), n)
        assert dropped2 == dropped
        buf = _d2h(dptr, int(off[-1]) * 32)
        assert {int(k): buf[int(off[i]) * 32:int(off[i + 1]) * 32] for i, k in enumerate(keys)} == want
        # a client leaves: its records are dropped from then on
        gone = list(connected)[:100]
        w.remove_clients(gone)
        for c in gone:
            del connected[c]
        got, _ = w.gate_to_clients(pay)
        assert got == W.gate_to_clients(pay, connected)


@pytest.mark.gpu
def test_gpu_wire_error_paths():
    import ctypes
    from goworld_amd import GwaoiError, Wire
    from goworld_amd._lib import WireGroups
    with Wire(0) as w:
        with pytest.raises(GwaoiError):
            w.gate_from_clients(_rec(bytes(16)), 0)  # no dispatcher
        with pytest.raises(GwaoiError):
            w.set_clients([bytes(16)], [0xFFFFFFFE])  # reserved index
        g = WireGroups()
        L = w._L
        assert L.gwaoi_wire_gate_to_clients_device(w._w, ctypes.c_void_p(8), 1, ctypes.byref(g)) == -1  # misaligned
        assert L.gwaoi_wire_dispatcher_to_games(w._w, None, 3, ctypes.byref(g)) == -1  # records missing
        # an empty table drops everything; removing an unknown id is a no-op
        w.remove_entities([bytes(16)])
        got, dropped = w.dispatcher_to_games(_rec(_id(1)) * 5)
        assert got == {} and dropped == 5


def test_host_c_comparator_matches_restatement():
    """oracle/wire_host.c (bench.py's wire_leg CPU comparator) == the Python restatement."""
    from oracle import oracle
    rng = np.random.default_rng(5)
    n = 3000
    ids = rng.integers(0, 256, (400, 16), dtype=np.uint8)
    rec = np.concatenate([ids[rng.integers(0, 400, n)], rng.integers(0, 256, (n, 16), dtype=np.uint8)], axis=1)
    games = rng.integers(1, 9, 300).astype(np.uint32)  # the last 100 ids have no game: dropped
    clients = rng.integers(0, 256, (50, 16), dtype=np.uint8)
    cidx = rng.permutation(1000)[:40].astype(np.uint32)  # 10 clients not connected
    rec48 = np.concatenate([clients[rng.integers(0, 50, n)], rec], axis=1)
    H = oracle.WireHost(ids[:300], games, clients[:40], cidx)

    def as_dict(k, o, out):
        return {int(key): out[int(o[i]) * 32:int(o[i + 1]) * 32].tobytes() for i, key in enumerate(k)}

    assert as_dict(*H.gate_from_clients(rec, 5)) == W.gate_from_clients(rec.tobytes(), 5)
    game_of = {bytes(ids[i]): int(games[i]) for i in range(300)}
    assert as_dict(*H.dispatcher_to_games(rec)) == W.dispatcher_to_games(rec.tobytes(), game_of)
    connected = {bytes(clients[i]): int(cidx[i]) for i in range(40)}
    assert as_dict(*H.gate_to_clients(rec48)) == W.gate_to_clients(rec48.tobytes(), connected)
