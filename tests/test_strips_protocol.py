"""Strip tiling of one space (config 5) on CPU: the protocol and the exchange.

The strips' union of events must equal, tick by tick, the net events of one
unsplit sequential go-aoi manager (oracle/xzlist.c) fed the same global call
stream -- including teleports across strips, teleporting pairs that stay
neighbours, Leaves, Enters and entities parked on strip edges and halo
bounds.  Each strip is the numpy model of gwaoi_strips.hip (tests/strip_model.py)
over its own sequential manager; the world_size-2 case runs the real
torch.distributed exchange (goworld_amd.strips.exchange) over gloo.
Bit-exact sets, no tolerance.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from goworld_amd.strips import (HALO_WORDS, as_words, count_row, exchange, exchange_local, kinds_of, local_slice,
                                matrix_counts, matrix_kinds, merge_kinds, owner_of, row_words)
from strip_model import ModelShard
from strip_scenario import D, Scenario, split_by_owner


def reference_ticks(oracle, sc: Scenario, ticks: int):
    m = oracle.XZList(D, sc.max_slots)
    out = []
    for _ in range(ticks):
        kind, sl, nx, nz, seq, px = sc.tick()
        m.apply(kind.astype(np.uint8), sl.astype(np.int32), nx, nz)
        out.append(oracle.net_events(*m.take_events()))
    return out


def run_strips_local(oracle, sc: Scenario, ticks: int):
    S = sc.edges.size + 1
    shards = [ModelShard(sc.max_slots, D, sc.edges, r, oracle) for r in range(S)]
    out = []
    for _ in range(ticks):
        per = split_by_owner(*sc.tick(), sc.edges)
        routed = [sh.route(as_words(o, HALO_WORDS)) for sh, o in zip(shards, per)]
        for q, (sh, (recv, tele, k)) in enumerate(zip(shards, exchange_local(routed, [s.kinds for s in shards]))):
            sh.finish(local_slice(routed[q][0], routed[q][1], q), recv, tele, kinds=k)
        out.append(tuple(np.concatenate([sh.last[i] for sh in shards]) for i in (0, 1)))
    return out


def assert_same(got, ref):
    for t, ((ge, gl), (re_, rl)) in enumerate(zip(got, ref)):
        assert np.unique(ge).size == ge.size and np.unique(gl).size == gl.size, f"tick {t}: duplicate events"
        assert np.array_equal(np.sort(ge), re_), f"tick {t}: enter events differ"
        assert np.array_equal(np.sort(gl), rl), f"tick {t}: leave events differ"


@pytest.mark.parametrize("n_strips,seed", [(2, 11), (4, 7)])
def test_strip_protocol_loopback_matches_one_manager(oracle_mod, n_strips, seed):
    ticks = 5
    ref = reference_ticks(oracle_mod, Scenario(n0=4000, n_strips=n_strips, seed=seed), ticks)
    got = run_strips_local(oracle_mod, Scenario(n0=4000, n_strips=n_strips, seed=seed), ticks)
    assert_same(got, ref)
    assert sum(e.size for e, _ in ref[1:]) > 0 and sum(l.size for _, l in ref[1:]) > 0


def test_scenario_exercises_strip_hazards():
    sc = Scenario(n0=4000, n_strips=4, seed=7)
    sc.tick()
    kind, sl, nx, nz, seq, px = sc.tick()
    own_b = owner_of(np.nan_to_num(px), sc.edges)
    own_a = owner_of(nx, sc.edges)
    moved = kind == 0
    assert np.any(moved & (own_a != own_b))  # ownership changes (migration)
    assert np.sum(moved & (np.abs(nx - px) > 12.5)) >= 20  # teleporters
    assert np.any(kind == 1) and np.any(kind == 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, seed, ticks, q, rows=False):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    from oracle import oracle
    sc = Scenario(n0=3000, n_strips=ws, seed=seed)
    sh = ModelShard(sc.max_slots, D, sc.edges, rank, oracle)
    res = []
    for _ in range(ticks):
        ops = split_by_owner(*sc.tick(), sc.edges)[rank]
        send, counts, tele = sh.route(as_words(ops, HALO_WORDS))
        M = None
        if rows:  # the device count rows (k_route_row's layout), gathered as StripShard.route(ops, dist) does
            row = torch.from_numpy(count_row(counts, int(tele.shape[0]), sh.kinds).view(np.int32))
            W = row.numel()
            mat = torch.zeros(ws * W, dtype=torch.int32)
            dist.all_gather([mat[r * W:(r + 1) * W] for r in range(ws)], row)
            M = mat.numpy().view(np.uint32).reshape(ws, W)
        recv, tele_all, kinds = exchange(dist, send, counts, tele, kinds=sh.kinds, matrix=M)
        sh.finish(local_slice(send, counts, rank), recv, tele_all, kinds=kinds)
        res.append((sh.last[0].tolist(), sh.last[1].tolist()))
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("ws,rows", [(2, False), (3, False), (2, True), (3, True), (8, True)])
def test_gloo_strip_exchange(oracle_mod, ws, rows):
    """ws ranks over gloo: counts (with the ENTER / LEAVE statistics the receivers
    queue their world batches with) all-gathered -- as host rows, or (rows) as the
    device count rows the RCCL path gathers inside the route -- records point to
    point (3 ranks: the middle strip talks to both neighbours, the outer ones
    reach each other only through teleports; 8 ranks: config 5's strip count)."""
    seed, ticks = 5, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, seed, ticks, q, rows)) for r in range(ws)]
    for p in procs:
        p.start()
    parts = dict(q.get(timeout=300) for _ in range(ws))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = [tuple(np.array(sum((parts[r][t][i] for r in range(ws)), []), np.uint64) for i in (0, 1))
           for t in range(ticks)]
    ref = reference_ticks(oracle_mod, Scenario(n0=3000, n_strips=ws, seed=seed), ticks)
    assert_same(got, ref)


def test_count_row_round_trip():
    """The device count row (k_route_row's layout, written by the host model here) parses back to
    the same counts and the same receiver statistics as the host row (merge_kinds)."""
    rng = np.random.default_rng(3)
    S = 5
    sends = []
    for src in range(S):
        counts = rng.integers(0, 40, S)
        n = int(counts.sum())
        rec = np.zeros(n, dtype=np.dtype([("slot", "<u4"), ("x", "<f4"), ("z", "<f4"), ("kind", "<u4"),
                                          ("seq", "<u8")]))
        rec["kind"] = rng.integers(0, 3, n)
        rec["x"] = rng.normal(0, 1e4, n).astype(np.float32)
        rec["z"] = rng.normal(0, 1e4, n).astype(np.float32)
        sends.append((rec, counts, int(rng.integers(0, 9))))
    M = np.stack([count_row(c, t, kinds_of(r, c)) for r, c, t in sends])
    assert M.shape == (S, row_words(S))
    assert np.array_equal(matrix_counts(M, S)[:, :S], np.stack([c for _, c, _ in sends]))
    assert np.array_equal(matrix_counts(M, S)[:, S], [t for _, _, t in sends])
    for rank in range(S):
        want = merge_kinds([tuple(k[rank] for k in kinds_of(r, c)) for r, c, _ in sends])
        got = matrix_kinds(M, S, rank)
        assert got[0] == want[0] and got[1] == want[1]
        assert (got[2] is None) == (want[2] is None)
        if want[2] is not None:
            assert np.array_equal(got[2], want[2])


def test_device_workload_strip_ops_one_sync():
    """DeviceUniformWorkload.strip_ops (one host sync for every tick's ops, the owned records
    first by a stable sort) gives exactly the records of the per-tick selection by nonzero it
    replaced, on the CPU device: Enter ops of the starting strip, then each tick's Moved ops of
    the entities the strip owns before the tick, slots ascending, seqs in global call order."""
    import torch
    from goworld_amd.strips import even_edges
    from goworld_amd.workload import DeviceUniformWorkload
    n, ticks, ws = 5000, 3, 3
    for rank in range(ws):
        wl = DeviceUniformWorkload(n, 77, "cpu")
        edges_t = torch.from_numpy(even_edges(ws, -wl.L / 2, wl.L / 2))
        got = wl.strip_ops(edges_t, rank, ticks)
        ref = DeviceUniformWorkload(n, 77, "cpu")
        own = ref.owner(ref.x, edges_t) == rank
        slots = torch.nonzero(own).flatten()
        want = [ref._records(slots, ref.x[slots], ref.z[slots], 1, 1 + slots.to(torch.int64))]
        seq_next = n + 1
        for t in range(ticks):
            g = torch.Generator(device="cpu")
            g.manual_seed((77 * 1000003 + t) & 0x7FFFFFFFFFFFFFFF)
            sx = (2 * torch.rand(n, generator=g, dtype=torch.float64) - 1).to(torch.float32)
            sz = (2 * torch.rand(n, generator=g, dtype=torch.float64) - 1).to(torch.float32)
            order = torch.randperm(n, generator=g)
            pos = torch.empty_like(order)
            pos[order] = torch.arange(n)
            own = ref.owner(ref.x, edges_t) == rank
            nx, nz = ref.x + sx, ref.z + sz
            slots = torch.nonzero(own).flatten()
            want.append(ref._records(slots, nx[slots], nz[slots], 0, seq_next + pos[slots]))
            ref.x, ref.z = nx, nz
            seq_next += n
        assert len(got) == len(want) == ticks + 1
        for a, b in zip(got, want):
            assert torch.equal(a, b)


def test_host_workload_strip_ops_partition():
    """HostUniformWorkload.strip_ops (the gloo rehearsal's host-generated config-5 inputs): over
    all ranks, every tick's records cover each entity exactly once, owned by the strip its
    position lay in before the tick, with the tick's seqs a permutation of one block of n (the
    global call order); the first batch is the Enter of every entity (seq 1 + slot)."""
    from goworld_amd.strips import even_edges
    from goworld_amd.workload import HostUniformWorkload
    n, ticks, ws = 3000, 3, 4
    per_rank = []
    for rank in range(ws):
        wl = HostUniformWorkload(n, 99)
        per_rank.append(wl.strip_ops(even_edges(ws, -wl.L / 2, wl.L / 2), rank, ticks))
    ref = HostUniformWorkload(n, 99)
    edges = even_edges(ws, -ref.L / 2, ref.L / 2).astype(np.float32)
    for t in range(ticks + 1):
        recs = np.concatenate([per_rank[r][t] for r in range(ws)])
        assert np.array_equal(np.sort(recs[:, 0]), np.arange(n))
        seq = recs[:, 4].view(np.uint32).astype(np.int64) | (recs[:, 5].astype(np.int64) << 32)
        if t == 0:
            assert (recs[:, 3] == 1).all() and np.array_equal(np.sort(seq), 1 + np.arange(n))
        else:
            assert (recs[:, 3] == 0).all()
            assert np.array_equal(np.sort(seq), n + 1 + (t - 1) * n + np.arange(n))
        if t:  # ownership by the position before the tick (the previous batch's x)
            own_x = np.concatenate([per_rank[r][t - 1] for r in range(ws)])
            xs = np.empty(n, np.float32)
            xs[own_x[:, 0]] = own_x[:, 1].view(np.float32)
            for r in range(ws):
                sl = per_rank[r][t][:, 0]
                assert (np.searchsorted(edges, xs[sl], side="right") == r).all()
