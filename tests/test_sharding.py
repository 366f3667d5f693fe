"""Multi-rank path on CPU: space assignment, and a world_size-2 gloo run
where every rank evaluates only its own spaces (no data-path collective)
and the reduced counters equal the single-process totals."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from goworld_amd.shard import assign_spaces, reduce_over_ranks


def test_assign_spaces_contiguous_and_balanced():
    rng = np.random.default_rng(3)
    counts = rng.integers(100, 3000, 257)
    for ws in (1, 2, 3, 8):
        r = assign_spaces(counts, ws)
        assert r[0][0] == 0 and r[-1][1] == counts.size
        for a, b in zip(r, r[1:]):
            assert a[1] == b[0]
        loads = [counts[b:e].sum() for b, e in r]
        assert max(loads) - counts.sum() / ws <= counts.max()


def test_assign_spaces_edge_cases():
    assert assign_spaces([], 4) == [(0, 0)] * 4
    assert sum(e - b for b, e in assign_spaces([5], 3)) == 1
    r = assign_spaces([1, 1], 4)
    assert sum(e - b for b, e in r) == 2
    with pytest.raises(ValueError):
        assign_spaces([1], 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spaces(n_spaces, per, seed):
    from goworld_amd.workload import make_workload
    return make_workload("cfg4", seed=seed, n_spaces=n_spaces, per_space=per)


def _rank_events(lo, hi, wl, oracle):
    """Directed enter events of the first flush + of one tick, over spaces [lo, hi)."""
    slots, x0, z0, sp = wl.initial()
    sel = (sp >= lo) & (sp < hi)
    seq0 = np.zeros(wl.n, np.uint64)
    seq0[slots] = 1 + np.arange(wl.n, dtype=np.uint64)
    spv = np.where(sel, sp, oracle.DEAD).astype(np.uint32)
    D = {s: wl.D for s in range(wl.n_spaces)}
    before = oracle.closed_form_pairs(x0, z0, seq0, spv, D)
    sl, nx, nz = wl.tick(0)
    x1, z1 = x0.copy(), z0.copy()
    x1[sl], z1[sl] = nx, nz
    seq1 = seq0.copy()
    seq1[sl] = wl.n + 1 + np.arange(sl.size, dtype=np.uint64)
    after = oracle.closed_form_pairs(x1, z1, seq1, spv, D)
    ent = np.setdiff1d(after, before).size
    lev = np.setdiff1d(before, after).size
    return before.size, ent, lev


def _worker(rank, ws, port, n_spaces, per, seed, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    from oracle import oracle
    wl = _spaces(n_spaces, per, seed)
    lo, hi = assign_spaces([per] * n_spaces, ws)[rank]
    counts = _rank_events(lo, hi, wl, oracle)
    el, tot = reduce_over_ranks(dist, 0.5 + rank, counts, "cpu")
    if rank == 0:
        q.put((el, tot))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_space_sharding(oracle_mod):
    n_spaces, per, seed = 12, 300, 0x5EED0004
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_spaces, per, seed, q)) for r in range(2)]
    for p in procs:
        p.start()
    el, tot = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert el == 1.5  # MAX over ranks
    wl = _spaces(n_spaces, per, seed)
    ref = _rank_events(0, n_spaces, wl, oracle_mod)
    assert tot == [float(v) for v in ref] and ref[0] > 0 and ref[1] > 0
