#!/usr/bin/env python3
"""AOI tick benchmark (BASELINE.json metric) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg3]

A step is one AOI flush (gwaoi_tick_device): one batch of Moved calls --
every entity of the space moves once, in a seeded random call order -- then
the GPU pipeline computes the new neighbour relation and compacts the net
enter/leave events into device memory.  The move batches are generated on the
host before timing and uploaded to HBM (inputs resident when the timed region
starts).  At N=1 the workload is config 3 (1M entities, 256 Gaussian crowd
hotspots + uniform background, AOI distance 100, step U(-1,1)) -- the config
BASELINE.json quotes the metric on.  With N>1 ranks (torch.distributed.run,
RCCL) every rank owns its own independent space of the same size (GoWorld
spaces are independent, Space.go:33): weak scaling, no data-path collective.

Printed: one JSON line with value = entity-moves/s over all ranks, plus
events/s, p50/p99 tick latency, the roofline of the dominant kernel (HIP
events on the world's stream) and the CPU baseline (the go-aoi restatement in
oracle/, one core, on a bounded sample of the same workload).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

T_START = time.perf_counter()  # the process's start, for the child job's phase clock
METRIC = "AOI entity-moves/sec + enter/leave events/sec at 1M entities; p99 tick ms"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)

WORKLOAD_DESC = {
    "cfg1": "test_game-style single space, 1k entities random walk (bot walk, p=0.5)",
    "cfg2": "one space, 100k entities uniform, step U(-1,1)",
    "cfg3": "one space, 1M entities clustered crowd hotspots (256 x sigma 250 + uniform), step U(-1,1)",
    "cfg4": "8192 spaces x 2k entities (per rank: spaces / n_gpus), step U(-1,1)",
    "cfg5": "single 2^24-entity world uniform (L=sqrt(N*1250)), step U(-1,1), tiled into one x-strip per rank "
            "with halo exchange over RCCL",
}


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_plan(gpus: int, env) -> list | None:
    """How `bench.py --gpus N` runs.  None: this process is the whole job (N=1, or
    a rank started by torch.distributed.run with WORLD_SIZE == N).  A list: the
    environments of the N rank processes to spawn (WORLD_SIZE unset, N > 1), one
    per GPU, rendezvous on 127.0.0.1.  Raises ValueError when an outside
    launcher's WORLD_SIZE disagrees with --gpus."""
    if gpus < 1:
        raise ValueError(f"--gpus {gpus}: need at least one GPU")
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            raise ValueError(f"--gpus {gpus} but WORLD_SIZE={ws} (the launcher started {ws} ranks)")
        return None
    if gpus == 1:
        return None
    port = str(_free_port())
    plan = []
    for r in range(gpus):
        e = dict(env)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(gpus), LOCAL_WORLD_SIZE=str(gpus),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        plan.append(e)
    return plan


def spawn_ranks(plan) -> int:
    """Run the rank processes of `plan` (children of this process, which has not
    touched the GPU) and return the job's exit code: the first failing rank's,
    else 0.  Rank 0 prints the JSON line."""
    import subprocess
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=e) for e in plan]
    codes = [p.wait() for p in procs]
    bad = [c for c in codes if c != 0]
    return bad[0] if bad else 0


def combined_pass_bytes(n: int, total_cells: int, events: float) -> float:
    """Algorithmic HBM bytes of one k_combined launch (Roofline):
    every frame entry once as the tile's own entity -- new record (x, z, seq:
    16 B) + previous-flush record (16 B) -- the cell_start index (4 B per
    cell) and one (slot, slot) pair of 8 B per directed event (`events` is
    the directed count).  Candidate re-reads of neighbouring rows are L2/LDS
    reuse, not algorithmic traffic."""
    return n * 32.0 + (total_cells + 1) * 4.0 + 8.0 * events


# the kernels behind each timed stage (the roofline's "kernel")
STAGE_KERNEL = {"apply": "k_moves_apply+k_moves_fixup", "keygen": "k_keygen",
                "sort": "k_scan64_agg+k_scan64+k_arrive+k_cell_merge", "gather": "k_gather",
                "combined": "k_combined", "finish": "k_finish"}


def stage_bytes(n: int, moves: float, cells: int, events: float) -> dict:
    """Algorithmic HBM bytes per flush of each pipeline stage:
    the bytes a stage must move at least, at its own data layout.
      apply    move (slot, x, z) 12 B read, slot rank 4 B read, claim 8 B and
               record 16 B written: 40 B per move
      keygen   S' record + slot/space 24 B and the previous key 4 B read, key
               4 B written per entity; per-cell entity/arrival counts 8 B
      sort     (incremental merge) counts 8 B/cell read, cell_start 4 B/cell
               written, previous cell_start 4 B/cell and keys 4 B/entity read,
               permutation + sorted key 8 B/entity written
      gather   permutation 4 B, S' 24 B, previous frame 24 B read; frame 24 B,
               previous-in-new-order 16 B, candidate 16 B, slot rank 8 B, key
               4 B written: 120 B per entity
      combined see combined_pass_bytes
      finish   each directed event pair (8 B) read and written once
    """
    return {"apply": 40.0 * moves, "keygen": 32.0 * n + 8.0 * cells, "sort": 12.0 * n + 16.0 * cells,
            "gather": 120.0 * n, "combined": combined_pass_bytes(n, cells, events), "finish": 16.0 * events}


def pmc_file():
    """the latest round's committed k_combined PMC summary (profiles/rNN_pmc_k_combined.json)"""
    import glob
    fs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_pmc_k_combined.json")))
    return fs[-1] if fs else None


def pmc_traffic(workload: str):
    """Bytes per k_combined launch from the committed PMC passes (L2 -> fabric reads by request size, or
    2 x FETCH_SIZE without that pass; + WRITE_SIZE), if one matches."""
    try:
        d = json.load(open(pmc_file()))
    except (OSError, ValueError, TypeError):
        return None
    if d.get("workload") != workload:
        return None
    return d.get("hbm_bytes_per_launch")


SYNC_REC = np.dtype([("id", "V16"), ("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("yaw", "<f4")])


def entity_ids(slots: np.ndarray) -> np.ndarray:
    """16-byte entity ids (common.ENTITYID_LENGTH) for slots: b"E" + 15 decimal digits."""
    ids = np.char.add(b"E", np.char.zfill(slots.astype(np.int64).astype("S15"), 15))
    return np.frombuffer(ids.astype("S16").tobytes(), np.uint8).reshape(-1, 16)


def sync_leg(w, n: int, batches, client_frac: float):
    """The per-tick position-sync path around the AOI flush (include/gwaoi_sync.h):
    HandleSyncPositionYawFromClient packets (32-B records, every entity once, seeded
    order) already in HBM -> GPU decode into the move batch -> flush ->
    CollectEntitySyncInfos fan-out into per-gate 48-B records left in HBM.
    Entities 0..n-1 get ids; a `client_frac` share has a client on one of 8 gates."""
    import torch
    slots = np.arange(n, dtype=np.uint32)
    w.entity_bind(slots, entity_ids(slots))
    rng = np.random.default_rng(0x5EED5C)
    has_client = rng.random(n) < client_frac
    for s in np.nonzero(has_client)[0]:
        w.entity_set_client(int(s), 1 + int(s) % 8, b"C" + b"%015d" % int(s))
    for s in range(n):
        w.entity_set_syncing(s, True)
    pays = []
    for sl, nx, nz in batches:
        r = np.zeros(sl.size, SYNC_REC)
        r["id"] = entity_ids(sl).view("V16").reshape(-1)
        r["x"], r["z"] = nx, nz
        r["y"] = 1.0
        r["yaw"] = rng.uniform(-3.1, 3.1, sl.size).astype(np.float32)
        pays.append(torch.from_numpy(r.view(np.uint8).copy()).to(f"cuda:{torch.cuda.current_device()}"))
    torch.cuda.synchronize()
    # first packet + flush + collect untimed (clears the flags that entity binding left)
    w.sync_from_clients_device(pays[0].data_ptr(), batches[0][0].size)
    w.tick_device()
    w.collect_sync_infos_device()
    w.sync()
    t_tick = t_col = 0.0
    recs = moves = 0
    for k in range(1, len(pays)):
        a = time.perf_counter()
        w.sync_from_clients_device(pays[k].data_ptr(), batches[k][0].size)
        w.tick_device()
        w.sync()
        b = time.perf_counter()
        ids, off, _ = w.collect_sync_infos_device()
        w.sync()
        c = time.perf_counter()
        t_tick += b - a
        t_col += c - b
        recs += off[-1]
        moves += batches[k][0].size
    k = max(1, len(pays) - 1)
    return {"steps": k, "clients": int(has_client.sum()), "gates": 8,
            "decode_flush_ms": t_tick / k * 1e3, "moves_per_s": moves / t_tick,
            "collect_ms": t_col / k * 1e3, "records_per_tick": recs / k,
            "records_per_s": recs / t_col, "record_write_GBps": recs * 48 / t_col / 1e9,
            "note": "client packets decoded on the GPU (hash lookup of 16-B ids), flush, then "
                    "CollectEntitySyncInfos into per-gate 48-B records in HBM; wall clock per phase"}


def wire_leg(steps: int, n_rec: int, n_out_rec: int, device: int):
    """The gate / dispatcher position-sync regroups (include/gwaoi_wire.h) on the GPU
    beside the host C regroup of the same records (oracle/wire_host.c, one thread --
    the reference appends records to per-destination packets on one goroutine):
      gate_from_clients   n_rec 32-B client records -> 8 dispatchers (GateService.go:398-425)
      dispatcher_to_games n_rec 32-B records, n_rec entities in the table -> 8 games
                          (DispatcherService.go:786-825)
      gate_to_clients     n_out_rec 48-B records of one gate's share of a collect over
                          n_out_rec / 64 connected clients (GateService.go:346-371)
    GPU forms: host records in (pageable numpy: H2D + regroup + grouped records back in
    pinned host memory) and device-resident (records in HBM, groups left in HBM).
    Wall clock per call, median over `steps` after one warmup call."""
    import ctypes as C
    import torch
    from goworld_amd import Wire
    from goworld_amd._lib import WireGroups
    from oracle import oracle
    rng = np.random.default_rng(0x5EED57)
    slots = np.arange(n_rec, dtype=np.uint32)
    eids = entity_ids(slots)
    pos = rng.uniform(-1000, 1000, (n_rec, 4)).astype(np.float32)
    rec = np.ascontiguousarray(np.concatenate([eids[rng.permutation(n_rec)], pos.view(np.uint8)], axis=1))
    games = (1 + slots % 8).astype(np.uint16)
    n_cli = max(1, n_out_rec // 64)
    cids = np.frombuffer(b"".join(b"C%015d" % c for c in range(n_cli)), np.uint8).reshape(n_cli, 16)
    cidx = np.arange(n_cli, dtype=np.uint32)
    who = rng.integers(0, n_cli, n_out_rec)
    rec48 = np.ascontiguousarray(np.concatenate(
        [cids[who], eids[rng.integers(0, n_rec, n_out_rec)], rng.uniform(-1, 1, (n_out_rec, 4)).astype(np.float32)
         .view(np.uint8)], axis=1))
    dev = f"cuda:{device}"
    d_rec = torch.from_numpy(rec).to(dev)
    d_rec48 = torch.from_numpy(rec48).to(dev)
    torch.cuda.synchronize()
    out = {}
    with Wire(device) as W:
        W.set_entity_games(eids, games)
        W.set_clients(cids, cidx)
        L = W._L
        H = oracle.WireHost(eids, games.astype(np.uint32), cids, cidx)
        legs = {
            "gate_from_clients": (n_rec, 32, lambda g: L.gwaoi_wire_gate_from_clients(W._w, _ptr(rec), n_rec, 8, g),
                                  lambda g: L.gwaoi_wire_gate_from_clients_device(W._w, C.c_void_p(d_rec.data_ptr()),
                                                                                  n_rec, 8, g),
                                  lambda: H.gate_from_clients(rec, 8)),
            "dispatcher_to_games": (n_rec, 32, lambda g: L.gwaoi_wire_dispatcher_to_games(W._w, _ptr(rec), n_rec, g),
                                    lambda g: L.gwaoi_wire_dispatcher_to_games_device(
                                        W._w, C.c_void_p(d_rec.data_ptr()), n_rec, g),
                                    lambda: H.dispatcher_to_games(rec)),
            "gate_to_clients": (n_out_rec, 48, lambda g: L.gwaoi_wire_gate_to_clients(W._w, _ptr(rec48), n_out_rec, g),
                                lambda g: L.gwaoi_wire_gate_to_clients_device(W._w, C.c_void_p(d_rec48.data_ptr()),
                                                                              n_out_rec, g),
                                lambda: H.gate_to_clients(rec48)),
        }
        for name, (n, rb, host_fn, dev_fn, cpu_fn) in legs.items():
            res = {"records": n, "record_bytes": rb}
            for form, fn in (("gpu_host_records", host_fn), ("gpu_device_records", dev_fn)):
                g = WireGroups()
                ts = []
                for k in range(steps + 1):
                    a = time.perf_counter()
                    rc = fn(C.byref(g))
                    if rc:
                        raise RuntimeError(f"wire {name}: rc {rc}")
                    if form == "gpu_device_records":
                        torch.cuda.synchronize()
                    if k:
                        ts.append(time.perf_counter() - a)
                t = float(np.median(ts))
                res[form] = {"ms": round(t * 1e3, 4), "records_per_s": n / t, "groups": int(g.n_groups)}
            ts = []
            for k in range(max(2, steps // 2)):
                a = time.perf_counter()
                cpu_fn()
                ts.append(time.perf_counter() - a)
            t = float(np.median(ts))
            res["cpu_host_c_1thread"] = {"ms": round(t * 1e3, 3), "records_per_s": n / t}
            res["gpu_device_vs_cpu"] = round(t / (res["gpu_device_records"]["ms"] * 1e-3), 2)
            res["gpu_host_vs_cpu"] = round(t / (res["gpu_host_records"]["ms"] * 1e-3), 2)
            out[name] = res
    out["note"] = ("wall clock per call (median); gpu_host_records = pageable host records in, grouped records in "
                   "pinned host memory out (PCIe both ways); gpu_device_records = records and groups in HBM; "
                   "cpu = oracle/wire_host.c, the reference's append-per-destination loop in C, one thread")
    return out


def _ptr(a):
    import ctypes as C
    return a.ctypes.data_as(C.c_void_p)


def cpu_core_counts() -> dict:
    """Host cores: the affinity mask's count, the cgroup CPU quota in cores (cgroup v2 cpu.max or
    v1 cfs quota / period; None when unlimited), and the number used = the smaller of the two.
    On the GPU box the affinity mask shows the whole machine while the quota is the box's share."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as fq, open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fp:
                q, per = int(fq.read()), int(fp.read())
                if q > 0:
                    quota = max(1, q // per)
        except (OSError, ValueError):
            pass
    used = max(1, min(aff, quota) if quota else aff)
    return {"affinity": aff, "cgroup_quota": quota, "used": used}


def cpu_cores() -> int:
    """Host cores the CPU comparators use: the affinity count, bounded by the cgroup quota."""
    return cpu_core_counts()["used"]


def cpu_baseline_spaces(args, target_s: float):
    """cfg4: independent 2000-entity spaces, one sequential XZ-list restatement
    per space, spaces run in parallel on all host cores (one thread per core;
    the C oracle runs with the GIL released).  Move batches are generated
    before timing."""
    import threading
    from goworld_amd.workload import make_workload
    from oracle import oracle
    cores = cpu_cores()
    work = []
    for k in range(cores):
        wl = make_workload("cfg4", seed=0x5EED0004 + 7919 * k, n_spaces=1)
        m = oracle.XZList(wl.D, wl.n, record=False)
        slots, x0, z0, _ = wl.initial()
        m.bulk_enter(slots.astype(np.int32), x0, z0)
        work.append((m, wl))
    done = [0] * cores
    stop = [False]

    def run(k):
        m, wl = work[k]
        t = 0
        while not stop[0]:
            sl, nx, nz = wl.tick(t)  # ~0.1 ms of numpy per ~10 ms of C (GIL released there)
            m.moved_batch(sl, nx, nz)
            done[k] += sl.size
            t += 1

    th = [threading.Thread(target=run, args=(k,)) for k in range(cores)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    timer = threading.Timer(target_s, lambda: stop.__setitem__(0, True))
    timer.start()
    for x in th:
        x.join()
    timer.cancel()
    dt = time.perf_counter() - t0
    ev = sum(sum(w[0].counts()) for w in work)
    return {"value": sum(done) / dt, "unit": "entity-moves/s", "events_per_s": ev / dt, "cores": cores,
            "nproc": os.cpu_count(), "core_counts": cpu_core_counts(), "kind": "port",
            "sample": f"{cores} independent cfg4 spaces (2000 entities each), one per core, every entity "
                      f"moving each tick ({sum(done)} Moved calls), sequential XZ-list restatement, {dt:.1f} s"}


def cpu_grid_baseline(args, target_s: float):
    """CPU-grid comparator: the same tick on all host cores --
    every tick the relation of config 3 recomputed with a cell grid and diffed
    against the last (oracle/cpu_grid.c, OpenMP).  Untimed populate, then
    whole ticks until target_s."""
    from goworld_amd.workload import make_workload
    from oracle import oracle
    cores = cpu_cores()
    wl = make_workload("cfg3", n=args.n)
    g = oracle.CpuGrid(wl.x, wl.z, wl.D, cores)
    batches = [wl.tick(t) for t in range(3)]
    done, ev, t = 0, 0, 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < target_s or t == 0:
        sl, nx, nz = batches[t % len(batches)] if t < len(batches) else wl.tick(t)
        ne, nl = g.tick(sl, nx, nz)
        done += sl.size
        ev += ne + nl
        t += 1
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "entity-moves/s", "ms_per_tick": dt / t * 1e3, "events_per_s": ev / dt,
            "cores": cores, "core_counts": cpu_core_counts(), "kind": "port",
            "sample": f"{t} whole cfg3 ticks ({wl.n} entities, every entity moving), relation recomputed on a cell "
                      f"grid and diffed per tick on {cores} threads, {dt:.1f} s"}


def host_tick_bench(ticks: int, threads: int):
    """The C++ host tick (tools/tick_bench.cpp, built in-tree): cfg3 from host
    arrays through gwaoi_moved_batch to events in pinned host memory, serial and
    pipelined (gwaoi_tick_begin/_end), plus the callback replay into per-entity
    InterestedIn / InterestedBy sets (Entity.go:236-246) on 1 and T threads."""
    import subprocess
    exe = os.path.join(ROOT, "goworld_amd", "lib", "gwaoi_tick_bench")
    if not os.path.exists(exe):
        return {"error": "gwaoi_tick_bench not built"}
    r = subprocess.run([exe, str(ticks), str(threads)], capture_output=True, text=True, timeout=300)
    try:
        return json.loads(r.stdout.strip().splitlines()[-1])
    except Exception:
        return {"error": (r.stderr or r.stdout)[-500:]}


class _Filler:
    """The caller side of the zero-copy batch: the tick's (slot, x, z) arrays written into the
    world's pinned staging views by 8 threads (numpy copies release the GIL), as a cgo adapter
    would append the moves it decodes."""

    def __init__(self, threads: int = 8):
        from concurrent.futures import ThreadPoolExecutor
        self.T = threads
        self.pool = ThreadPoolExecutor(threads)

    def fill(self, views, batch):
        n = batch[0].size
        cuts = np.linspace(0, n, self.T + 1).astype(np.int64)

        def part(k):
            a, b = cuts[k], cuts[k + 1]
            for v, src in zip(views, batch):
                v[a:b] = src[a:b]
        list(self.pool.map(part, range(self.T)))

    def close(self):
        self.pool.shutdown()


def host_io_leg(w, host_batches, hio, dist, red_dev):
    """The host -> host tick (p50/p99 "end-to-end from H2D to event CSR in host
    memory"): host move arrays in, the events delivered to pinned host memory.

    pinned (the headline twin): each tick's moves sit in a pinned host buffer of the caller's
      (gwaoi_pinned_alloc; a cgo adapter fills it as the sync packets arrive over the game tick, so the
      batch is in host memory when the tick starts, as the bench's device leg has it in HBM), and
      gwaoi_moved_batch_pinned queues one H2D of it on a copy stream; the moves are checked on the device.
      Serial: batch + gwaoi_tick.  Pipelined: the batch of t+1 is queued while flush t runs (its H2D beside
      the copy-out of t-1's events), gwaoi_pairs_host takes t-1's events, then gwaoi_tick_finish(NEXT|PAIRS)
      queues flush t+1 before t's summary is read and starts t's copy-out (one event per mirrored pair)
      without waiting for it.  (Taking t's events right after that call instead: 0.364 vs 0.341 ms per
      tick, p99 latency 0.86 vs 0.87 ms, r04n / r04m.)
      Latency = the batch call -> its events in host memory.
    stage_commit: the caller writing the moves into the library's pinned staging (gwaoi_moved_batch_stage /
      _commit, 8 numpy threads here): the fill cost a caller pays per tick, and those ticks' latency.
    staged_copy_api (gwaoi_moved_batch: validation + copy into pinned staging on 8 library threads): the
      same ticks through the copying API, for comparison."""
    import gc
    import torch
    from goworld_amd.shard import reduce_over_ranks
    n_ser, n_pip = hio, hio + 1
    zc, rest = host_batches[:3 + n_ser + 2 * n_pip], host_batches[3 + n_ser + 2 * n_pip:]
    # the caller's pinned batch buffers, filled before timing (untimed, like the device leg's HBM batches)
    bufs = []
    for b in zc:
        ptr, views = w.pinned_batch(b[0].size)
        for v, src in zip(views, b):
            v[:] = src
        bufs.append((ptr, views, b[0].size))
    # warmup (sizes the device staging halves and host event buffers; the pipeline's fill)
    w.moved_batch_pinned(bufs[0][1], bufs[0][2]); w.tick(copy=False)
    w.moved_batch_pinned(bufs[1][1], bufs[1][2]); w.tick_begin()
    w.moved_batch_pinned(bufs[2][1], bufs[2][2]); w.tick_end_begin(copy=False)
    w.tick_end(copy=False)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    gc.disable()  # no collector pauses inside the timed ticks
    s_lat, h_ev = [], 0
    ser = bufs[3:3 + n_ser]
    s0 = time.perf_counter()
    for _, views, k in ser:
        a = time.perf_counter()
        w.moved_batch_pinned(views, k)
        ent, lev = w.tick(copy=False)
        s_lat.append(time.perf_counter() - a)
        h_ev += len(ent) + len(lev)
    s_el = time.perf_counter() - s0
    def pipelined(pb, pairs):
        lat, issue = [], []
        end_begin = w.tick_end_begin_pairs_async if pairs else w.tick_end_begin_async
        take = w.pairs_host if pairs else w.events_host
        t0 = time.perf_counter()
        issue.append(t0)
        w.moved_batch_pinned(pb[0][1], pb[0][2])
        w.tick_begin()
        for k in range(len(pb)):
            if k + 1 < len(pb):
                issue.append(time.perf_counter())
                w.moved_batch_pinned(pb[k + 1][1], pb[k + 1][2])  # batch t+1's H2D, queued while flush t runs
                end_begin()  # finish t, queue t+1, start t's copy-out
                take(copy=False)  # tick t's events in host memory (flush t+1 keeps the GPU busy meanwhile)
            else:
                w.tick_end(copy=False)
            lat.append(time.perf_counter() - issue[k])
        return time.perf_counter() - t0, lat

    pb = bufs[3 + n_ser:3 + n_ser + n_pip]
    d_el, d_lat = pipelined(pb, False)  # every directed event to host memory
    pb = bufs[3 + n_ser + n_pip:]
    p_el, p_lat = pipelined(pb, True)   # one event per mirrored pair: half the D2H bytes
    gc.enable()
    torch.cuda.synchronize()
    for ptr, _, _ in bufs:
        w.free_pinned_batch(ptr)
    # stage / commit: the caller's fill into the library's staging, and those ticks' latency from the commit
    F = _Filler()
    f_ms, c_lat = [], []
    for b in rest[:6]:
        t = time.perf_counter()
        F.fill(w.stage_moves(b[0].size), b)
        a = time.perf_counter()
        w.commit_moves(b[0].size)
        w.tick(copy=False)
        c_lat.append(time.perf_counter() - a)
        f_ms.append(a - t)
    F.close()
    # staged (copying API): the same measurement through gwaoi_moved_batch
    st = rest[6:]
    k = max(2, (len(st) - 1) // 2)
    w.moved_batch(*st[0]); w.tick(copy=False)
    g_lat = []
    for b in st[1:k + 1]:
        a = time.perf_counter()
        w.moved_batch(*b)
        w.tick(copy=False)
        g_lat.append(time.perf_counter() - a)
    cp = st[k + 1:2 * k + 1]
    cq_lat = []
    w.moved_batch(*cp[0])
    c0 = iss = time.perf_counter()
    for j in range(len(cp)):
        w.tick_begin()
        nxt = time.perf_counter()
        if j + 1 < len(cp):
            w.moved_batch(*cp[j + 1])
        w.tick_end(copy=False)
        cq_lat.append(time.perf_counter() - iss)
        iss = nxt
    c_el = time.perf_counter() - c0
    if dist is not None:
        dist.barrier()
    p_el, (h_moves, h_evs) = reduce_over_ranks(dist, p_el, [sum(b[2] for b in pb), h_ev], red_dev)
    d_el, _ = reduce_over_ranks(dist, d_el, [0.0], red_dev)
    pct = lambda v, q: float(np.percentile(np.array(v) * 1e3, q))
    FILL = 2  # the pipelined loops' first two ticks fill the pipeline (their H2Ds queue back to back)
    return {"value": h_moves / p_el, "unit": "entity-moves/s", "ms_per_step": p_el / len(pb) * 1e3,
            "p50_tick_ms": pct(p_lat[FILL:], 50), "p99_tick_ms": pct(p_lat[FILL:], 99), "steps": len(pb),
            "fill_ticks": FILL, "ticks_ms": [round(v * 1e3, 3) for v in p_lat],
            "directed_events_out": {"ms_per_step": d_el / n_pip * 1e3, "p50_tick_ms": pct(d_lat[FILL:], 50),
                                    "p99_tick_ms": pct(d_lat[FILL:], 99), "steps": n_pip},
            "serial": {"ms_per_step": s_el / len(ser) * 1e3, "p50_tick_ms": pct(s_lat, 50),
                       "p99_tick_ms": pct(s_lat, 99), "steps": len(ser), "events_per_s": h_evs / max(s_el, 1e-9)},
            "stage_commit": {"caller_fill_ms_p50": pct(f_ms, 50), "serial_p50_tick_ms": pct(c_lat, 50),
                             "steps": len(c_lat)},
            "staged_copy_api": {"serial_p50_tick_ms": pct(g_lat, 50), "serial_p99_tick_ms": pct(g_lat, 99),
                                "pipelined_ms_per_step": c_el / len(cp) * 1e3,
                                "pipelined_p99_tick_ms": pct(cq_lat[1:], 99), "steps": len(g_lat)},
            "note": "pinned: each tick's moves in a caller-owned pinned buffer (gwaoi_pinned_alloc, filled before "
                    "timing as a game server fills it while packets arrive), one H2D per tick, checked on the "
                    "device; pipelined = batch t+1 queued while flush t runs, then gwaoi_tick_finish(NEXT|PAIRS) "
                    "(flush t+1 queued before t's summary, t's copy-out started: one event per mirrored pair "
                    "(a,b)/(b,a), from which the callbacks of both entities follow), then t's pairs taken "
                    "(gwaoi_pairs_host) while flush t+1 runs; directed_events_out = the same ticks copying every "
                    "directed event (gwaoi_tick_finish(NEXT|HOST) + gwaoi_events_host).  Tick latency = batch call "
                    "-> events in pinned host memory; pipelined percentiles over the ticks after the first "
                    "fill_ticks (every tick's latency in ticks_ms; ms_per_step counts them all).  PCIe here carries one direction at a time "
                    "(tools/pcie_probe.py), so a pipelined tick costs H2D + D2H.  stage_commit = the caller "
                    "writing the moves into the library's staging per tick (its fill cost); staged_copy_api = "
                    "gwaoi_moved_batch"}


def line_summary(out: dict) -> dict:
    """The headline numbers of every leg, compact, at the end of the JSON line (a driver that keeps
    the tail of stdout keeps these)."""
    def g(d, *ks):
        for k in ks:
            if not isinstance(d, dict):
                return None
            d = d.get(k)
        return round(d, 4) if isinstance(d, float) else d
    cfg5 = out.get("cfg5_strips") or {}
    return {
        "ms_per_step": g(out, "ms_per_step"), "p99_tick_ms": g(out, "p99_tick_ms"),
        "claims_ms_per_step": g(out, "claims_tick", "ms_per_step"), "claims_p99_ms": g(out, "claims_tick", "p99_tick_ms"),
        "claims_counts_equal": g(out, "claims_tick", "counts_equal_headline"),
        "combined_ms": g(out, "roofline", "avg_launch_ms"), "roofline_frac": g(out, "roofline", "frac"),
        "host_to_host_tick_ms": g(out, "host_to_host_tick", "ms_per_step"),
        "host_to_host_p50_ms": g(out, "host_to_host_tick", "p50_tick_ms"),
        "host_to_host_p99_ms": g(out, "host_to_host_tick", "p99_tick_ms"),
        "host_to_host_serial_p99_ms": g(out, "host_to_host_tick", "serial_p99_tick_ms"),
        "host_tick_with_replay_ms": g(out, "host_tick", "pipelined", "ms_per_tick"),
        "host_tick_with_replay_p99_ms": g(out, "host_tick", "pipelined", "latency_ms_p99"),
        "small_flush_p50_ms": {k: g(v, "device", "p50_ms") for k, v in (out.get("small_flush") or {}).items()
                               if isinstance(v, dict)},
        "sync_decode_flush_ms": g(out, "sync_leg", "decode_flush_ms"), "sync_collect_ms": g(out, "sync_leg", "collect_ms"),
        "cfg4_ms_per_step": g(out, "cfg4_strong", "ms_per_step"),
        "cfg5_ms_per_step": g(cfg5, "ms_per_step"), "cfg5_error": cfg5.get("error"),
        "cfg5_job_wall_s": g(cfg5, "job", "wall_s"),
        "cpu_port_moves_per_s": g(out, "cpu_baseline", "value"),
        "cpu_grid_ms_per_tick": g(out, "cpu_baseline", "cpu_grid", "ms_per_tick"),
    }


def claims_leg(args, n, n_spaces, D, initial, device, row_ptrs, moves_per_tick, t0: int, t1: int, ref_counts):
    """The headline's ticks through the general AOIManager contract: a world WITHOUT
    GWAOI_F_UNIQUE_MOVES, so every flush stores the last-op claims and runs the repeated-slot fixup
    that go-aoi's Moved semantics need when a batch may name an entity twice (the gate appends every
    client sync record without deduplication, /root/reference/components/gate/GateService.go:398-405,
    and the game applies each in order, components/game/GameService.go:396-403).  Same initial state,
    same device batches, same speculative loop as the timed region: ticks t0 .. t1-1 after ticks
    0 .. t0-1 untimed.  Every tick's (enters, leaves) must equal the headline world's."""
    from goworld_amd import World
    slots, x0, z0, sp = initial
    w = World(n, max_spaces=n_spaces, device=device, cells_per_dist=args.cells_per_dist, unique_moves=False)
    try:
        spaces = [w.space_create(D) for _ in range(n_spaces)]
        for s in range(n_spaces):
            sel = np.nonzero(sp == s)[0] if n_spaces > 1 else slice(None)
            w.enter_batch(spaces[s], slots[sel], x0[sel], z0[sel])
        w.tick_device()
        counts = {}
        for t in range(t0):
            ps, px, pz = row_ptrs[t]
            w.moved_batch_device(ps, px, pz, moves_per_tick[t])
            counts[t] = w.tick_device()
        w.sync()
        lat = []
        a0 = time.perf_counter()
        ps, px, pz = row_ptrs[t0]
        w.moved_batch_device(ps, px, pz, moves_per_tick[t0])
        w.tick_begin()
        for t in range(t0, t1):
            a = time.perf_counter()
            if t + 1 < t1:
                ps, px, pz = row_ptrs[t + 1]
                w.moved_batch_device(ps, px, pz, moves_per_tick[t + 1])
                counts[t] = w.tick_end_begin_device()
            else:
                counts[t] = w.tick_end_device()
            lat.append(time.perf_counter() - a)
        w.sync()
        elapsed = time.perf_counter() - a0
        dbg = w.debug_counters()
    finally:
        w.close()
    k = t1 - t0
    lat_ms = np.array(lat) * 1e3
    bad = [t for t in ref_counts if counts.get(t) != ref_counts[t]]
    moves = sum(moves_per_tick[t0:t1])
    return {"value": moves / elapsed, "unit": "entity-moves/s", "steps": k, "ms_per_step": elapsed / k * 1e3,
            "p50_tick_ms": float(np.percentile(lat_ms, 50)), "p99_tick_ms": float(np.percentile(lat_ms, 99)),
            "unique_flushes": int(dbg["unique_flushes"]), "speculative_launches": int(dbg["speculative_launches"]),
            "counts_equal_headline": not bad, "ticks_compared": len(ref_counts), "mismatched_ticks": bad[:8],
            "note": "general contract (last-op claims + repeated-slot fixup: a batch may repeat an entity, the "
                    "last call wins); the headline's batches, initial state and speculative loop"}


def small_flush_leg(w, last, reps: int, sizes=(1, 64, 4096, 65536)):
    """What one flush of k Moved calls costs on the config-3 world (1M entities): the game
    loop's price for read-after-write interest sets (a flush after each timer callback that
    moves entities).  k random entities move U(-1,1) from their current
    positions; the wall clock runs from the host batch call to the flush's events in HBM
    (gwaoi_moved_batch + gwaoi_tick_device), and again with the events copied to host memory
    (gwaoi_tick).  Events are checked for nothing here (the parity tests do that)."""
    sl, x, z = (np.array(a) for a in last)
    rng = np.random.default_rng(0x5EEDF1)
    out = {}
    for k in sizes:
        res = {}
        for mode in ("device", "host"):
            ts, tq, evs, sparse0 = [], [], [], w.debug_counters().get("sparse_flushes", 0)
            for r in range(reps + 3):
                idx = rng.choice(sl.size, k, replace=False)
                x[idx] += rng.uniform(-1.0, 1.0, k).astype(np.float32)
                z[idx] += rng.uniform(-1.0, 1.0, k).astype(np.float32)
                bs, bx, bz = sl[idx], x[idx], z[idx]
                a = time.perf_counter()
                w.moved_batch(bs, bx, bz)
                b = time.perf_counter()
                if mode == "device":
                    ne, nl = w.tick_device()
                else:
                    e, l = w.tick()
                    ne, nl = len(e), len(l)
                if r >= 3:
                    ts.append(time.perf_counter() - a)
                    tq.append(b - a)
                    evs.append(ne + nl)
            t = np.array(ts) * 1e3
            q = np.array(tq) * 1e3
            res[mode] = {"p50_ms": round(float(np.percentile(t, 50)), 4), "p99_ms": round(float(np.percentile(t, 99)), 4),
                         "mean_ms": round(float(t.mean()), 4), "events_mean": float(np.mean(evs)),
                         "queue_p50_ms": round(float(np.percentile(q, 50)), 4),
                         "sparse_flushes": w.debug_counters().get("sparse_flushes", 0) - sparse0}
        out[str(k)] = res
    out["note"] = ("one flush of k Moved calls on the 1M-entity config-3 world, wall clock from the host batch call "
                   "to the events (device: in HBM; host: in host memory); reps per size after 3 untimed; "
                   "queue_p50_ms: the gwaoi_moved_batch call alone (host validation + staging + H2D issue)")
    return out


def cfg4_leg(args, ws, rank, device, dist, red_dev):
    """Config 4 as a strong-scaling sub-record of every line: 8192 independent
    spaces x 2000 entities in total, sharded over the ranks in contiguous
    blocks balanced by entity count (goworld_amd.shard.assign_spaces), one
    world per rank covering all of its spaces with one launch sequence.  Move
    batches (every entity, U(-1,1), random call order) are generated on the
    GPU before timing; value = all ranks' moves / max time over ranks."""
    import torch
    from goworld_amd import World
    from goworld_amd.shard import assign_spaces, reduce_over_ranks
    per, total = 2000, args.cfg4_spaces
    lo, hi = assign_spaces([per] * total, ws)[rank]
    ns = max(0, hi - lo)
    n = ns * per
    L = float(np.sqrt(per * 1250.0))
    dev = torch.device(f"cuda:{device}")
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED0004 + lo)
    t_setup = time.perf_counter()
    ticks = args.cfg4_warmup + args.cfg4_steps
    x = (torch.rand(n, generator=g, device=dev, dtype=torch.float64) * L - L / 2).to(torch.float32)
    z = (torch.rand(n, generator=g, device=dev, dtype=torch.float64) * L - L / 2).to(torch.float32)
    batches = []
    for _ in range(ticks):
        order = torch.randperm(n, generator=g, device=dev).to(torch.int32)
        x = x + (2 * torch.rand(n, generator=g, device=dev, dtype=torch.float64) - 1).to(torch.float32)
        z = z + (2 * torch.rand(n, generator=g, device=dev, dtype=torch.float64) - 1).to(torch.float32)
        batches.append((order, x[order.long()].contiguous(), z[order.long()].contiguous()))
    x0h = batches[0][1].new_empty(n)
    x0h[batches[0][0].long()] = batches[0][1]
    z0h = batches[0][2].new_empty(n)
    z0h[batches[0][0].long()] = batches[0][2]
    x0h, z0h = x0h.cpu().numpy(), z0h.cpu().numpy()
    torch.cuda.synchronize(dev)
    w = World(max(n, 1), max_spaces=max(ns, 1), device=device)
    sp = [w.space_create(100.0) for _ in range(ns)]
    slots = np.arange(n, dtype=np.uint32)
    for k in range(ns):
        a, b = k * per, (k + 1) * per
        w.enter_batch(sp[k], slots[a:b], x0h[a:b], z0h[a:b])
    w.tick_device()  # populate at batch 0's positions
    setup_s = time.perf_counter() - t_setup
    ptrs = [(o.data_ptr(), bx.data_ptr(), bz.data_ptr()) for o, bx, bz in batches]
    for t in range(1, args.cfg4_warmup):
        w.moved_batch_device(*ptrs[t], n)
        w.tick_device()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    w.sync()
    ev = 0
    t0 = time.perf_counter()
    for t in range(max(1, args.cfg4_warmup), ticks):
        w.moved_batch_device(*ptrs[t], n)
        ne, nl = w.tick_device()
        ev += ne + nl
    w.sync()
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    steps = ticks - max(1, args.cfg4_warmup)
    el_max, (moves_all, ev_all) = reduce_over_ranks(dist, el, [n * steps, ev], red_dev)
    w.close()
    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu_baseline and args.cfg4_cpu_seconds > 0:
        try:
            cpu = cpu_baseline_spaces(args, args.cfg4_cpu_seconds)
        except Exception as e:  # the baseline must not take the GPU number down with it
            cpu = {"error": repr(e)}
    return {"metric": "AOI entity-moves/sec, config 4 (strong scaling: fixed total work over the ranks)",
            "value": moves_all / el_max, "unit": "entity-moves/s", "ms_per_step": el_max / steps * 1e3,
            "steps": steps, "n_gpus": ws, "scaling": "strong", "events_per_s": ev_all / el_max,
            "spaces_total": total, "entities_total": total * per, "entities_rank0": n, "setup_s_rank0": round(setup_s, 2),
            "data": "synthetic (torch Philox on the GPU, generated before timing, resident in HBM)",
            "cpu_baseline": cpu}


def cpu_baseline(args, wl_factory, target_s: float):
    """go-aoi XZListAOIManager restatement (oracle/xzlist.c), one core, timed on
    a prefix of tick 0's move batch of the same workload (cfg4: one space per
    core, cpu_baseline_spaces)."""
    if args.workload == "cfg4":
        return cpu_baseline_spaces(args, target_s)
    from oracle import oracle
    wl = wl_factory()
    m = oracle.XZList(wl.D, wl.n, record=False)
    slots, x0, z0, sp = wl.initial()
    if wl.n_spaces != 1:
        per = wl.n // wl.n_spaces
        slots, x0, z0 = slots[:per], x0[:per], z0[:per]
    m.bulk_enter(slots.astype(np.int32), x0, z0)
    sl, nx, nz = wl.tick(0)
    if wl.n_spaces != 1:
        keep = sl < slots.size
        sl, nx, nz = sl[keep], nx[keep], nz[keep]
    done = 0
    chunk = 256
    t0 = time.perf_counter()
    while done < sl.size and time.perf_counter() - t0 < target_s:
        k = min(chunk, sl.size - done)
        m.moved_batch(sl[done:done + k], nx[done:done + k], nz[done:done + k])
        done += k
        chunk = min(chunk * 2, 8192)
    dt = time.perf_counter() - t0
    ne, nl = m.counts()
    return {
        "value": done / dt,
        "unit": "entity-moves/s",
        "events_per_s": (ne + nl) / dt,
        "cores": 1,
        "kind": "port",
        "sample": f"first {done} Moved calls of tick 0 of {args.workload} "
                  f"({'1 space of ' + str(slots.size) if wl.n_spaces != 1 else str(wl.n)} entities), "
                  f"sequential XZ-list restatement, {dt:.1f} s",
    }


def cfg5_cpu_baseline(x0, z0, ops0, target_s: float):
    """CPU-XZ at config 5 (BASELINE.md:49): the go-aoi restatement (oracle/xzlist.c), one
    core, populated with the 2^24 entities (bulk populate, untimed), then timed on the
    first Moved calls of tick 0 in call order until target_s; the per-move cost is
    extrapolated to the whole tick (every entity moves once)."""
    from oracle import oracle
    n = x0.size
    t0 = time.perf_counter()
    m = oracle.XZList(D_CFG5, n, record=False)
    m.bulk_enter(np.arange(n, dtype=np.int32), x0, z0)
    pop_s = time.perf_counter() - t0
    rec = np.ascontiguousarray(ops0).view(np.uint8)
    rec = np.frombuffer(rec.tobytes(), np.dtype([("slot", "<u4"), ("x", "<f4"), ("z", "<f4"), ("kind", "<u4"),
                                                 ("seq", "<u8")]))
    rec = rec[np.argsort(rec["seq"], kind="stable")]  # call order
    sl = rec["slot"].astype(np.int32)
    nx, nz = rec["x"].astype(np.float32), rec["z"].astype(np.float32)
    done, chunk = 0, 16
    t0 = time.perf_counter()
    while done < sl.size and time.perf_counter() - t0 < target_s:
        k = min(chunk, sl.size - done)
        m.moved_batch(sl[done:done + k], nx[done:done + k], nz[done:done + k])
        done += k
        chunk = min(chunk * 2, 256)
    dt = time.perf_counter() - t0
    ne, nl = m.counts()
    rate = done / dt
    return {"value": rate, "unit": "entity-moves/s", "events_per_s": (ne + nl) / dt, "cores": 1, "kind": "port",
            "extrapolated_tick_s": n / rate,
            "sample": f"first {done} Moved calls of tick 0 of cfg5 ({n} entities in one space, populated in "
                      f"{pop_s:.1f} s untimed), sequential XZ-list restatement, {dt:.1f} s; the tick "
                      f"(every entity moving once) extrapolated from the per-move cost",
            "note": "BASELINE.md asks for a 65,536-move prefix: at ~50 moves/s (each Moved walks ~23k x-list and "
                    "~23k z-list nodes at this size) that is ~20 min, so the prefix is time-bounded instead"}


class PhaseClock:
    """Wall time of each phase of a (child) job, in seconds: kept for its JSON record and printed
    to stderr as each phase ends, so that a run killed at its time limit still shows where its
    time went.  t0: the process's start (perf_counter of main())."""

    def __init__(self, tag: str, t0: float | None = None, pre: dict | None = None):
        self.tag = tag
        self.t0 = t0 if t0 is not None else time.perf_counter()
        self.phases = dict(pre or {})
        self.last = self.t0 + sum(self.phases.values())
        self.mark("to_strip_setup")

    def mark(self, name: str):
        now = time.perf_counter()
        self.phases[name] = round(now - self.last, 3)
        self.last = now
        print(f"[{self.tag}] {name} {self.phases[name]:.3f} s (at {now - self.t0:.2f} s)", file=sys.stderr, flush=True)

    def note(self, **kv):
        for k, v in kv.items():
            self.phases[k] = round(v, 3)

    def record(self) -> dict:
        return dict(self.phases, total=round(time.perf_counter() - self.t0, 3))


def strip_inputs(args, ws, rank, local, on_host: bool = False):
    """Config 5's inputs for this rank's strip, generated before the process group exists:
    on the GPU (DeviceUniformWorkload), or, when several ranks share one GPU (on_host: the gloo
    rehearsal), on the host (HostUniformWorkload) and sent in one copy -- there, torch's
    generation kernels from several processes at once stalled the shared GPU for 40-90 s per
    tick.  Returns the inputs and their phase times."""
    import torch
    from goworld_amd.strips import even_edges
    from goworld_amd.workload import DeviceUniformWorkload, HostUniformWorkload
    dev = torch.device(f"cuda:{local}")
    t0 = time.perf_counter()
    n = args.n or (1 << 24)
    ticks = args.warmup + args.steps
    cpu_here = rank == 0 and ws == 1 and not args.no_cpu_baseline
    if on_host:
        wl = HostUniformWorkload(n, 0x5EED0005)
        edges = even_edges(ws, -wl.L / 2, wl.L / 2)
        x0h, z0h = (wl.x.copy(), wl.z.copy()) if cpu_here else (None, None)
        t1 = time.perf_counter()
        parts = wl.strip_ops(edges, rank, ticks)
        rows = np.cumsum([0] + [p.shape[0] for p in parts])
        allh = torch.from_numpy(np.concatenate(parts))
        ops0h = parts[1] if cpu_here else None
        alld = allh.to(dev)  # one allocation, one copy
        allops = [alld[int(rows[q]):int(rows[q + 1])] for q in range(len(parts))]
        del parts, allh
    else:
        wl = DeviceUniformWorkload(n, 0x5EED0005, dev)
        edges = even_edges(ws, -wl.L / 2, wl.L / 2)
        edges_t = torch.from_numpy(edges).to(dev)
        x0h = wl.x.cpu().numpy() if cpu_here else None
        z0h = wl.z.cpu().numpy() if cpu_here else None
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        allops = wl.strip_ops(edges_t, rank, ticks)  # one host sync
        ops0h = allops[1].cpu().numpy() if cpu_here else None
    init_ops, ops = allops[0], allops[1:]
    del wl, allops
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return {"n": n, "edges": edges, "ticks": ticks, "cpu_here": cpu_here, "x0h": x0h, "z0h": z0h,
            "init_ops": init_ops, "ops": ops, "ops0h": ops0h, "generated_on": "host" if on_host else "gpu",
            "phases": {"positions": round(t1 - t0, 3), "inputs": round(t2 - t1, 3)}}


def run_strips(args, ws, rank, local, dist, inp):
    """Config 5: one 2^24-entity space cut into one x-strip per rank; every
    tick routes the owned moves, exchanges halo records (the count rows
    all-gathered on the device, RCCL; records point to point to the neighbour
    strips in one RCCL send/recv group) and queues each strip's tick on the
    GPU (the strip records become device Leave / Enter / Moved batches of its
    world, which flushes; the filter keeps the strip's events).  The next
    tick's route waits once for its counts and completes the previous tick
    with that same wait (goworld_amd/strips.py).  Inputs (``strip_inputs``)
    were generated on the GPU before the process group; value = all N moves
    per tick / max time."""
    import torch
    from goworld_amd.shard import reduce_over_ranks
    from goworld_amd.strips import StripShard, exchange, exchange_local, local_slice, setup_count_group

    dev = torch.device(f"cuda:{local}")
    ph = PhaseClock(f"cfg5 rank {rank}", args.phases_t0, args.phases_pre)  # wall time per phase (JSON + stderr)
    if dist is not None:
        setup_count_group(dist)  # collective over every rank: the host count all-gather's gloo group
        dist.barrier()  # RCCL's communicator exists before the first batched send/recv
        ph.mark("count_group_and_barrier")
    n, edges, ticks, cpu_here = inp["n"], inp["edges"], inp["ticks"], inp["cpu_here"]
    x0h, z0h, init_ops, ops, ops0h = inp["x0h"], inp["z0h"], inp["init_ops"], inp["ops"], inp["ops0h"]
    t_setup = time.perf_counter() - sum(inp["phases"].values())
    sh = StripShard(n, float(D_CFG5), edges, rank, device=local, cells_per_dist=args.cells_per_dist)
    ph.mark("strip_world_create")
    via_cpu = args.dist_backend == "gloo"

    dev_counts = dist is not None and args.strip_counts == "device"

    def one(o, phases=None):
        a = time.perf_counter()
        # the tick's one host wait; it completes the previous tick.  Device counts: every strip's count
        # row all-gathered on the world's stream before that wait (RCCL), no host collective per tick
        send, counts, tele = sh.route(o, dist) if dev_counts else sh.route(o)
        prev = sh.wait()  # the previous tick's counts, completed by the route: no wait
        b = time.perf_counter()
        if dist is not None:
            recv, tele_all, kinds = exchange(dist, send, counts, tele, via_cpu=via_cpu, kinds=sh.kinds,
                                             matrix=sh.matrix)
        else:
            recv, tele_all, kinds = exchange_local([(send, counts, tele)], kinds=[sh.kinds])[0]
        c = time.perf_counter()
        sh.finish(local_slice(send, counts, rank), recv, tele_all, kinds=kinds)  # queued, no wait
        if phases is not None:
            phases[0] += b - a
            phases[1] += c - b
            phases[2] += time.perf_counter() - c
        return int(counts.sum() - counts[rank]), int(recv.shape[0]), prev

    ph0 = [0.0, 0.0, 0.0]
    one(init_ops, ph0)
    ph.mark("populate_route_exchange_queue")
    ne0, nl0 = sh.wait()
    ph.mark("populate_flush_wait")
    setup_s = time.perf_counter() - t_setup
    ph.note(populate_route=ph0[0], populate_exchange=ph0[1], populate_queue=ph0[2])
    for t in range(args.warmup):
        one(ops[t])
    sh.wait()
    ph.mark("warmup_ticks")
    w = sh.world
    w.set_stage_timing([] if args.no_timing else ["combined"])
    w.reset_stage_times()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    lat, events, sent, recvd = [], 0, 0, 0
    phases = [0.0, 0.0, 0.0]
    waits0 = sh.host_waits()
    t0 = time.perf_counter()
    for t in range(args.warmup, ticks):
        a = time.perf_counter()
        ns, nr, (ne, nl) = one(ops[t], phases)
        if t > args.warmup:  # the previous tick's events (the first timed route completes a warmup tick)
            events += ne + nl
        lat.append(time.perf_counter() - a)
        sent += ns
        recvd += nr
    waits = sh.host_waits() - waits0  # (the last tick's completion below is outside the per-tick count)
    ne, nl = sh.wait()  # the last tick
    events += ne + nl
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ph.mark("timed_ticks")
    timed = w.stage_times() if not args.no_timing else {}
    info = w.info()
    el_max, (moves_all, events_all, halo_all, live_all, waits_all) = reduce_over_ranks(
        dist, elapsed, [n * args.steps / ws, events, sent, info["live"], waits],
        "cpu" if args.dist_backend == "gloo" else dev)
    ph.mark("rank_reduction")
    cpu = None
    if cpu_here:
        try:
            cpu = cfg5_cpu_baseline(x0h, z0h, ops0h, args.cpu_seconds)
        except Exception as e:  # the baseline must not take the GPU number down with it
            cpu = {"error": repr(e)}
        ph.mark("cpu_sample")
    if rank == 0:
        lat_ms = np.array(lat) * 1e3
        tm = {k: v[0] / max(v[1], 1) for k, v in timed.items() if v[1]}
        roofline = None
        if "combined" in tm:
            alg = combined_pass_bytes(info["live"], info["total_cells"], events / max(args.steps, 1))
            ach = alg / (tm["combined"] * 1e-3) / 1e9
            roofline = {"bound": "hbm", "kernel": "k_combined", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": None,
                        "alg_bytes_per_launch": alg, "avg_launch_ms": round(tm["combined"], 4),
                        "note": "rank 0's strip world"}
        out = {
            "metric": METRIC, "value": moves_all / el_max, "unit": "entity-moves/s", "n_gpus": ws,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": el_max / args.steps * 1e3,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (torch Philox on the GPU, generated before timing, resident in HBM)",
            "config": {"workload": f"cfg5: {WORKLOAD_DESC['cfg5']}", "entities": n, "strips": ws,
                       "aoi_distance": float(D_CFG5), "halo": sh.halo,
                       "parallelism": f"one x-strip per rank x{ws}, halo records point to point (RCCL send/recv) "
                                              "to the neighbour strips"},
            "events_per_s": events_all / el_max,
            "p50_tick_ms": float(np.percentile(lat_ms, 50)), "p99_tick_ms": float(np.percentile(lat_ms, 99)),
            "events_per_tick": events_all / max(args.steps, 1), "initial_enter_events_rank0": ne0,
            "halo_records_per_tick": halo_all / max(args.steps, 1),
            "halo_note": "records sent to other ranks (24 B each), all ranks",
            "host_waits_per_tick": waits_all / ws / max(args.steps, 1),
            "strip_world_entities_sum": live_all, "setup_s": round(setup_s, 2), "phases_s": ph.record(),
            "strip_counts": args.strip_counts if dist is not None else "local",
            "inputs_generated_on": inp["generated_on"],
            "rank0_phase_ms_per_tick": {"route_and_previous_tick_wait": round(phases[0] / args.steps * 1e3, 4),
                                        "exchange": round(phases[1] / args.steps * 1e3, 4),
                                        "tick_queue": round(phases[2] / args.steps * 1e3, 4)},
            "tick_note": "asynchronous strip tick: route's one host wait brings its counts and completes the "
                         "previous tick (receive, world Leave/Enter/Moved device batches, flush, filter); "
                         "p50/p99 = route + exchange + queue per tick",
            "roofline": roofline, "cpu_baseline": cpu,
        }
        line = json.dumps(out)
        if args.json_out:
            with open(args.json_out, "w") as fh:
                fh.write(line + "\n")
        else:
            print(line, flush=True)
    sh.close()


def cfg5_job(args, ws, rank, local):
    """The config-5 strip run as a sub-record of the default line (`cfg5_strips`): one child
    job of ws ranks (`bench.py --workload cfg5`), started here before this process touches
    the GPU and waited for with a time limit, so that the strip / RCCL path runs on the
    driver's own multi-GPU launches while a hang or crash in it cannot take the headline
    down.  Returns the child's JSON (rank 0) or an error record."""
    import subprocess
    import tempfile
    out = os.path.join(tempfile.gettempdir(), f"gwaoi_cfg5_{os.getpid()}_{rank}.json")
    env = dict(os.environ)
    port = int(os.environ.get("MASTER_PORT", "0") or 0)
    env.update(RANK=str(rank), LOCAL_RANK=str(local), WORLD_SIZE=str(ws), LOCAL_WORLD_SIZE=str(ws),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port + 1 if port else _free_port()))
    cmd = [sys.executable, os.path.abspath(__file__), "--workload", "cfg5", "--gpus", str(ws), "--steps",
           str(args.cfg5_steps), "--warmup", str(args.cfg5_warmup), "--dist-backend", args.dist_backend,
           "--json-out", out, "--cpu-seconds", str(args.cfg5_cpu_seconds), "--strip-counts", args.strip_counts]
    if args.cfg5_entities:
        cmd += ["--entities", str(args.cfg5_entities)]
    if args.no_cpu_baseline or args.cfg5_cpu_seconds <= 0:
        cmd.append("--no-cpu-baseline")
    t0 = time.perf_counter()
    err_path = out + ".err"
    err_text = ""
    with open(err_path, "w") as err_fh, open(err_path) as tail_fh:
        p = subprocess.Popen(cmd, env=env, stdout=subprocess.DEVNULL, stderr=err_fh)
        rc = None
        beat = t0
        while rc is None:  # the child's stderr passed on as it comes (its phase lines show a slow run live)
            try:
                rc = p.wait(timeout=2.0)
            except subprocess.TimeoutExpired:
                now = time.perf_counter()
                if now - t0 > args.cfg5_timeout:
                    p.kill()
                    p.wait()
                    rc = "timeout"
                elif now - beat >= 60.0:
                    beat = now
                    print(f"[cfg5 job, rank {rank}] child running for {now - t0:.0f} s", file=sys.stderr, flush=True)
            new = tail_fh.read()
            if new:
                err_text += new
                sys.stderr.write(new)
                sys.stderr.flush()
        new = tail_fh.read()
        err_text += new
        sys.stderr.write(new)
    wall = round(time.perf_counter() - t0, 1)
    try:
        os.unlink(err_path)
    except OSError:
        pass
    phase_lines = [ln for ln in err_text.splitlines() if ln.startswith("[cfg5 rank")]
    if rank != 0:
        return None
    res = None
    try:
        with open(out) as fh:
            res = json.loads(fh.read().strip().splitlines()[-1])
        os.unlink(out)
    except (OSError, ValueError, IndexError):
        pass
    if res is None:
        return {"error": f"cfg5 child job: exit {rc} after {wall} s, no result", "phase_lines": phase_lines[-24:]}
    res["job"] = {"wall_s": wall, "exit": rc, "note": "child job of the default bench (bench.py --workload cfg5), "
                                                      "one rank per GPU, run before the cfg3 line's own ranks "
                                                      "touch the GPU"}
    return res


D_CFG5 = np.float32(100.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="cfg3", choices=sorted(WORKLOAD_DESC))
    ap.add_argument("--entities", dest="n", type=int, default=None, help="override entity count (cfg2/3/5)")
    ap.add_argument("--spaces", type=int, default=None, help="cfg4: total spaces (default 8192)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--time-every", type=int, default=4,
                    help="bracket the dominant kernel with HIP events on every k-th timed tick (the events "
                         "stall the queue for ~10 us around the launch)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: exchange through host memory (multi-rank rehearsal on one GPU)")
    ap.add_argument("--no-timing", action="store_true", help="no HIP events at all (no roofline / breakdown)")
    ap.add_argument("--breakdown-steps", type=int, default=10,
                    help="extra ticks after the timed region with every stage timed by HIP events")
    ap.add_argument("--cells-per-dist", type=float, default=0.0)
    ap.add_argument("--sync-steps", type=int, default=5,
                    help="extra ticks through the entity-sync path: client packets decoded in HBM, flush, "
                         "CollectEntitySyncInfos fan-out (0 = off)")
    ap.add_argument("--sync-clients", type=float, default=0.5,
                    help="fraction of entities with a client (players) in the sync leg")
    ap.add_argument("--host-io-steps", type=int, default=30,
                    help="extra ticks timed with host move batches in and host event arrays out (PCIe-inclusive), "
                         "serial and pipelined")
    ap.add_argument("--host-tick-steps", type=int, default=10,
                    help="ticks of the C++ host tick bench (tools/tick_bench.cpp; 0 = off)")
    ap.add_argument("--cfg4-steps", type=int, default=5,
                    help="cfg3 runs: timed ticks of the config-4 strong-scaling sub-record (0 = off)")
    ap.add_argument("--cfg4-warmup", type=int, default=3)
    ap.add_argument("--serial-issue", action="store_true",
                    help="register tick t+1's move batch only after tick t's flush returned (default: registered "
                         "while the flush of tick t runs, gwaoi_tick_begin/_end, as a game loop receives moves)")
    ap.add_argument("--cfg4-spaces", type=int, default=8192)
    ap.add_argument("--no-speculative", action="store_true",
                    help="overlap mode without gwaoi_tick_finish(NEXT): each flush is queued after the commit "
                         "of the previous one (A/B of the speculative launch)")
    ap.add_argument("--wire-steps", type=int, default=5,
                    help="timed calls per gate/dispatcher regroup in the wire leg (0 = off)")
    ap.add_argument("--wire-records", type=int, default=1_000_000, help="32-B client records per wire regroup call")
    ap.add_argument("--wire-out-records", type=int, default=4_000_000,
                    help="48-B game records per gate_to_clients call (one gate's share of a cfg3 collect)")
    ap.add_argument("--claims", action="store_true",
                    help="A/B: apply the moves through the last-op claims + repeated-slot fixup instead of "
                         "GWAOI_F_UNIQUE_MOVES (the workload's batches name every entity once per tick)")
    ap.add_argument("--claims-steps", type=int, default=20,
                    help="cfg3 at N=1: timed ticks of the claims sub-record (the general-contract flush: a batch "
                         "may repeat an entity; 0 = off)")
    ap.add_argument("--small-flush-reps", type=int, default=20,
                    help="cfg3: timed flushes per size of the small-flush leg (1/64/4096/65536 moves; 0 = off)")
    ap.add_argument("--strip-counts", default="device", choices=["device", "host"],
                    help="cfg5: the per-tick count exchange -- device: all-gathered on the GPU inside the route's "
                         "one host wait (RCCL); host: gloo all-gather of host tensors after it")
    ap.add_argument("--cfg5-steps", type=int, default=5,
                    help="cfg3 runs: timed ticks of the config-5 strip sub-record (child job; 0 = off)")
    ap.add_argument("--cfg5-warmup", type=int, default=3)
    ap.add_argument("--cfg5-entities", type=int, default=0, help="cfg5 sub-record entities (default 2^24)")
    ap.add_argument("--cfg5-timeout", type=float, default=420.0, help="seconds before the cfg5 child job is killed")
    ap.add_argument("--cfg5-cpu-seconds", type=float, default=10.0,
                    help="CPU-XZ sample of the cfg5 sub-record (rank 0 at N=1; 0 = off)")
    ap.add_argument("--cfg4-cpu-seconds", type=float, default=10.0,
                    help="CPU-XZ of the cfg4 sub-record on all cores (rank 0 at N=1; 0 = off)")
    ap.add_argument("--json-out", default=None, help="write the JSON line to this file instead of stdout")
    args = ap.parse_args()

    # --gpus N without an outside launcher: spawn the N ranks here, before anything touches the GPU
    try:
        plan = launch_plan(args.gpus, os.environ)
    except ValueError as e:
        print(f"bench.py: {e}", file=sys.stderr)
        sys.exit(2)
    if plan is not None:
        sys.exit(spawn_ranks(plan))
    ws, rank, local = dist_env()
    # the config-5 strip sub-record runs first, as a child job, while this process has not touched the GPU
    cfg5 = cfg5_job(args, ws, rank, local) if args.workload == "cfg3" and args.cfg5_steps > 0 else None
    dist = None
    args.phases_t0 = T_START
    args.phases_pre = {}
    strip_inp = None
    if ws > 1:
        import torch
        import torch.distributed as dist
        if args.dist_backend == "nccl" and torch.cuda.device_count() < ws:
            print(f"bench.py: {ws} ranks over RCCL need {ws} GPUs, {torch.cuda.device_count()} visible "
                  "(RCCL allows one rank per device; --dist-backend gloo rehearses several ranks on one GPU)",
                  file=sys.stderr)
            sys.exit(2)
        if args.dist_backend == "gloo":  # rehearsal: several ranks may share a GPU
            local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        t_in = time.perf_counter()
        if args.workload == "cfg5":  # the inputs before the process group (strip_inputs)
            strip_inp = strip_inputs(args, ws, rank, local, on_host=ws > torch.cuda.device_count())
        t_pg = time.perf_counter()
        dist.init_process_group(args.dist_backend)
        args.phases_pre = {"start_to_inputs": round(t_in - T_START, 3)}
        if strip_inp is not None:
            args.phases_pre.update(strip_inp["phases"])
        args.phases_pre["init_process_group"] = round(time.perf_counter() - t_pg, 3)
        if args.workload == "cfg5":
            print(f"[cfg5 rank {rank}] {args.phases_pre}", file=sys.stderr, flush=True)
    device = local
    red_dev = "cpu" if args.dist_backend == "gloo" else f"cuda:{device}"
    if args.workload == "cfg5":
        if strip_inp is None:
            t_in = time.perf_counter()
            strip_inp = strip_inputs(args, ws, rank, local)
            args.phases_pre = {"start_to_inputs": round(t_in - T_START, 3)} | strip_inp["phases"]
        run_strips(args, ws, rank, local, dist, strip_inp)
        if dist is not None:
            dist.destroy_process_group()
        return

    from goworld_amd import World
    from goworld_amd.shard import assign_spaces, reduce_over_ranks
    from goworld_amd.workload import make_workload

    def wl_factory():
        if args.workload == "cfg4":
            # total spaces fixed, split over the ranks in contiguous blocks balanced by entity
            # count (strong scaling); each rank generates its own block
            total = args.spaces or 8192
            lo, hi = assign_spaces([2000] * total, ws)[rank]
            return make_workload("cfg4", seed=0x5EED0004 + 7919 * lo, n_spaces=max(1, hi - lo))
        seed = 0x5EED0000 + int(args.workload[-1]) + 7919 * rank
        return make_workload(args.workload, n=args.n, seed=seed)

    t_setup = time.perf_counter()
    wl = wl_factory()
    n = wl.n
    bd = 0 if args.no_timing else max(0, args.breakdown_steps)
    timed_end = args.warmup + args.steps
    ticks = timed_end + bd
    hio = max(0, args.host_io_steps)
    # ---- synthetic move batches, generated before timing, resident in HBM
    import torch
    torch.cuda.set_device(device)
    batches = []
    for t in range(ticks):
        sl, nx, nz = wl.tick(t)
        batches.append((sl, nx, nz))
    # PCIe-inclusive leg (host memory): three untimed warmup ticks (one serial, two pipelined: they
    # allocate both pinned staging buffers) + hio serial + hio + 1 pipelined
    host_batches = [wl.tick(ticks + t) for t in range(4 * hio + 17 if hio else 0)]
    sync_steps = max(0, args.sync_steps) if ws == 1 or args.workload != "cfg4" else 0
    sync_batches = [wl.tick(ticks + len(host_batches) + t) for t in range(sync_steps + 1 if sync_steps else 0)]
    d_slots = torch.from_numpy(np.stack([b[0] for b in batches]).astype(np.int32)).to(f"cuda:{device}")
    d_x = torch.from_numpy(np.stack([b[1] for b in batches])).to(f"cuda:{device}")
    d_z = torch.from_numpy(np.stack([b[2] for b in batches])).to(f"cuda:{device}")
    moves_per_tick = [b[0].size for b in batches]
    last_batch = batches[-1]  # every entity's position after the last tick (the small-flush leg moves from there)
    del batches
    torch.cuda.synchronize()

    # the move batches are in HBM before the timed region; each names every moving entity once (a
    # permutation per tick): GWAOI_F_UNIQUE_MOVES, checked on the device by every flush (a repeated slot
    # would fail the tick).  The claims sub-record times the general contract beside it.
    w = World(n, max_spaces=wl.n_spaces, device=device, cells_per_dist=args.cells_per_dist,
              unique_moves=not args.claims)
    spaces = [w.space_create(wl.D) for _ in range(wl.n_spaces)]
    wl0 = wl_factory()  # initial positions (wl has advanced through the batches)
    initial = wl0.initial()
    slots, x0, z0, sp = initial
    del wl0
    for s in range(wl.n_spaces):
        sel = np.nonzero(sp == s)[0] if wl.n_spaces > 1 else slice(None)
        w.enter_batch(spaces[s], slots[sel], x0[sel], z0[sel])
    ne0, nl0 = w.tick_device()  # populate: every pair is an enter event
    setup_s = time.perf_counter() - t_setup

    # device addresses of each tick's batch, taken once (torch row views cost microseconds of host time
    # per call, during which the GPU would sit idle between ticks)
    row_ptrs = [(d_slots[t].data_ptr(), d_x[t].data_ptr(), d_z[t].data_ptr()) for t in range(ticks)]

    tick_counts = {}  # (enters, leaves) per tick: the claims sub-record must match them

    def step(t):
        ps, px, pz = row_ptrs[t]
        w.moved_batch_device(ps, px, pz, moves_per_tick[t])
        tick_counts[t] = w.tick_device()
        return tick_counts[t]

    # warmup; its last ticks time every stage to find the dominant one
    dom = "combined"
    for t in range(args.warmup):
        if not args.no_timing and t == max(0, args.warmup - 2):
            w.set_stage_timing(None)
            w.reset_stage_times()
        step(t)
    if not args.no_timing and args.warmup:
        w.sync()
        wst = {k: v[0] / v[1] for k, v in w.stage_times().items() if v[1] and k in STAGE_KERNEL}
        if wst:
            dom = max(wst, key=wst.get)
    # timed region: HIP events only around the dominant kernel (the roofline's launch time)
    w.set_stage_timing([] if args.no_timing else [dom])
    w.reset_stage_times()

    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    w.sync()
    lat = []
    events = 0
    moves = 0
    every = max(1, args.time_every)
    overlap = not args.serial_issue
    spec = overlap and not args.no_speculative

    def timing_for(t):
        if not args.no_timing:
            w.set_stage_timing([dom] if (t - args.warmup) % every == 0 else [])

    if overlap:  # tick t's batch is registered before the timed loop, like the later ones during a flush
        ps, px, pz = row_ptrs[args.warmup]
        w.moved_batch_device(ps, px, pz, moves_per_tick[args.warmup])
    t0 = time.perf_counter()
    if spec:
        timing_for(args.warmup)
        w.tick_begin()
    for t in range(args.warmup, timed_end):
        a = time.perf_counter()
        if spec:
            # flush t is in flight; tick t+1's batch is registered meanwhile, then one call finishes t and
            # queues t+1 on the GPU before t's summary is waited for (gwaoi_tick_finish(NEXT))
            if t + 1 < timed_end:
                ps, px, pz = row_ptrs[t + 1]
                w.moved_batch_device(ps, px, pz, moves_per_tick[t + 1])
                timing_for(t + 1)
                ne, nl = w.tick_end_begin_device()
            else:
                ne, nl = w.tick_end_device()
        elif overlap:
            timing_for(t)
            # flush t on the GPU; tick t+1's batch is registered (queued for the next flush) meanwhile
            w.tick_begin()
            if t + 1 < timed_end:
                ps, px, pz = row_ptrs[t + 1]
                w.moved_batch_device(ps, px, pz, moves_per_tick[t + 1])
            ne, nl = w.tick_end_device()
        else:
            timing_for(t)
            ne, nl = step(t)
        lat.append(time.perf_counter() - a)
        tick_counts[t] = (ne, nl)
        events += ne + nl
        moves += moves_per_tick[t]
    w.sync()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    timed_stages = w.stage_times() if not args.no_timing else {}
    info = w.info()
    dbg_all = w.debug_counters()
    spec_launches = dbg_all["speculative_launches"]
    ovl_flushes = dbg_all.get("overlapped_flushes", 0)
    # ---- per-stage breakdown: separate ticks, every stage bracketed by HIP events
    stages = {}
    if bd:
        w.set_stage_timing(None)
        w.reset_stage_times()
        for t in range(timed_end, ticks):
            step(t)
        w.sync()
        stages = w.stage_times()
        w.set_stage_timing([])

    claims = None
    if args.claims_steps > 0 and ws == 1 and args.workload == "cfg3" and not args.claims:
        c1 = min(timed_end, args.warmup + args.claims_steps)
        try:
            claims = claims_leg(args, n, wl.n_spaces, wl.D, initial, device, row_ptrs, moves_per_tick, args.warmup,
                                c1, {t: tick_counts[t] for t in range(c1) if t in tick_counts})
        except Exception as e:  # a side leg must not take the headline down with it
            claims = {"error": repr(e)}
    del initial
    small = None
    if args.small_flush_reps > 0 and ws == 1 and args.workload == "cfg3":
        small = small_flush_leg(w, last_batch, args.small_flush_reps)
    # ---- PCIe-inclusive leg (SURVEY.md §8d's tick, BASELINE.md's p50/p99 "end-to-end from H2D to event CSR in
    # host memory"): host move arrays -> pinned staging -> H2D -> flush -> events in pinned host memory
    host_io = host_io_leg(w, host_batches, hio, dist, red_dev) if hio else None
    sync = sync_leg(w, n, sync_batches, args.sync_clients) if sync_batches else None
    wire = None
    if args.wire_steps > 0 and ws == 1 and args.workload == "cfg3":
        try:
            wire = wire_leg(args.wire_steps, args.wire_records, args.wire_out_records, device)
        except Exception as e:  # a side leg must not take the headline down with it
            wire = {"error": repr(e)}
    elapsed_max, (moves_all, events_all) = reduce_over_ranks(dist, elapsed, [moves, events], red_dev)
    w.close()
    cfg4 = None
    if args.workload == "cfg3" and args.cfg4_steps > 0:
        cfg4 = cfg4_leg(args, ws, rank, device, dist, red_dev)

    if rank == 0:
        lat_ms = np.array(lat) * 1e3
        # dominant kernel = the costliest stage per tick (HIP events on the world's stream)
        roofline = None
        stage_ms = {k: v[0] / max(v[1], 1) for k, v in stages.items() if v[1]}
        timed_ms = {k: v[0] / max(v[1], 1) for k, v in timed_stages.items() if v[1]}
        if timed_ms.get(dom):
            ev_tick = events / max(args.steps, 1)
            alg = stage_bytes(n, moves / max(args.steps, 1), info["total_cells"], ev_tick)[dom]
            t_s = timed_ms[dom] * 1e-3
            ach = alg / t_s / 1e9
            roofline = {"bound": "hbm", "kernel": STAGE_KERNEL[dom], "achieved": round(ach, 2),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 5),
                        "traffic": pmc_traffic(args.workload) if dom == "combined" else None,
                        "alg_bytes_per_launch": alg, "avg_launch_ms": round(timed_ms[dom], 4),
                        "timed_launches": int(timed_stages[dom][1])}
            if stage_ms.get(dom):
                # in the timed region the next flush's first kernels run beside this kernel (overlapped
                # flushes, two streams), so its launch time there is shared; the stage-timed ticks after
                # the timed region run one flush at a time: the kernel alone
                t_i = stage_ms[dom] * 1e-3
                roofline["isolated"] = {"avg_launch_ms": round(stage_ms[dom], 4),
                                        "achieved": round(alg / t_i / 1e9, 2),
                                        "frac": round(alg / t_i / 1e9 / HBM_PEAK_GBS, 5),
                                        "note": "stage-timed ticks, no flush overlap (the kernel alone on the GPU)"}
        stage_roof = {}
        if stage_ms:
            sb = stage_bytes(n, moves / max(args.steps, 1), info["total_cells"], events / max(args.steps, 1))
            for k, b in sb.items():
                if stage_ms.get(k):
                    gbs = b / (stage_ms[k] * 1e-3) / 1e9
                    stage_roof[k] = {"ms": round(stage_ms[k], 4), "alg_MB": round(b / 1e6, 2),
                                     "GBps": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}
        cpu = None
        if not args.no_cpu_baseline:
            try:
                cpu = cpu_baseline(args, wl_factory, args.cpu_seconds)
            except Exception as e:  # the baseline must not take the GPU number down with it
                cpu = {"error": repr(e)}
            if args.workload == "cfg3" and ws == 1 and isinstance(cpu, dict):
                try:
                    cpu["cpu_grid"] = cpu_grid_baseline(args, args.cpu_seconds)
                except Exception as e:
                    cpu["cpu_grid"] = {"error": repr(e)}
        host_tick = None
        if args.workload == "cfg3" and ws == 1 and args.host_tick_steps > 0 and not args.n:
            host_tick = host_tick_bench(args.host_tick_steps, cpu_cores())
        out = {
            "metric": METRIC,
            "value": moves_all / elapsed_max,
            "unit": "entity-moves/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if args.workload == "cfg4" else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded SplitMix64, generated on host, resident in HBM before timing)",
            "config": {"workload": f"{args.workload}: {WORKLOAD_DESC[args.workload]}", "entities_per_rank": n,
                       "spaces_per_rank": wl.n_spaces, "aoi_distance": float(wl.D),
                       "parallelism": (f"spaces sharded over {ws} ranks, contiguous blocks balanced by entity count"
                                       if args.workload == "cfg4" else
                                       f"one independent space per rank x{ws}") + " (no data-path collective)",
                       "total_cells": info["total_cells"],
                       "move_apply": ("claims (last-op claims + repeated-slot fixup)" if args.claims else
                                      "GWAOI_F_UNIQUE_MOVES (each batch names every entity once; checked on the "
                                      "device every flush)")},
            "events_per_s": events_all / elapsed_max,
            "p50_tick_ms": float(np.percentile(lat_ms, 50)),
            "p99_tick_ms": float(np.percentile(lat_ms, 99)),
            "events_per_tick": events / max(args.steps, 1),
            "initial_enter_events": ne0,
            "setup_s": round(setup_s, 2),
            "tick_loop": ("speculative: gwaoi_tick_finish(NEXT) queues flush t+1 before flush t's summary "
                          f"({spec_launches} of {args.steps} timed flushes; {ovl_flushes} flushes of the run overlapped: "
                          "their first kernels on a second stream beside the pair passes and finish of the flush "
                          "before)" if spec else
                          "overlap: batch t+1 registered while flush t runs" if overlap else "serial"),
            "roofline": roofline,
            "debug_counters": {k: int(dbg_all[k]) for k in ("flushes", "combined_replays", "combined_queue_drains",
                                                             "special_global", "event_regrows", "speculative_launches",
                                                             "unique_flushes", "overlapped_flushes")
                               if k in dbg_all},
            "host_to_host_tick": ({k: host_io[k] for k in ("value", "unit", "ms_per_step", "p50_tick_ms", "p99_tick_ms")}
                                  | {"serial_p50_tick_ms": host_io["serial"]["p50_tick_ms"],
                                     "serial_p99_tick_ms": host_io["serial"]["p99_tick_ms"],
                                     "directed_events_out": host_io["directed_events_out"],
                                     "note": "headline twin: BASELINE.md's tick, the host move batch (caller's "
                                             "pinned buffer, one H2D) -> events in pinned host memory (pipelined: "
                                             "one event per mirrored pair; serial and directed_events_out: every "
                                             "directed event); details in pcie_inclusive"} if host_io else None),
            "pcie_inclusive": host_io,
            "claims_tick": claims,
            "small_flush": small,
            "sync_leg": sync,
            "wire_leg": wire,
            "stages_ms_per_tick": {k: round(v, 4) for k, v in stage_ms.items()},
            "stage_roofline": stage_roof,
            "stages_note": f"separate {bd} ticks after the timed region, every stage bracketed by HIP events "
                           "(the events add ~0.07 ms per tick, so these sum above ms_per_step)",
            "cpu_baseline": cpu,
            "host_tick": host_tick,
            "cfg4_strong": cfg4,
            "cfg5_strips": cfg5,
        }
        if cpu and "value" in cpu:
            out["speedup_vs_cpu"] = out["value"] / ws / cpu["value"]
        out["summary"] = line_summary(out)  # last: the part of the line a tail of stdout keeps
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
