"""Strip tiling of one oversized space over several GPUs (BASELINE config 5,
SURVEY.md §8e "Partitioning (config 5)"; C ABI in include/gwaoi_strips.h).

GoWorld gives every Space one AOI manager (engine/entity/Space.go:33,105).
A space too big for one GPU is cut into x-strips: rank r owns the entities
with x in [edges[r-1], edges[r]) and mirrors, as ghosts, the ones within the
halo H of its strip.  Each tick:

1. ``StripShard.route(ops)``: the AOIManager calls of this tick for the
   entities the rank owned before it (Moved / Leave) or that enter the space
   inside its strip (Enter) become halo records per destination rank, plus
   teleport records (HIP kernels, ``k_route``).
2. ``exchange``: the per-destination counts (with how many of them are
   ENTER / LEAVE records and the box of the ENTERs) are all-gathered on the
   device by the route itself (RCCL, between its kernels and its one host
   wait; gloo on host tensors in a gloo job), then the records go point to point in one
   ``batch_isend_irecv`` group over RCCL (xGMI) -- to the two neighbour
   strips only, when strips are at least H + teleport wide; teleport records
   go to every rank only when some rank has any.  This is the path's one real
   data exchange.
3. ``StripShard.finish(recv, tele, kinds)``: queued on the GPU without a host
   wait (gwaoi_strips_tick_async): the records become device Leave / Enter /
   Moved batches of the rank's gwaoi world (explicit global seqs), the world
   flushes, and only the events this strip owns are kept (enter: owner after
   the tick; leave: owner before it).  The union over ranks is the whole
   space's net diff.  The next ``route`` completes the tick with the same
   host wait that brings its counts: one host wait per tick.

``tile_tick`` runs the three steps for one rank of a ``torch.distributed``
job; ``local_tick`` runs several strips in one process (loopback exchange,
used by the single-GPU parity tests).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import List, Sequence, Tuple

import numpy as np

from ._lib import Events, GwaoiError, StripsConfig, World, load, _p

HALO_MOVE, HALO_ENTER, HALO_LEAVE = 0, 1, 2
HALO_DTYPE = np.dtype([("slot", "<u4"), ("x", "<f4"), ("z", "<f4"), ("kind", "<u4"), ("seq", "<u8")])
TELE_DTYPE = np.dtype([("slot", "<u4"), ("flags", "<u4"), ("px", "<f4"), ("pz", "<f4"), ("pseq", "<u8"),
                       ("x", "<f4"), ("z", "<f4"), ("seq", "<u8")])
HALO_WORDS = HALO_DTYPE.itemsize // 4  # 6 int32 per record (torch transport dtype)
TELE_WORDS = TELE_DTYPE.itemsize // 4  # 10


def default_teleport(D: float) -> float:
    return float(np.float32(D) / np.float32(8.0))


def halo_width(D: float, teleport: float = 0.0) -> float:
    """H = 2D + teleport + 1 (include/gwaoi_strips.h)."""
    t = teleport if teleport > 0 else default_teleport(D)
    return float(np.float32(2.0 * float(np.float32(D)) + float(np.float32(t)) + 1.0))


def even_edges(n_strips: int, lo: float, hi: float) -> np.ndarray:
    """n_strips-1 interior x edges cutting [lo, hi) into equal strips."""
    return np.linspace(lo, hi, n_strips + 1)[1:-1].astype(np.float32)


def balanced_edges(x: np.ndarray, n_strips: int) -> np.ndarray:
    """Interior edges at the entity-count quantiles of x (equal owned counts)."""
    if n_strips <= 1:
        return np.empty(0, np.float32)
    q = np.quantile(np.asarray(x, np.float64), np.arange(1, n_strips) / n_strips)
    e = q.astype(np.float32)
    for i in range(1, e.size):  # strictly increasing
        if e[i] <= e[i - 1]:
            e[i] = np.nextafter(e[i - 1], np.float32(np.inf))
    return e


def owner_of(x: np.ndarray, edges: np.ndarray) -> np.ndarray:
    """Strip owning each x (same float32 compares as the device strip_of)."""
    return np.searchsorted(np.asarray(edges, np.float32), np.asarray(x, np.float32), side="right").astype(np.int64)


def make_ops(slots, x, z, seq, kind=HALO_MOVE) -> np.ndarray:
    """Structured op array (HALO_DTYPE) of one tick's calls."""
    slots = np.asarray(slots, np.uint32)
    a = np.empty(slots.size, HALO_DTYPE)
    a["slot"] = slots
    a["x"] = np.asarray(x, np.float32) if x is not None else 0.0
    a["z"] = np.asarray(z, np.float32) if z is not None else 0.0
    a["kind"] = kind
    a["seq"] = np.asarray(seq, np.uint64)
    return a


def kinds_of(send: np.ndarray, counts) -> tuple:
    """Kind statistics of routed records (HALO_DTYPE, grouped by destination): per destination,
    the ENTER and LEAVE records and the box (x0, z0, x1, z1) of the ENTER positions, as
    gwaoi_strips_route_kinds reports them (CPU model and checks)."""
    S = len(counts)
    ent = np.zeros(S, np.int64)
    lev = np.zeros(S, np.int64)
    box = np.tile(np.array([np.inf, np.inf, -np.inf, -np.inf], np.float32), (S, 1))
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    for q in range(S):
        r = send[off[q]:off[q + 1]]
        e = r[r["kind"] == HALO_ENTER]
        ent[q] = e.size
        lev[q] = int(np.sum(r["kind"] == HALO_LEAVE))
        if e.size:
            box[q] = (e["x"].min(), e["z"].min(), e["x"].max(), e["z"].max())
    return ent, lev, box


def merge_kinds(parts) -> tuple:
    """A receiver's (enters, leaves, box) from the senders' (enters, leaves, box) for it."""
    ne = sum(int(p[0]) for p in parts)
    nl = sum(int(p[1]) for p in parts)
    b = np.array([np.inf, np.inf, -np.inf, -np.inf], np.float32)
    for p in parts:
        if int(p[0]):
            b = np.array([min(b[0], p[2][0]), min(b[1], p[2][1]), max(b[2], p[2][2]), max(b[3], p[2][3])],
                         np.float32)
    return ne, nl, (b if ne else None)


def row_words(S: int) -> int:
    """Words of a strip's device count row (gwaoi_strips_route_begin)."""
    return S + 1 + 6 * S + 1


def _o2f(v) -> np.ndarray:
    """Order-preserving int32 (the device's box words) -> float32."""
    i = np.asarray(v, np.uint32).view(np.int32)
    return np.where(i >= 0, i, i ^ np.int32(0x7FFFFFFF)).astype(np.int32).view(np.float32)


def _f2o(v) -> np.ndarray:
    """float32 -> order-preserving int32 bits (uint32), the device box words."""
    i = np.asarray(v, np.float32).view(np.int32)
    return np.where(i >= 0, i, i ^ np.int32(0x7FFFFFFF)).astype(np.int32).view(np.uint32)


def count_row(counts, n_tele: int, kinds, err: int = 0) -> np.ndarray:
    """The count row gwaoi_strips_route_begin writes on the device (k_route_row), built on the
    host from a route's counts and kinds (CPU model, tests)."""
    S = len(counts)
    ent, lev, box = kinds
    row = np.zeros(row_words(S), np.uint32)
    row[:S] = np.asarray(counts, np.int64)
    row[S] = n_tele
    for d in range(S):
        k = row[S + 1 + 6 * d:S + 7 + 6 * d]
        k[0], k[1] = int(ent[d]), int(lev[d])
        # an empty box is the device's fold identity (INT_MAX, INT_MAX, INT_MIN, INT_MIN)
        k[2:6] = _f2o(box[d]) if int(ent[d]) else np.array([0x7FFFFFFF, 0x7FFFFFFF, 0x80000000, 0x80000000], np.uint32)
    row[-1] = err
    return row


def matrix_counts(matrix: np.ndarray, S: int) -> np.ndarray:
    """M[src, dst] (records) and M[src, S] (teleports) from the gathered device rows."""
    return np.asarray(matrix[:, :S + 1], np.uint32).astype(np.int64)


def matrix_kinds(matrix: np.ndarray, S: int, rank: int) -> tuple:
    """This receiver's (enters, leaves, box) from the gathered device rows (merge_kinds)."""
    parts = []
    for q in range(S):
        k = np.asarray(matrix[q, S + 1 + 6 * rank:S + 1 + 6 * rank + 6], np.uint32)
        ent, lev = int(k[0]), int(k[1])
        box = _o2f(k[2:6]) if ent else np.array([np.inf, np.inf, -np.inf, -np.inf], np.float32)
        parts.append((ent, lev, box))
    return merge_kinds(parts)


def as_words(rec: np.ndarray, words: int):
    """Structured records -> torch int32 (n, words) view (CPU tensor)."""
    import torch
    return torch.from_numpy(np.ascontiguousarray(rec).view(np.int32).reshape(-1, words))


class StripShard:
    """One strip: a gwaoi world holding the strip's owned entities + ghosts,
    and the strip layer (libgwaoi, include/gwaoi_strips.h) on top of it."""

    def __init__(self, max_slots: int, D: float, edges: Sequence[float], rank: int, teleport: float = 0.0,
                 device: int = 0, event_capacity: int = 0, cells_per_dist: float = 0.0):
        import torch
        self._L = load()
        self.torch = torch
        self.device = device
        self.dev = torch.device(f"cuda:{device}")
        self.edges = np.ascontiguousarray(edges, np.float32)
        self.n_strips = self.edges.size + 1
        self.rank = rank
        self.D = np.float32(D)
        self.world = World(max_slots, 1, device=device, event_capacity=event_capacity,
                           cells_per_dist=cells_per_dist)
        self.space = self.world.space_create(D)
        cfg = StripsConfig(self.n_strips, rank, _p(self.edges) if self.edges.size else None, C.c_float(D),
                           C.c_float(teleport))
        h = C.c_void_p()
        self._check(self._L.gwaoi_strips_create(self.world._w, self.space, C.byref(cfg), C.byref(h)), strips=False)
        self._s = h
        hf = C.c_float()
        self._check(self._L.gwaoi_strips_halo(self._s, C.byref(hf)))
        self.halo = hf.value
        # the world's HIP stream as a torch stream: the strip's kernels and torch's producers /
        # consumers of its buffers are ordered by stream waits, not host synchronisation
        self._host_sync = os.environ.get("GWAOI_STRIPS_HOSTSYNC", "0") == "1"  # A/B: host waits instead
        self._inflight = []  # tensors the world's stream may still read (released by finish's host wait)
        w = C.c_uint32()
        self._check(self._L.gwaoi_strips_route_row_words(self._s, C.byref(w)))
        self.row_words = w.value
        self._row = self._mat = self._ext = None  # device count rows (route with dist)
        self.matrix = None  # every strip's count row of the last route with dist (numpy, S x row_words)

    def _cur(self) -> int:
        return self.torch.cuda.current_stream(self.dev).cuda_stream

    def _after_torch(self, *tensors):
        """The world's stream waits for torch's current stream (the producers of `tensors`); the
        tensors are kept referenced until finish() has waited for the world's stream, so the
        caching allocator cannot hand their blocks out while the strip kernels read them."""
        if self._host_sync:
            self.torch.cuda.current_stream(self.dev).synchronize()
            return
        self.world.stream_after(self._cur())
        self._inflight.extend(t for t in tensors if t is not None)

    def _torch_after(self):
        """torch's current stream waits for the world's stream (consumers of the strip's writes)."""
        if self._host_sync:
            self.torch.cuda.synchronize(self.dev)
        else:
            self.world.stream_before(self._cur())

    def close(self):
        if getattr(self, "_s", None):
            self._L.gwaoi_strips_destroy(self._s)
            self._s = None
        if getattr(self, "world", None) is not None:
            self.world.close()
            self.world = None

    def __del__(self):
        self.close()

    def _check(self, rc, strips=True):
        if rc != 0:
            msg = self._L.gwaoi_strips_last_error(self._s).decode() if strips and getattr(self, "_s", None) else ""
            raise GwaoiError(rc, self._L.gwaoi_strerror(rc).decode() + (f" ({msg})" if msg else ""))
        return rc

    # ---- step 1: route this tick's owned ops
    def route(self, ops, dist=None, group=None):
        """ops: device int32 (n, 6) tensor of HALO_DTYPE records.  Returns
        (send (m,6) int32 grouped by destination rank, counts[n_strips] int64,
        tele (k,10) int32).

        dist: the count exchange happens here, on the device: this strip's
        count row is all-gathered from every rank of ``group`` (RCCL over xGMI
        with the nccl backend) on the world's stream, between the route's
        kernels and its one host wait (gwaoi_strips_route_begin / _end);
        ``self.matrix`` then holds every strip's row for ``exchange``, which
        needs no host collective."""
        torch = self.torch
        n = int(ops.shape[0])
        self._after_torch(ops)
        counts = (C.c_uint64 * (self.n_strips + 1))()  # the one host wait of the route: the counts
        pops = C.c_void_p(ops.data_ptr() if n else 0)
        if dist is None:
            self.matrix = None
            self._check(self._L.gwaoi_strips_route(self._s, pops, n, counts))
        else:
            S, W = self.n_strips, self.row_words
            if self._row is None:  # persistent: the world's stream and the collective reuse them every tick
                self._row = torch.zeros(W, dtype=torch.int32, device=self.dev)
                self._mat = torch.zeros(S * W, dtype=torch.int32, device=self.dev)
                self._ext = torch.cuda.ExternalStream(self.world.stream(), device=self.dev)
            self._check(self._L.gwaoi_strips_route_begin(self._s, pops, n, C.c_void_p(self._row.data_ptr())))
            with torch.cuda.stream(self._ext):  # ordered after the route's kernels, before its D2H
                if dist.get_backend(group) == "nccl":
                    dist.all_gather_into_tensor(self._mat, self._row, group=group)
                else:  # gloo rehearsal (CUDA tensors staged through the host by gloo)
                    dist.all_gather([self._mat[q * W:(q + 1) * W] for q in range(S)], self._row, group=group)
            hp = C.c_void_p()
            self._check(self._L.gwaoi_strips_route_end(self._s, C.c_void_p(self._mat.data_ptr()), C.byref(hp),
                                                      counts))
            self.matrix = np.ctypeslib.as_array(C.cast(hp, C.POINTER(C.c_uint32)), shape=(S, W)).copy()
        c = np.array(counts[:], np.int64)
        S = self.n_strips
        ent, lev = (C.c_uint64 * S)(), (C.c_uint64 * S)()
        box = np.empty((S, 4), np.float32)
        self._check(self._L.gwaoi_strips_route_kinds(self._s, ent, lev, _p(box)))
        self.kinds = (np.array(ent[:], np.int64), np.array(lev[:], np.int64), box)
        self._inflight = [ops]  # the route's host wait completed the previous tick; the scatter reads ops
        send = torch.empty((int(c[:-1].sum()), HALO_WORDS), dtype=torch.int32, device=self.dev)
        tele = torch.empty((int(c[-1]), TELE_WORDS), dtype=torch.int32, device=self.dev)
        self._after_torch(send, tele)
        self._check(self._L.gwaoi_strips_route_scatter(self._s, C.c_void_p(send.data_ptr() if send.numel() else 0),
                                                       C.c_void_p(tele.data_ptr() if tele.numel() else 0)))
        self._torch_after()  # the transport reads them after the scatter
        return send, c[:-1], tele

    # ---- step 3: apply the exchanged records, flush, keep this strip's events
    def finish(self, local, recv, tele, kinds=None):
        """local: this strip's own slice of its send buffer; recv: the records
        from the other strips; tele: all teleport records; kinds: this receiver's
        (ENTER records, LEAVE records, box of the ENTERs or None) over local + recv,
        from the senders' route statistics (``exchange(..., kinds=...)``).  With
        kinds the tick is queued and nothing waits (complete it with ``wait`` /
        ``events`` / the next ``route``); returns None.  Without, the strip layer
        reads the kinds back first and waits for the tick: returns (n_enter, n_leave)."""
        nlo, nr, nt = int(local.shape[0]), int(recv.shape[0]), int(tele.shape[0])
        self._after_torch(local, recv, tele)  # the exchange's writes land before the tick reads them
        pl, pr, pt = (C.c_void_p(t.data_ptr() if k else 0) for t, k in ((local, nlo), (recv, nr), (tele, nt)))
        if kinds is None:
            ne, nl = C.c_uint64(), C.c_uint64()
            self._check(self._L.gwaoi_strips_tick(self._s, pl, nlo, pr, nr, pt, nt, C.byref(ne), C.byref(nl)))
            self._inflight.clear()  # gwaoi_strips_tick returned after its last host wait: nothing in flight
            return ne.value, nl.value
        n_ent, n_lev, box = kinds
        b = np.ascontiguousarray(box, np.float32) if box is not None else None
        self._check(self._L.gwaoi_strips_tick_async(self._s, pl, nlo, pr, nr, pt, nt, int(n_ent), int(n_lev),
                                                    _p(b) if b is not None else None))
        return None

    def wait(self) -> Tuple[int, int]:
        """Complete the queued tick: its (n_enter, n_leave).  Right after ``route`` (which
        completed it) this reads the counts without a wait, and the route's scatter keeps its
        inputs referenced."""
        w0 = self.host_waits()
        ne, nl = C.c_uint64(), C.c_uint64()
        self._check(self._L.gwaoi_strips_wait(self._s, C.byref(ne), C.byref(nl)))
        if self.host_waits() != w0:  # the stream drained: nothing queued still reads the held tensors
            self._inflight.clear()
        return ne.value, nl.value

    def host_waits(self) -> int:
        """Stream synchronisations of the strip layer so far (gwaoi_strips_host_waits)."""
        n = C.c_uint64()
        self._check(self._L.gwaoi_strips_host_waits(self._s, C.byref(n)))
        return n.value

    def events(self):
        """This strip's events of the last tick as (n,2) uint32 arrays [a, b] (completes a queued tick)."""
        ev = Events()
        self._check(self._L.gwaoi_strips_events(self._s, C.byref(ev)))
        self._inflight.clear()
        ne, nl = ev.n_enter, ev.n_leave
        ent = np.ctypeslib.as_array(ev.enter, shape=(2 * ne,)).reshape(ne, 2).copy() if ne else np.empty((0, 2), np.uint32)
        lev = np.ctypeslib.as_array(ev.leave, shape=(2 * nl,)).reshape(nl, 2).copy() if nl else np.empty((0, 2), np.uint32)
        return ent, lev

    def events_device(self):
        e, l = C.c_void_p(), C.c_void_p()
        self._check(self._L.gwaoi_strips_events_device(self._s, C.byref(e), C.byref(l)))
        self._inflight.clear()
        return e.value, l.value


# ---------------------------------------------------------------- exchange ---

def local_slice(send, counts, rank):
    """This rank's own records inside its send buffer (they never travel)."""
    c = np.concatenate([[0], np.cumsum(counts)])
    return send[int(c[rank]):int(c[rank + 1])]


_COUNT_GROUPS = {}


def _group_key(dist, group):
    return tuple(range(dist.get_world_size())) if group is None else tuple(dist.get_process_group_ranks(group))


def setup_count_group(dist, group=None):
    """Create the process group that carries the per-destination counts: gloo,
    on host tensors.  route() has the counts on the host already (its scatter
    is sized by them), so exchanging them over gloo costs no device sync; with
    a gloo job it is the job's own group.  ``new_group`` is collective over the
    whole default group, so EVERY rank of the job calls this once at setup
    (tile_tick's callers, bench.py's strip run), before the first exchange --
    not lazily inside exchange, where ranks outside ``group`` would never join.
    Cached on the group's rank tuple."""
    if dist.get_backend(group) == "gloo":
        return group
    key = _group_key(dist, group)
    if key not in _COUNT_GROUPS:
        _COUNT_GROUPS[key] = dist.new_group(ranks=list(key), backend="gloo")
    return _COUNT_GROUPS[key]


def count_group(dist, group=None):
    """The count group set up by ``setup_count_group`` (gloo jobs: the group itself)."""
    if dist.get_backend(group) == "gloo":
        return group
    key = _group_key(dist, group)
    if key not in _COUNT_GROUPS:
        raise RuntimeError("strips.exchange over a non-gloo group needs setup_count_group(dist, group) on every "
                           "rank at setup (dist.new_group is collective)")
    return _COUNT_GROUPS[key]


def exchange(dist, send, counts, tele, group=None, via_cpu=False, kinds=None, matrix=None):
    """The halo exchange of one tick over torch.distributed: the count matrix
    is all-gathered on the host (gloo, ``count_group``), then every record
    travels point to point, batched in one group (``batch_isend_irecv``:
    RCCL send/recv over xGMI for GPU tensors) from its source to its
    destination only -- for strips at least H + teleport wide these are the
    two neighbours -- and a rank's own slice stays put (``local_slice``).
    Teleport records go point to point to every rank, at their exact sizes
    (the count matrix carries them), in the same batch.  Returns
    (records from the other ranks in source-rank order, all teleports).
    via_cpu: GPU tensors go through host memory (gloo rehearsal of several
    ranks sharing one GPU; RCCL allows one rank per device).
    kinds: this rank's route statistics (enters[S], leaves[S], boxes[S, 4]);
    they travel in the same count row, and the receiver's merged
    (enters, leaves, box) is returned third (for ``StripShard.finish``).
    matrix: every strip's device count row, already gathered by
    ``StripShard.route(ops, dist)`` (``shard.matrix``): no host collective
    here; with kinds, the receiver's statistics come from it."""
    import torch
    if via_cpu and send.is_cuda:
        dev = send.device
        torch.cuda.current_stream(dev).synchronize()
        res = exchange(dist, send.cpu(), counts, tele.cpu(), group, kinds=kinds, matrix=matrix)
        return (res[0].to(dev), res[1].to(dev)) + tuple(res[2:])
    S = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = send.device
    rk = None
    if matrix is not None:
        M = matrix_counts(matrix, S)  # M[src, dst]; column S = teleports of src
        if kinds is not None:
            rk = matrix_kinds(matrix, S, rank)
    else:
        row = list(np.asarray(counts, np.int64)) + [int(tele.shape[0])]
        if kinds is not None:
            ent, lev, box = kinds
            row += list(np.asarray(ent, np.int64)) + list(np.asarray(lev, np.int64))
            row += list(np.ascontiguousarray(box, np.float32).reshape(-1).view(np.int32).astype(np.int64))
        mine = torch.tensor(row, dtype=torch.int64)
        rows = [torch.empty_like(mine) for _ in range(S)]
        dist.all_gather(rows, mine, group=count_group(dist, group))
        M = torch.stack(rows).numpy()  # M[src, dst]; column S = teleports of src (host tensors: no device sync)
        if kinds is not None:  # the senders' statistics for this receiver
            bx = M[:, 3 * S + 1:].astype(np.int32).view(np.float32).reshape(S, S, 4)
            rk = merge_kinds([(M[q, S + 1 + rank], M[q, 2 * S + 1 + rank], bx[q, rank]) for q in range(S)])
    off = np.concatenate([[0], np.cumsum(M[rank, :S])]).astype(np.int64)
    peer = (lambda q: q) if group is None else (lambda q: dist.get_global_rank(group, q))
    T = M[:, S]  # teleport records per source rank
    ops, parts, tparts = [], [], {rank: tele}
    for q in range(S):
        if q == rank:
            continue
        if M[rank, q]:
            ops.append(dist.P2POp(dist.isend, send[int(off[q]):int(off[q + 1])], peer(q), group))
        if M[q, rank]:
            buf = torch.empty((int(M[q, rank]), send.shape[1]), dtype=send.dtype, device=dev)
            parts.append(buf)
            ops.append(dist.P2POp(dist.irecv, buf, peer(q), group))
        # teleport records travel to every rank, exact sizes (the count matrix has them): no padding
        if T[rank]:
            ops.append(dist.P2POp(dist.isend, tele, peer(q), group))
        if T[q]:
            tb = torch.empty((int(T[q]), tele.shape[1]), dtype=tele.dtype, device=dev)
            tparts[q] = tb
            ops.append(dist.P2POp(dist.irecv, tb, peer(q), group))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    recv = torch.cat(parts) if parts else send[:0]
    tele_all = tele[:0] if T.sum() == 0 else torch.cat([tparts[r] for r in range(S) if T[r]])
    return (recv, tele_all) if kinds is None else (recv, tele_all, rk)


def exchange_local(outs: List[Tuple], kinds=None):
    """Loopback exchange for several strips in one process: outs[r] =
    (send, counts, tele) of strip r.  Returns [(recv, tele_all)] per strip
    (records from the other strips in source rank order, like ``exchange``);
    with kinds[r] = strip r's route statistics, [(recv, tele_all, kinds of the
    receiver)]."""
    import torch
    S = len(outs)
    starts = []
    for send, counts, _ in outs:
        c = np.concatenate([[0], np.cumsum(counts)])
        starts.append(c)
    tele_all = torch.cat([o[2] for o in outs]) if S else None
    res = []
    for q in range(S):
        parts = [outs[r][0][int(starts[r][q]):int(starts[r][q + 1])] for r in range(S) if r != q]
        if not parts:
            parts = [outs[q][0][:0]]
        r = (torch.cat(parts), tele_all)
        if kinds is not None:
            r += (merge_kinds([(kinds[src][0][q], kinds[src][1][q], kinds[src][2][q]) for src in range(S)]),)
        res.append(r)
    return res


def tile_tick(shard: StripShard, dist, ops, group=None, via_cpu=False, device_counts=None):
    """One tick of this rank's strip in a torch.distributed job: route (the tick's one host
    wait, which also completes the previous tick), exchange, and the tick queued on the GPU
    (``shard.wait()`` / ``shard.events()`` complete it).  device_counts (default: the group's
    backend is nccl): the count rows are all-gathered on the device inside the route."""
    if device_counts is None:
        device_counts = dist.get_backend(group) == "nccl"
    send, counts, tele = shard.route(ops, dist, group) if device_counts else shard.route(ops)
    recv, tele_all, kinds = exchange(dist, send, counts, tele, group=group, via_cpu=via_cpu, kinds=shard.kinds,
                                     matrix=shard.matrix)
    shard.finish(local_slice(send, counts, dist.get_rank(group)), recv, tele_all, kinds=kinds)
    return send, counts, recv


def local_tick(shards: Sequence[StripShard], ops_per_strip, sync=False):
    """One tick of several strips in one process (loopback exchange), queued on each
    strip's stream; sync=True: gwaoi_strips_tick instead (reads the kinds back, waits)."""
    outs = [sh.route(o) for sh, o in zip(shards, ops_per_strip)]
    if sync:
        ex = exchange_local(outs)
        return [sh.finish(local_slice(o[0], o[1], q), r, t) for q, (sh, o, (r, t)) in enumerate(zip(shards, outs, ex))]
    ex = exchange_local(outs, kinds=[sh.kinds for sh in shards])
    for q, (sh, o, (r, t, k)) in enumerate(zip(shards, outs, ex)):
        sh.finish(local_slice(o[0], o[1], q), r, t, kinds=k)
    return None
