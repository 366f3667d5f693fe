"""CPU model of one strip rank -- TEST INFRASTRUCTURE ONLY.

Restates the strip protocol of goworld_amd/csrc/gwaoi_strips.hip (route,
receive, filter, teleporter pairs) in numpy, with the sequential go-aoi
restatement (oracle/xzlist.c) as the rank's world.  It lets the CPU suite
check the protocol itself -- halo width, ownership rule, teleport patch --
and the torch.distributed exchange (gloo, world_size 2) without a GPU; the
GPU tests check the HIP kernels against a single unsplit world.
"""
from __future__ import annotations

import numpy as np

from goworld_amd.strips import (HALO_DTYPE, HALO_ENTER, HALO_LEAVE, HALO_MOVE, HALO_WORDS, TELE_DTYPE, TELE_WORDS,
                                as_words, default_teleport, kinds_of)


def region_bounds(edges, D, teleport=0.0):
    """float32 region [rlo, rhi) of every strip, rounded outward (gwaoi_strips_create)."""
    S = edges.size + 1
    tele = np.float32(teleport) if teleport > 0 else np.float32(default_teleport(D))
    H = 2.0 * float(np.float32(D)) + float(tele) + 1.0
    lo = np.empty(S, np.float32)
    hi = np.empty(S, np.float32)
    for q in range(S):
        a = -np.inf if q == 0 else float(edges[q - 1]) - H
        b = np.inf if q == S - 1 else float(edges[q]) + H
        fa, fb = np.float32(a), np.float32(b)
        if float(fa) > a:
            fa = np.nextafter(fa, np.float32(-np.inf))
        if float(fb) < b:
            fb = np.nextafter(fb, np.float32(np.inf))
        lo[q], hi[q] = fa, fb
    return lo, hi, tele


def strip_of(x, edges):
    return np.searchsorted(edges, np.asarray(x, np.float32), side="right")


def rel(ax, az, as_, bx, bz, bs, D):
    D = np.float32(D)
    own = as_ > bs
    wx, wz = np.where(own, ax, bx), np.where(own, az, bz)
    px, pz = np.where(own, bx, ax), np.where(own, bz, az)
    return ((px >= np.float32(wx - D)) & (px <= np.float32(wx + D)) & (pz >= np.float32(wz - D))
            & (pz <= np.float32(wz + D)))


class ModelShard:
    def __init__(self, max_slots, D, edges, rank, oracle):
        self.D = np.float32(D)
        self.edges = np.asarray(edges, np.float32)
        self.S = self.edges.size + 1
        self.rank = rank
        self.rlo, self.rhi, self.tele = region_bounds(self.edges, D)
        self.cur = np.full((max_slots, 2), np.nan, np.float32)
        self.cseq = np.zeros(max_slots, np.uint64)
        self.prv = np.full((max_slots, 2), np.nan, np.float32)
        self.pseq = np.zeros(max_slots, np.uint64)
        self.ptick = np.zeros(max_slots, np.int64)
        self.ttick = np.zeros(max_slots, np.int64)
        self.tick_id = 0
        self.oracle = oracle
        self.world = oracle.XZList(D, max_slots)
        self.last = (np.empty(0, np.uint64), np.empty(0, np.uint64))

    def _mask(self, x):
        return (x >= self.rlo) & (x < self.rhi)  # per strip

    def route(self, ops):
        ops = np.frombuffer(ops.numpy().tobytes(), HALO_DTYPE) if hasattr(ops, "numpy") else ops
        sends = [[] for _ in range(self.S)]
        tele = []
        for op in ops:
            s, kind = int(op["slot"]), int(op["kind"])
            pv = self.cur[s]
            have = not np.isnan(pv[0])
            mine = have and strip_of(pv[0], self.edges) == self.rank
            if kind == HALO_MOVE:
                assert mine, f"move of slot {s} not owned by strip {self.rank}"
            elif kind == HALO_ENTER:
                assert not have and strip_of(op["x"], self.edges) == self.rank
            else:
                assert mine
            mP = self._mask(pv[0]) if kind != HALO_ENTER else np.zeros(self.S, bool)
            mN = self._mask(op["x"]) if kind != HALO_LEAVE else np.zeros(self.S, bool)
            for q in range(self.S):
                if not (mP[q] or mN[q]):
                    continue
                r = np.zeros(1, HALO_DTYPE)
                r["slot"] = s
                r["kind"] = HALO_MOVE if (mP[q] and mN[q]) else (HALO_ENTER if mN[q] else HALO_LEAVE)
                if mN[q]:
                    r["x"], r["z"], r["seq"] = op["x"], op["z"], op["seq"]
                else:
                    r["x"], r["z"], r["seq"] = pv[0], pv[1], self.cseq[s]
                sends[q].append(r)
            if kind == HALO_MOVE and abs(np.float32(op["x"] - pv[0])) > self.tele:
                t = np.zeros(1, TELE_DTYPE)
                t["slot"], t["flags"] = s, 3
                t["px"], t["pz"], t["pseq"] = pv[0], pv[1], self.cseq[s]
                t["x"], t["z"], t["seq"] = op["x"], op["z"], op["seq"]
                tele.append(t)
        counts = np.array([len(v) for v in sends], np.int64)
        allr = [r for v in sends for r in v]
        send = np.concatenate(allr) if allr else np.empty(0, HALO_DTYPE)
        tel = np.concatenate(tele) if tele else np.empty(0, TELE_DTYPE)
        self.kinds = kinds_of(send, counts)  # what gwaoi_strips_route_kinds reports
        return as_words(send, HALO_WORDS), counts, as_words(tel, TELE_WORDS)

    def _before(self, s):
        if self.ptick[s] == self.tick_id:
            return self.prv[s], self.pseq[s]
        return self.cur[s], self.cseq[s]

    def finish(self, local, recv, tele, kinds=None):
        O = self.oracle
        self.tick_id += 1
        t = self.tick_id
        recv = np.concatenate([np.frombuffer(local.numpy().tobytes(), HALO_DTYPE),
                               np.frombuffer(recv.numpy().tobytes(), HALO_DTYPE)])
        if kinds is not None:  # the senders' statistics, as the exchange delivered them, match the records
            e, l, b = kinds_of(recv, [recv.size])
            assert (int(kinds[0]), int(kinds[1])) == (int(e[0]), int(l[0])), (kinds, e, l)
            assert (kinds[2] is None) == (e[0] == 0) and (kinds[2] is None or np.array_equal(kinds[2], b[0]))
        tele = np.frombuffer(tele.numpy().tobytes(), TELE_DTYPE)
        leaves, rest = [], []
        for r in recv:
            s = int(r["slot"])
            have = not np.isnan(self.cur[s][0])
            assert (int(r["kind"]) == HALO_ENTER) != have, "record for a slot in the wrong state"
            self.prv[s], self.pseq[s], self.ptick[s] = self.cur[s], self.cseq[s], t
            if int(r["kind"]) == HALO_LEAVE:
                self.cur[s] = np.nan
                self.cseq[s] = 0
                leaves.append(s)
            else:
                self.cur[s] = (r["x"], r["z"])
                self.cseq[s] = r["seq"]
                rest.append(r)
        for s in tele["slot"]:
            self.ttick[int(s)] = t
        # the world: leaves, then enters/moves in global seq order (= its call order)
        ops, ids, xs, zs = [], [], [], []
        for s in leaves:
            ops.append(O.OP_LEAVE); ids.append(s); xs.append(0); zs.append(0)
        for r in sorted(rest, key=lambda r: int(r["seq"])):
            ops.append(O.OP_ENTER if int(r["kind"]) == HALO_ENTER else O.OP_MOVED)
            ids.append(int(r["slot"])); xs.append(r["x"]); zs.append(r["z"])
        if ops:
            self.world.apply(np.array(ops), np.array(ids), np.array(xs, np.float32), np.array(zs, np.float32))
        ent, lev = O.net_events(*self.world.take_events())
        T = lambda k: (self.ttick[(k >> np.uint64(32)).astype(np.int64)] == t) & (
            self.ttick[(k & np.uint64(0xFFFFFFFF)).astype(np.int64)] == t)
        a_ent = (ent >> np.uint64(32)).astype(np.int64)
        own_now = ~np.isnan(self.cur[a_ent, 0]) & (strip_of(self.cur[a_ent, 0], self.edges) == self.rank)
        keep_e = ent[own_now & ~T(ent)] if ent.size else ent
        a_lev = (lev >> np.uint64(32)).astype(np.int64)
        bx = np.array([self._before(int(a))[0][0] for a in a_lev], np.float32)
        own_bef = ~np.isnan(bx) & (strip_of(bx, self.edges) == self.rank) if lev.size else np.zeros(0, bool)
        keep_l = lev[own_bef & ~T(lev)] if lev.size else lev
        te, tl = [], []
        for i in range(tele.size):
            A = tele[i]
            own_n = bool(A["flags"] & 2) and strip_of(A["x"], self.edges) == self.rank
            own_b = bool(A["flags"] & 1) and strip_of(A["px"], self.edges) == self.rank
            for j in range(tele.size):
                if i == j:
                    continue
                B = tele[j]
                was = bool(A["flags"] & 1 and B["flags"] & 1 and rel(A["px"], A["pz"], A["pseq"], B["px"], B["pz"],
                                                                     B["pseq"], self.D))
                now = bool(A["flags"] & 2 and B["flags"] & 2 and rel(A["x"], A["z"], A["seq"], B["x"], B["z"],
                                                                     B["seq"], self.D))
                k = (np.uint64(A["slot"]) << np.uint64(32)) | np.uint64(B["slot"])
                if own_n and now and not was:
                    te.append(k)
                if own_b and was and not now:
                    tl.append(k)
        self.last = (np.sort(np.concatenate([keep_e, np.array(te, np.uint64)])),
                     np.sort(np.concatenate([keep_l, np.array(tl, np.uint64)])))
        return self.last[0].size, self.last[1].size
