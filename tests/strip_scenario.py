"""Seeded op streams for the strip-tiling tests (config-5 style, small).

One space, N0 entities uniform in [-L/2, L/2)^2 (L = sqrt(N0*1250), mean ~32
neighbours), cut into S strips at the x quantiles.  Tick 0 enters everyone;
every later tick moves every live entity by U(-1,1) and mixes in what makes
strip tiling hard: teleports across strips (single and in pairs that stay
together -- the teleporter x teleporter case), Leaves, Enters of fresh and of
re-used slots, and entities parked exactly on strip edges and on halo bounds.
One op per entity per tick; seqs are a global random order per tick.
"""
from __future__ import annotations

import math

import numpy as np

from goworld_amd.strips import HALO_ENTER, HALO_LEAVE, HALO_MOVE, balanced_edges, halo_width

D = np.float32(100.0)


class Scenario:
    def __init__(self, n0=6000, spare=600, n_strips=4, seed=7, teleports=30, pair_teleports=8, churn=20,
                 edge_hops=40):
        self.rng = np.random.default_rng(seed)
        self.n0, self.max_slots = n0, n0 + spare
        self.L = math.sqrt(n0 * 1250.0)
        r = self.rng
        self.x = np.full(self.max_slots, np.nan, np.float32)
        self.z = np.full(self.max_slots, np.nan, np.float32)
        self.seq = np.zeros(self.max_slots, np.uint64)
        self.live = np.zeros(self.max_slots, bool)
        x0 = (r.random(n0) * self.L - self.L / 2).astype(np.float32)
        z0 = (r.random(n0) * self.L - self.L / 2).astype(np.float32)
        self.edges = balanced_edges(x0, n_strips)
        H = np.float32(halo_width(float(D)))
        # park some entities exactly on edges and on halo bounds (+- 1 ulp)
        k = 0
        for e in self.edges:
            for v in (e, e - H, e + H, np.nextafter(e, -np.inf), np.nextafter(e - H, np.inf),
                      np.nextafter(e + H, -np.inf), e - D, e + D):
                if k < n0:
                    x0[k] = np.float32(v)
                    k += 1
        self.init = (np.arange(n0, dtype=np.uint32), x0, z0)
        self.next_seq = 1
        self.t = 0
        self.teleports, self.pair_teleports, self.churn = teleports, pair_teleports, churn
        self.edge_hops = edge_hops

    def _seqs(self, n):
        s = self.next_seq + self.rng.permutation(n).astype(np.uint64)
        self.next_seq += n
        return s

    def tick(self):
        """Global ops of the next tick: (kind, slot, x, z, seq) arrays, in seq order."""
        r = self.rng
        if self.t == 0:
            slots, x0, z0 = self.init
            kind = np.full(slots.size, HALO_ENTER, np.uint32)
            sl, nx, nz = slots, x0, z0
        else:
            live = np.nonzero(self.live)[0].astype(np.uint32)
            dead = np.nonzero(~self.live)[0].astype(np.uint32)
            r.shuffle(live)
            n_leave = min(self.churn, live.size // 10)
            leavers = live[:n_leave]
            movers = live[n_leave:]
            nx = (self.x[movers] + (2 * r.random(movers.size) - 1).astype(np.float32)).astype(np.float32)
            nz = (self.z[movers] + (2 * r.random(movers.size) - 1).astype(np.float32)).astype(np.float32)
            # single teleports (|dx| in 50..1500, crossing strips)
            k = min(self.teleports, movers.size // 4)
            jump = (np.sign(r.random(k) - 0.5) * (50 + 1450 * r.random(k))).astype(np.float32)
            nx[:k] = (self.x[movers[:k]] + jump).astype(np.float32)
            # pair teleports: a near neighbour b of a jumps with a by the same offset
            # (the pair is related before and after: the teleporter x teleporter case)
            used = np.zeros(movers.size, bool)
            used[:k] = True
            mx, mz = self.x[movers], self.z[movers]
            for p in range(self.pair_teleports):
                i = k + p
                if i >= movers.size or used[i]:
                    continue
                near = np.nonzero((np.abs(mx - mx[i]) < 60) & (np.abs(mz - mz[i]) < 60) & ~used)[0]
                near = near[near != i]
                if near.size == 0:
                    continue
                j = int(near[0])
                used[i] = used[j] = True
                off = np.float32((1 if r.random() < 0.5 else -1) * (300 + 900 * r.random()))
                nx[i] = np.float32(mx[i] + off)
                nx[j] = np.float32(mx[j] + off)
                nz[i], nz[j] = mz[i], mz[j]
            # short teleports across an edge (13 < |dx| < 190): the mover keeps
            # neighbours on both sides, which is what sizes the halo at 2D + teleport
            if self.edges.size:
                dist = np.min(np.abs(mx[:, None] - self.edges[None, :]), axis=1)
                cand = np.nonzero((dist < 150) & ~used)[0][: self.edge_hops]
                for i in cand:
                    e = self.edges[np.argmin(np.abs(self.edges - mx[i]))]
                    step = np.float32(13 + 177 * r.random())
                    nx[i] = np.float32(mx[i] + (step if mx[i] < e else -step))
                    used[i] = True
            # enters: fresh or re-used slots
            n_enter = min(self.churn, dead.size)
            enter = r.choice(dead, n_enter, replace=False) if n_enter else np.empty(0, np.uint32)
            ex = (r.random(n_enter) * self.L - self.L / 2).astype(np.float32)
            ez = (r.random(n_enter) * self.L - self.L / 2).astype(np.float32)
            sl = np.concatenate([movers, leavers, enter]).astype(np.uint32)
            kind = np.concatenate([np.full(movers.size, HALO_MOVE), np.full(leavers.size, HALO_LEAVE),
                                   np.full(enter.size, HALO_ENTER)]).astype(np.uint32)
            nx = np.concatenate([nx, np.zeros(leavers.size, np.float32), ex]).astype(np.float32)
            nz = np.concatenate([nz, np.zeros(leavers.size, np.float32), ez]).astype(np.float32)
        seq = self._seqs(sl.size)
        order = np.argsort(seq, kind="stable")
        kind, sl, nx, nz, seq = kind[order], sl[order], nx[order], nz[order], seq[order]
        # previous positions (owner before the tick) and the state after it
        px = self.x[sl].copy()
        mv = kind != HALO_LEAVE
        self.x[sl[mv]], self.z[sl[mv]], self.seq[sl[mv]] = nx[mv], nz[mv], seq[mv]
        self.live[sl[mv]] = True
        lv = kind == HALO_LEAVE
        self.live[sl[lv]] = False
        self.x[sl[lv]] = np.nan
        self.z[sl[lv]] = np.nan
        self.t += 1
        return kind, sl, nx, nz, seq, px

    def state(self):
        """(x, z, seq, space) per slot after the last tick (space DEAD if not live)."""
        sp = np.where(self.live, 0, 0xFFFFFFFF).astype(np.uint32)
        return self.x.copy(), self.z.copy(), self.seq.copy(), sp


def split_by_owner(kind, sl, nx, nz, seq, px, edges):
    """Per strip: the structured ops its owner receives (Moved/Leave by the
    owner before the tick, Enter by the strip containing the new position)."""
    from goworld_amd.strips import make_ops, owner_of
    own = np.where(kind == HALO_ENTER, owner_of(nx, edges), owner_of(np.nan_to_num(px), edges))
    out = []
    for q in range(edges.size + 1):
        m = own == q
        ops = make_ops(sl[m], nx[m], nz[m], seq[m])
        ops["kind"] = kind[m]
        out.append(ops)
    return out
