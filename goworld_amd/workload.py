"""Seeded synthetic AOI workloads (BASELINE.json configs 1-5).

Everything is derived from SplitMix64 so that the HIP path, the CPU oracle and
the committed golden fixtures all consume bit-identical float32 inputs.

* ``cfg1`` -- examples/test_game-style single space: N=1000 Avatars at integer
  positions in [-400,400) (examples/test_game/Avatar.go:127-134), each tick
  every entity moves with p=0.5 by the test_client bot random walk
  ``X += -0.01 + 0.02*rand``, ``Z += -0.01 + 0.01*rand`` in float32
  (examples/test_client/ClientBot.go:227-233).
* ``cfg2`` -- one space, N=100k uniform, L=sqrt(N*1250) (mean ~32 neighbours),
  every entity moves by U(-1,1) per axis per tick.
* ``cfg3`` -- one space, N=1M, half uniform, half in 256 Gaussian hotspots
  (sigma 250, centres uniform in [-0.4L,0.4L]^2): skewed cell occupancy.
  Scaled to another N, the hotspot count scales with N (256 N / 1M, at least
  1) so that every hotspot keeps ~1953 entities at sigma 250: the crowd
  density -- and the long cell rows it produces -- is the same at every N.
* ``cfg4`` -- 8192 independent spaces x 2000 entities, per-space L=1581.1.
* ``cfg5`` -- one 2^24-entity world, L=sqrt(N*1250).

Each tick's move order (= the seq order the AOI manager sees) is a seeded
random permutation of that tick's movers (argsort of SplitMix64 keys).
A move is ``x' = fl32(x + fl32(step))`` with no clamping: the reference has no
world bounds (Space.GetSpaceRange is unused, engine/entity/Space.go:52-54).
"""
from __future__ import annotations

import math
import os
import sys
import time
from dataclasses import dataclass

import numpy as np

GAMMA = 0x9E3779B97F4A7C15
M64 = (1 << 64) - 1
D_DEFAULT = np.float32(100.0)  # EnableAOI(100), examples/test_game/MySpace.go:55-57


def mix64(z: int) -> int:
    """SplitMix64 finaliser on a Python int."""
    z &= M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def subseed(seed: int, *tags: int) -> int:
    h = seed & M64
    for t in tags:
        h = mix64(h ^ ((t * GAMMA) & M64))
    return h


def splitmix(seed: int, n: int) -> np.ndarray:
    """n consecutive SplitMix64 outputs of the stream starting at ``seed``."""
    with np.errstate(over="ignore"):
        s = np.uint64(seed & M64) + np.uint64(GAMMA) * np.arange(1, n + 1, dtype=np.uint64)
        z = s
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def unit_f64(r: np.ndarray) -> np.ndarray:
    """u = (r >> 11) * 2^-53 in [0,1), double."""
    return (r >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def unit_f32(r: np.ndarray) -> np.ndarray:
    """float32 in [0,1) with 24 random bits (rand.Float32 analogue)."""
    return ((r >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)).astype(np.float32)


def permutation(seed: int, n: int) -> np.ndarray:
    return np.argsort(splitmix(seed, n), kind="stable").astype(np.uint32)


@dataclass
class Workload:
    name: str
    n: int
    D: np.float32
    x: np.ndarray  # float32 current positions (by slot)
    z: np.ndarray
    space: np.ndarray  # uint32 space id per slot
    n_spaces: int
    seed: int
    L: float

    def initial(self):
        """(slots, x, z, space) of the initial Enter batch, in seq order (slot order)."""
        slots = np.arange(self.n, dtype=np.uint32)
        return slots, self.x.copy(), self.z.copy(), self.space.copy()

    def tick(self, t: int):
        """Return the move batch of tick ``t`` (slots in seq order, new x, new z) and advance."""
        n = self.n
        s = subseed(self.seed, 0x71C, t)
        if self.name == "cfg1":
            r = splitmix(s, 3 * n)
            p = unit_f32(r[0:n])
            movers = np.nonzero(p < np.float32(0.5))[0].astype(np.uint32)
            rx = unit_f32(r[n:2 * n])[movers]
            rz = unit_f32(r[2 * n:3 * n])[movers]
            mr = np.float32(0.01)
            sx = (np.float32(-mr) + (np.float32(2.0) * mr) * rx).astype(np.float32)
            sz = (np.float32(-mr) + mr * rz).astype(np.float32)
        else:
            r = splitmix(s, 2 * n)
            movers = np.arange(n, dtype=np.uint32)
            sx = (2.0 * unit_f64(r[0:n]) - 1.0).astype(np.float32)
            sz = (2.0 * unit_f64(r[n:2 * n]) - 1.0).astype(np.float32)
        nx = (self.x[movers] + sx).astype(np.float32)
        nz = (self.z[movers] + sz).astype(np.float32)
        order = permutation(subseed(self.seed, 0x0D3, t), movers.size)
        slots = movers[order]
        nx, nz = nx[order], nz[order]
        self.x[slots] = nx
        self.z[slots] = nz
        return slots, nx, nz


def _uniform_xy(seed: int, n: int, L: float):
    r = splitmix(seed, 2 * n)
    x = (unit_f64(r[0:n]) * L - L / 2).astype(np.float32)
    z = (unit_f64(r[n:2 * n]) * L - L / 2).astype(np.float32)
    return x, z


def make_workload(cfg: str, n: int | None = None, seed: int | None = None,
                  n_spaces: int | None = None, per_space: int | None = None) -> Workload:
    """Build config ``cfg`` ('cfg1'..'cfg5'); ``n`` scales cfg2/3/5 at constant density."""
    idx = int(cfg[-1])
    if seed is None:
        seed = 0x5EED0000 + idx
    D = D_DEFAULT
    if cfg == "cfg1":
        n = n or 1000
        r = splitmix(subseed(seed, 1), 2 * n)
        x = (np.float32(-400) + (r[0:n] % np.uint64(800)).astype(np.float32)).astype(np.float32)
        z = (np.float32(-400) + (r[n:2 * n] % np.uint64(800)).astype(np.float32)).astype(np.float32)
        sp = np.zeros(n, np.uint32)
        return Workload(cfg, n, D, x, z, sp, 1, seed, 800.0)
    if cfg in ("cfg2", "cfg5"):
        n = n or (100_000 if cfg == "cfg2" else 1 << 24)
        L = math.sqrt(n * 1250.0)
        x, z = _uniform_xy(subseed(seed, 1), n, L)
        return Workload(cfg, n, D, x, z, np.zeros(n, np.uint32), 1, seed, L)
    if cfg == "cfg3":
        n = n or 1_000_000
        L = math.sqrt(n * 1250.0)
        nu = n // 2
        xu, zu = _uniform_xy(subseed(seed, 1), nu, L)
        nh = n - nu
        hot = max(1, round(256 * n / 1_000_000))  # density-preserving: ~1953 entities per hotspot
        rc = splitmix(subseed(seed, 2), 2 * hot)
        cx = (unit_f64(rc[0:hot]) * 0.8 - 0.4) * L
        cz = (unit_f64(rc[hot:]) * 0.8 - 0.4) * L
        r = splitmix(subseed(seed, 3), 5 * nh)
        h = (r[0:nh] % np.uint64(hot)).astype(np.int64)
        u1 = 1.0 - unit_f64(r[nh:2 * nh])  # (0,1]
        u2 = unit_f64(r[2 * nh:3 * nh])
        u3 = 1.0 - unit_f64(r[3 * nh:4 * nh])
        u4 = unit_f64(r[4 * nh:5 * nh])
        sigma = 250.0
        gx = np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * math.pi * u2)
        gz = np.sqrt(-2.0 * np.log(u3)) * np.cos(2.0 * math.pi * u4)
        xh = (cx[h] + sigma * gx).astype(np.float32)
        zh = (cz[h] + sigma * gz).astype(np.float32)
        x = np.concatenate([xu, xh]).astype(np.float32)
        z = np.concatenate([zu, zh]).astype(np.float32)
        return Workload(cfg, n, D, x, z, np.zeros(n, np.uint32), 1, seed, L)
    if cfg == "cfg4":
        n_spaces = n_spaces or 8192
        per_space = per_space or 2000
        n = n_spaces * per_space
        L = math.sqrt(per_space * 1250.0)
        x, z = _uniform_xy(subseed(seed, 1), n, L)
        sp = (np.arange(n, dtype=np.int64) // per_space).astype(np.uint32)
        return Workload(cfg, n, D, x, z, sp, n_spaces, seed, L)
    raise ValueError(f"unknown workload {cfg}")


class DeviceUniformWorkload:
    """Config 5 generated on the GPU with torch (bench only): N entities
    uniform in [-L/2, L/2)^2 with L = sqrt(N*1250), every tick every entity
    moves by U(-1,1) per axis in float32, in a random global call order.

    Every rank of a strip-tiled run replays the same global simulation from
    the same seed (Philox streams are identical on every device) and keeps
    only the ops of the entities its strip owned before the tick, as
    int32 (n, 6) halo records (goworld_amd.strips.HALO_DTYPE).  The numpy
    generators above feed the parity tests; this one only has to produce a
    workload of config 5's shape fast enough to pre-generate 16.8M moves per
    tick before the timed region."""

    def __init__(self, n: int, seed: int, device):
        import torch
        self.torch = torch
        self.n = n
        self.dev = torch.device(device)
        self.L = math.sqrt(n * 1250.0)
        self.D = D_DEFAULT
        self.seed = seed
        g = torch.Generator(device=self.dev)
        g.manual_seed(seed)
        self.x = ((torch.rand(n, generator=g, device=self.dev, dtype=torch.float64) * self.L - self.L / 2)
                  .to(torch.float32))
        self.z = ((torch.rand(n, generator=g, device=self.dev, dtype=torch.float64) * self.L - self.L / 2)
                  .to(torch.float32))
        self.next_seq = 1
        self.t = 0

    def _records(self, slots, x, z, kind, seq):
        torch = self.torch
        r = torch.empty((slots.numel(), 6), dtype=torch.int32, device=self.dev)
        r[:, 0] = slots.to(torch.int32)
        r[:, 1] = x.view(torch.int32)
        r[:, 2] = z.view(torch.int32)
        r[:, 3] = kind
        r[:, 4] = (seq & 0xFFFFFFFF).to(torch.int64).to(torch.int32)
        r[:, 5] = (seq >> 32).to(torch.int32)
        return r

    def owner(self, x, edges_t):
        return self.torch.bucketize(x, edges_t, right=True)

    def strip_ops(self, edges_t, rank: int, ticks: int):
        """[Enter ops of the entities whose start position is in strip `rank` (kind 1, seq = 1 +
        slot)] + [Moved ops of each of `ticks` ticks for the entities the strip owns before it
        (kind 0)], advancing the world; int32 (m, 6) halo records, slots ascending.  One host
        sync for all of them (the owned counts): several ranks sharing one GPU (the gloo
        rehearsal) time-slice the device, and a sync per tick cost seconds each there."""
        torch = self.torch
        trace = os.environ.get("GWAOI_INPUT_TRACE") == "1"  # per-tick wall times to stderr (diagnostics)
        t0 = time.perf_counter()
        pend = []
        own = self.owner(self.x, edges_t) == rank
        pend.append(self._owned_first(own, self.x, self.z, 1, 1 + torch.arange(self.n, device=self.dev)))
        self.next_seq = max(self.next_seq, self.n + 1)
        for _ in range(ticks):
            g = torch.Generator(device=self.dev)
            g.manual_seed((self.seed * 1000003 + self.t) & 0x7FFFFFFFFFFFFFFF)
            sx = (2 * torch.rand(self.n, generator=g, device=self.dev, dtype=torch.float64) - 1).to(torch.float32)
            sz = (2 * torch.rand(self.n, generator=g, device=self.dev, dtype=torch.float64) - 1).to(torch.float32)
            order = torch.randperm(self.n, generator=g, device=self.dev)
            pos = torch.empty_like(order)
            pos[order] = torch.arange(self.n, device=self.dev)
            own = self.owner(self.x, edges_t) == rank
            nx = self.x + sx
            nz = self.z + sz
            pend.append(self._owned_first(own, nx, nz, 0, self.next_seq + pos))
            self.x, self.z = nx, nz
            self.next_seq += self.n
            self.t += 1
            if trace:
                torch.cuda.synchronize(self.dev) if self.dev.type == "cuda" else None
                print(f"[strip_ops rank {rank}] tick {self.t} at {time.perf_counter() - t0:.2f} s", file=sys.stderr,
                      flush=True)
        counts = torch.stack([c for _, c in pend]).cpu().tolist()  # the one host sync
        return [r[:c].clone() for (r, _), c in zip(pend, counts)]

    def _owned_first(self, own, x, z, kind, seq):
        """Records of every entity, the owned ones first in slot order (a stable sort of the
        ownership flag), and the owned count on the device."""
        torch = self.torch
        idx = torch.argsort((~own).to(torch.uint8), stable=True)
        return self._records(idx, x[idx], z[idx], kind, seq[idx]), own.sum()


class HostUniformWorkload:
    """Config 5 as DeviceUniformWorkload lays it out, generated on the host with numpy (bench
    only): the same shape (N uniform in [-L/2, L/2)^2, U(-1,1) steps per axis in float32, a
    random global call order per tick), another random stream.  For ranks that share one GPU
    (the gloo rehearsal): torch's generation kernels from several processes at once stalled the
    shared GPU for tens of seconds per tick there, and these records reach the GPU in one copy."""

    def __init__(self, n: int, seed: int):
        self.n = n
        self.L = math.sqrt(n * 1250.0)
        self.D = D_DEFAULT
        self.seed = seed
        rng = np.random.default_rng(seed)
        self.x = (rng.random(n) * self.L - self.L / 2).astype(np.float32)
        self.z = (rng.random(n) * self.L - self.L / 2).astype(np.float32)
        self.t = 0

    @staticmethod
    def _records(slots, x, z, kind, seq):
        r = np.empty((slots.size, 6), np.int32)
        r[:, 0] = slots.astype(np.int32)
        r[:, 1] = x.view(np.int32)
        r[:, 2] = z.view(np.int32)
        r[:, 3] = kind
        r[:, 4] = (seq & 0xFFFFFFFF).astype(np.uint32).view(np.int32)
        r[:, 5] = (seq >> 32).astype(np.int32)
        return r

    def strip_ops(self, edges: np.ndarray, rank: int, ticks: int):
        """The records of DeviceUniformWorkload.strip_ops (Enter ops of the starting strip, then each
        tick's Moved ops of the entities the strip owns before it), as numpy arrays."""
        e = np.asarray(edges, np.float32)
        own = np.searchsorted(e, self.x, side="right") == rank  # torch.bucketize(..., right=True)
        slots = np.nonzero(own)[0]
        out = [self._records(slots, self.x[slots], self.z[slots], 1, 1 + slots.astype(np.int64))]
        next_seq = self.n + 1
        for _ in range(ticks):
            rng = np.random.default_rng((self.seed * 1000003 + self.t) & 0x7FFFFFFFFFFFFFFF)
            sx = (2 * rng.random(self.n) - 1).astype(np.float32)
            sz = (2 * rng.random(self.n) - 1).astype(np.float32)
            order = rng.permutation(self.n)
            pos = np.empty(self.n, np.int64)
            pos[order] = np.arange(self.n)
            own = np.searchsorted(e, self.x, side="right") == rank
            nx = self.x + sx
            nz = self.z + sz
            slots = np.nonzero(own)[0]
            out.append(self._records(slots, nx[slots], nz[slots], 0, next_seq + pos[slots]))
            self.x, self.z = nx, nz
            next_seq += self.n
            self.t += 1
        return out
