"""CPU replay of k_combined's sweep structure on the config-3 frame (numpy, no GPU):
lane-slots the lock-step sweep loads per entity against the candidates it needs, the
flat sweep's slots per row grouping, and the block schedule's makespan in frame order
against heaviest-first (the tail that k_tile_order removes).

    python tools/sim_sweep_slots.py [cells_per_dist=4]
"""
import numpy as np, sys
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from goworld_amd.workload import make_workload
W = make_workload("cfg3")
x, z = W.x.astype(np.float64), W.z.astype(np.float64)
D = 100.0; c = float(sys.argv[1]) if len(sys.argv) > 1 else 4
cell = D / c
lo, hi = D - 2.0, D + 2.0
ox, oz = x.min(), z.min()
gx = int((x.max() - ox) // cell) + 1; gz = int((z.max() - oz) // cell) + 1
cx = ((x - ox) // cell).astype(np.int64); cz = ((z - oz) // cell).astype(np.int64)
key = cz * gx + cx
order = np.argsort(key, kind='stable')
key_s = key[order]; xs = x[order]; zs = z[order]
cnt = np.bincount(key_s, minlength=gx * gz + 1)
cs = np.concatenate([[0], np.cumsum(cnt)])
def cellx(v): return np.clip(((v - ox) // cell).astype(np.int64), 0, gx - 1)
def cellz(v): return np.clip(((v - oz) // cell).astype(np.int64), 0, gz - 1)
n = len(xs)
# Z strip rows
zr0, zr1 = cellz(zs + lo), cellz(zs + hi)
zc0, zc1 = cellx(xs - hi), cellx(xs + hi)
xr0, xr1 = cellz(zs - lo), cellz(zs + lo)
xc0, xc1 = cellx(xs + lo), cellx(xs + hi)
def rowlen(r, c0, c1, valid):
    b = r * gx
    L = cs[b + c1 + 1] - cs[b + c0]
    return np.where(valid, L, 0)
NZ = 3; NX = int(2 * c + 3)
Zl = np.stack([rowlen(np.minimum(zr0 + q, gz - 1), zc0, zc1, zr0 + q <= zr1) for q in range(NZ)], 1)
Xl = np.stack([rowlen(np.minimum(xr0 + q, gz - 1), xc0, xc1, xr0 + q <= xr1) for q in range(NX)], 1)
print("rows Z mean %.2f  X mean %.2f" % ((zr1 - zr0 + 1).mean(), (xr1 - xr0 + 1).mean()))
useful = Zl.sum() + Xl.sum()
print("candidates per entity: Z %.1f X' %.1f" % (Zl.sum() / n, Xl.sum() / n))
# class perm inside 256-blocks
cls = ((zr1 > zr0).astype(int)) | ((xc1 > xc0).astype(int) << 1)
perm = np.arange(n)
for b0 in range(0, n, 256):
    seg = np.arange(b0, min(b0 + 256, n))
    perm[b0:b0 + len(seg)] = seg[np.argsort(cls[seg], kind='stable')]
Zl = Zl[perm]; Xl = Xl[perm]
nw = n // 64
Zw = Zl[:nw * 64].reshape(nw, 64, NZ); Xw = Xl[:nw * 64].reshape(nw, 64, NX)
slots = 0
# Z: per row, U=4 if any len>2 else 2 if any len>0
for q in range(NZ):
    m = Zw[:, :, q].max(1)
    U = np.where(m > 2, 4, 2)
    slots += (np.ceil(m / U) * U * 64).sum()
# X': pairs of rows as one virtual range
for q in range(0, NX, 2):
    tot = Xw[:, :, q:q + 2].sum(2)
    m = tot.max(1)
    U = np.where(m > 2, 4, 2)
    slots += (np.ceil(m / U) * U * 64).sum()
print("lockstep lane-slots per entity %.1f, useful %.1f, efficiency %.2f" % (slots / n, useful / n, useful / slots))
# flattened: per wave ceil(total/64) chunks
T = Zw.sum((1, 2)) + Xw.sum((1, 2))
print("flattened chunks slots per entity %.1f" % ((np.ceil(T / 64) * 64).sum() / n))
# per-lane single virtual sequence (all rows), lanes sorted by total within block
tl = (Zl.sum(1) + Xl.sum(1))
print("single virtual range, no sort: %.1f" % ((tl[:nw*64].reshape(nw,64).max(1)*64).sum()/n))
ts = tl.copy()
for b0 in range(0, n, 256):
    ts[b0:b0+256] = np.sort(ts[b0:b0+256])
print("single virtual range, block-sorted by total: %.1f" % ((ts[:nw*64].reshape(nw,64).max(1)*64).sum()/n))
def flat_slots(P_x, G, zP=2):
    s = 0
    Zs = Zw[:, :, :zP].sum(2).sum(1)  # all Z rows (<=2) as one group
    s += (np.ceil(Zs / G) * G).sum()
    for q in range(0, NX, P_x):
        t = Xw[:, :, q:q + P_x].sum(2).sum(1)
        s += (np.ceil(t / G) * G).sum()
    return s / n
for Px in (2, 3, 4, 5, 9, 11):
    print("flat X' P=%d: slots/entity G=128: %.1f  G=64: %.1f" % (Px, flat_slots(Px, 128), flat_slots(Px, 64)))
TT = Zw.sum((1,2)) + Xw.sum((1,2))
print("one group all: G=128 %.1f" % ((np.ceil(TT/128)*128).sum()/n))
print("X' groups count per wave (P=2): %.1f" % (np.ceil(NX/2)))
import heapq
# per-wave iterations under flat (Z group + X' groups of 2), G=128
it = np.ceil(Zw[:, :, :2].sum(2).sum(1) / 128)
for q in range(0, NX, 2):
    it += np.ceil(Xw[:, :, q:q + 2].sum(2).sum(1) / 128)
wave_t = 6 + it  # overhead in iteration units
nt = nw // 4
blk = wave_t[:nt * 4].reshape(nt, 4).max(1)
def makespan(order_fn, slots=224):
    q = nt // 8; r = nt % 8; tot = 0; worst = 0
    for x in range(8):
        lo = x * q + min(x, r); hi = lo + q + (1 if x < r else 0)
        d = blk[lo:hi]
        d = order_fn(d)
        h = [0.0] * slots
        for v in d:
            t = heapq.heappop(h); heapq.heappush(h, t + v)
        worst = max(worst, max(h))
        tot += d.sum()
    return worst, tot / (8 * slots)
for name, fn in [("frame order", lambda d: d), ("heavy first", lambda d: np.sort(d)[::-1])]:
    w, ideal = makespan(fn)
    print("%s: makespan %.1f ideal %.1f eff %.2f" % (name, w, ideal, ideal / w))
print("block work: mean %.1f max %.1f p90 %.1f" % (blk.mean(), blk.max(), np.percentile(blk, 90)))
def makespan_w(d_all, order_fn, slots):
    nt_ = len(d_all); q = nt_ // 8; r = nt_ % 8; worst = 0; tot = 0
    for x in range(8):
        lo = x * q + min(x, r); hi = lo + q + (1 if x < r else 0)
        d = order_fn(d_all[lo:hi]); h = [0.0] * slots
        for v in d:
            t = heapq.heappop(h); heapq.heappush(h, t + v)
        worst = max(worst, max(h)); tot += d.sum()
    return worst, tot / (8 * slots)
for name, fn in [("frame order", lambda d: d), ("heavy first", lambda d: np.sort(d)[::-1])]:
    w, ideal = makespan_w(wave_t, fn, 896)
    print("wave tiles %s: makespan %.1f ideal %.1f eff %.2f" % (name, w, ideal, ideal / w))
print("wave work: mean %.1f max %.1f" % (wave_t.mean(), wave_t.max()))
# 128-entity tiles (2 waves)
b2 = wave_t[:nw//2*2].reshape(-1, 2).max(1)
for name, fn in [("frame order", lambda d: d), ("heavy first", lambda d: np.sort(d)[::-1])]:
    w, ideal = makespan_w(b2, fn, 448)
    print("2-wave tiles %s: makespan %.1f ideal %.1f eff %.2f" % (name, w, ideal, ideal / w))
