"""CPU replay (numpy) of k_combined's X' row trimming by per-cell x bounds on the config-3 frame:
candidates per entity in the X' rows with and without trimming the end cells whose entries all
lie outside the band, at D/4 and D/2 cells.

    python tools/sim_cell_bounds.py
"""
import numpy as np, sys
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from goworld_amd.workload import make_workload
W = make_workload("cfg3")
x, z = W.x.astype(np.float64), W.z.astype(np.float64)
D = 100.0
for c in (4, 2):
    cell = D / c
    lo, hi = D - 2.0, D + 2.0
    ox, oz = x.min(), z.min()
    gx = int((x.max() - ox) // cell) + 1; gz = int((z.max() - oz) // cell) + 1
    cx = ((x - ox) // cell).astype(np.int64); cz = ((z - oz) // cell).astype(np.int64)
    key = cz * gx + cx
    order = np.argsort(key, kind='stable')
    key_s = key[order]; xs = x[order]; zs = z[order]
    ncell = gx * gz
    cnt = np.bincount(key_s, minlength=ncell + 1)
    cs = np.concatenate([[0], np.cumsum(cnt)])
    xmin = np.full(ncell + 1, np.inf); xmax = np.full(ncell + 1, -np.inf)
    np.minimum.at(xmin, key_s, xs); np.maximum.at(xmax, key_s, xs)
    def cellx(v): return np.clip(((v - ox) // cell).astype(np.int64), 0, gx - 1)
    def cellz(v): return np.clip(((v - oz) // cell).astype(np.int64), 0, gz - 1)
    n = len(xs)
    zr0 = cellz(zs + lo)
    xr0, xr1 = cellz(zs - lo), np.minimum(cellz(zs + lo), zr0 - 1)
    xc0, xc1 = cellx(xs + lo), cellx(xs + hi)
    tot = 0; trim = 0; rows=0; rows_t=0
    for q in range(int(2 * c + 3)):
        r = xr0 + q; v = r <= xr1
        b = np.minimum(r, gz - 1) * gx
        c0 = b + xc0; c1 = b + xc1
        L = np.where(v, cs[c1 + 1] - cs[c0], 0)
        # trim left end cell(s): c0 if xmax < xs+lo ; right end c1 if xmin > xs+hi
        s0 = c0.copy(); e1 = c1.copy()
        dropl = v & (xmax[s0] < xs + lo); s0 = np.where(dropl, s0 + 1, s0)
        dropr = v & (s0 <= e1) & (xmin[e1] > xs + hi); e1 = np.where(dropr, e1 - 1, e1)
        Lt = np.where(v & (s0 <= e1), cs[np.maximum(e1, s0 - 1) + 1] - cs[s0], 0)
        tot += L.sum(); trim += Lt.sum(); rows += (v & (L > 0)).sum(); rows_t += (v & (Lt > 0)).sum()
    # Z rows
    zr1 = cellz(zs + hi); zc0, zc1 = cellx(xs - hi), cellx(xs + hi)
    ztot = 0
    for q in range(4):
        r = zr0 + q; v = r <= zr1
        b = np.minimum(r, gz - 1) * gx
        ztot += np.where(v, cs[b + zc1 + 1] - cs[b + zc0], 0).sum()
    print(f"c={c}: X' cand/entity {tot/n:.1f} -> trimmed {trim/n:.1f} ({100*(1-trim/tot):.0f}% fewer); nonempty X' rows/entity {rows/n:.2f} -> {rows_t/n:.2f}; Z cand/entity {ztot/n:.1f}")
