"""CPU replay (numpy, config-3 frame at D/3 cells) of k_combined's flat-sweep row groups: per
wave, the groups of two rows of the merged strips and their 128-position chunks, as the kernel
runs them and with each lane's empty rows dropped first.
    python tools/sim_row_groups.py"""
import numpy as np, sys, os
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
exec(open(os.path.join(HERE, 'sim_sweep_slots.py')).read().split("print(\"rows Z mean")[0].replace("float(sys.argv[1]) if len(sys.argv) > 1 else 4", "3.0"))
# merged list per lane: X' rows below zr0, then Z rows
NXr = int(2 * c + 3)
lists = []
xe = np.minimum(xr1, zr0 - 1)
nx = np.maximum(xe - xr0 + 1, 0)
nzr = zr1 - zr0 + 1
R = NXr + 3
L = np.zeros((n, R), np.int64)
for q in range(NXr):
    v = q < nx
    L[:, q] = np.where(v, rowlen(np.minimum(xr0 + q, gz - 1), xc0, xc1, v), 0)
# append Z rows after the lane's X' rows: shift per lane
Zr = np.stack([rowlen(np.minimum(zr0 + q, gz - 1), zc0, zc1, zr0 + q <= zr1) for q in range(3)], 1)
M = np.zeros((n, R + 3), np.int64); nrows = nx + nzr
for i in range(3):
    idx = nx + i
    ok = i < nzr
    M[np.arange(n)[ok], idx[ok]] = Zr[ok, i]
M[:, :NXr] += L[:, :NXr]
W = n // 64
M = M[:W * 64].reshape(W, 64, -1); nrows = nrows[:W * 64].reshape(W, 64)
def stats(M, nrows):
    groups = (nrows.max(1) + 1) // 2
    G = M.shape[2] // 2
    T = M[:, :, 0:2 * G:2].sum(1) + M[:, :, 1:2 * G:2].sum(1)  # W x G
    chunks = np.ceil(T / 128.0)
    active = np.arange(G)[None, :] < groups[:, None]
    nonzero = (T > 0) & active
    return groups.sum(), nonzero.sum(), chunks.sum(), T.sum()
print("current  groups %d  nonempty groups %d  chunks %d  items %d" % stats(M, nrows))
# compacted: non-empty rows first (stable)
Mc = np.zeros_like(M)
nn = (M > 0).sum(2)
for wv in range(M.shape[0]):
    for l in range(64):
        r = M[wv, l][M[wv, l] > 0]
        Mc[wv, l, :r.size] = r
print("compact  groups %d  nonempty groups %d  chunks %d  items %d" % stats(Mc, nn))
