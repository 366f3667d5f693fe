"""CPU model of the incremental frame sort (gwaoi_kernels.hip k_scan64 / k_arrive /
k_cell_merge): the per-cell shift rule for stayers of unchanged cells plus the three-part layout
of changed cells must equal the stable sort of S' by the new cell keys.  The GPU kernels are checked
against the oracle by tests/test_gpu_parity.py; this test pins the rule they implement."""
import numpy as np
import pytest


def incremental_sort_model(p_key, key, n_cells, sentinel):
    n_prev = len(p_key)
    old = np.concatenate([p_key, np.full(len(key) - n_prev, sentinel)])
    pcs = np.searchsorted(p_key, np.arange(n_cells + 1))  # previous cell starts
    ch = key != old
    arr = np.bincount(key[ch & (key != sentinel)], minlength=n_cells + 1)[:n_cells + 1]
    dep = np.bincount(old[ch & (old != sentinel)], minlength=n_cells + 1)[:n_cells + 1]
    ea = np.concatenate([[0], np.cumsum(arr)])[:n_cells + 1]
    ed = np.concatenate([[0], np.cumsum(dep)])[:n_cells + 1]
    start = pcs + ea - ed                     # k_scan64: new cell_start
    changed = (arr | dep) != 0
    n_new = int((key != sentinel).sum())
    perm = np.full(n_new, -1)
    # k_arrive: a stayer of an unchanged cell keeps its rank, shifted by the cell's move
    for i in np.nonzero((key == old) & (key != sentinel))[0]:
        c = key[i]
        if not changed[c]:
            perm[i + start[c] - pcs[c]] = i
    # k_cell_merge: a changed cell is [arrivals below its previous run] [stayers] [arrivals past
    # it]: an arrival's S' index never lies inside the run (the run is exactly the entries whose
    # previous key is c), so the three parts are already in S' index order
    for c in np.nonzero(changed[:n_cells])[0]:
        stay = [i for i in range(pcs[c], pcs[c + 1]) if key[i] == c]
        arrivals = sorted(np.nonzero(ch & (key == c))[0].tolist())
        assert not any(pcs[c] <= v < pcs[c + 1] for v in arrivals)
        run = [v for v in arrivals if v < pcs[c]] + stay + [v for v in arrivals if v >= pcs[c + 1]]
        assert start[c] + len(run) == start[c + 1]
        perm[start[c]:start[c] + len(run)] = run
    return perm, start


@pytest.mark.parametrize("seed", range(8))
def test_shift_rule_is_the_stable_sort(seed):
    rng = np.random.default_rng(seed)
    C, n_prev, S = 400, 2500, 400
    p_key = np.sort(rng.integers(0, C, n_prev))
    n_app = int(rng.integers(0, 60))
    key = np.concatenate([p_key.copy(), rng.integers(0, C, n_app)])
    moved = rng.random(n_prev) < 0.05
    key[:n_prev][moved] = rng.integers(0, C, int(moved.sum()))
    left = rng.random(n_prev) < 0.01
    key[:n_prev][left] = S
    perm, start = incremental_sort_model(p_key, key, C, S)
    ref = np.argsort(np.where(key == S, C + 1, key), kind="stable")[:len(perm)]
    assert (perm == ref).all()
    assert (start == np.searchsorted(np.sort(key[key != S]), np.arange(C + 1))).all()
