"""The AOIManager mirror over the GPU world: entity interest sets after
every flush equal the sequential oracle's neighbour sets, and In == By
(the symmetry TestCallAll checks)."""
import numpy as np
import pytest

from goworld_amd import aoi as A

pytestmark = pytest.mark.gpu


def test_entity_interest_matches_oracle(oracle_mod):
    rng = np.random.default_rng(77)
    n = 600
    D = [np.float32(100.0), np.float32(60.0)]
    with A.AOIWorld(n + 8, max_spaces=2) as W:
        mgrs = [W.new_xzlist_aoi_manager(d) for d in D]
        ents = [A.EntityInterest(i, 100.0) for i in range(n)]
        where = [None] * n
        orc = oracle_mod.SpacesOracle({0: D[0], 1: D[1]}, n + 8)
        pos = rng.uniform(-500, 500, (n, 2)).astype(np.float32)
        for tick in range(15):
            for i in rng.permutation(n).tolist():
                e = ents[i]
                r = rng.random()
                if where[i] is None:
                    if r < 0.7 or tick == 0:
                        s = int(rng.integers(2))
                        mgrs[s].enter(e.aoi, pos[i, 0], pos[i, 1])
                        where[i] = s
                        orc.enter(s, e.aoi.slot, pos[i, 0], pos[i, 1])
                elif r < 0.04:
                    mgrs[where[i]].leave(e.aoi)
                    orc.leave(e.aoi.slot)
                    where[i] = None
                elif r < 0.06:  # switch space (Space.leave + Space.enter)
                    mgrs[where[i]].leave(e.aoi)
                    orc.leave(e.aoi.slot)
                    s = 1 - where[i]
                    mgrs[s].enter(e.aoi, pos[i, 0], pos[i, 1])
                    orc.enter(s, e.aoi.slot, pos[i, 0], pos[i, 1])
                    where[i] = s
                else:
                    pos[i] += rng.uniform(-4, 4, 2).astype(np.float32)
                    mgrs[where[i]].moved(e.aoi, pos[i, 0], pos[i, 1])
                    orc.moved(e.aoi.slot, pos[i, 0], pos[i, 1])
            W.flush()
            orc.take_events()
            for i in range(n):
                e = ents[i]
                assert e.interested_in == e.interested_by
                if where[i] is None:
                    assert not e.interested_in
                    continue
                want = {ents_by_slot.data.id for ents_by_slot in
                        [W._by_slot[s] for s in orc.neighbors(e.aoi.slot).tolist()]}
                assert {o.id for o in e.interested_in} == want, (tick, i)
