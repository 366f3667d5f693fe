"""Debug helper: run a sync scenario on the GPU and print the first mismatch in detail."""
import sys
import numpy as np
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
import sync_scenario as SS
from oracle import oracle
from goworld_amd import World, pair_keys

seed, n, flushes, devmode = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4] == "dev"
sc = SS.make(seed=seed, n=n, flushes=flushes)
exp = []
def on_flush_o(i, g):
    ent, lev = oracle.net_events(*g.take_raw())
    exp.append((ent, lev))
    g.collect()
SS.run_oracle(sc, on_flush_o)
import torch
def dev(b):
    t = torch.frombuffer(bytearray(b), dtype=torch.uint8).to("cuda:0")
    torch.cuda.synchronize()
    return t.data_ptr(), t
bad = []
def on_flush(i, w, ent=None, lev=None):
    if ent is None:
        w.collect_sync_infos(); return
    ge, gl = pair_keys(ent), pair_keys(lev)
    oe, ol = exp[i]
    for name, g, o in (("enter", ge, oe), ("leave", gl, ol)):
        extra = np.setdiff1d(g, o); miss = np.setdiff1d(o, g)
        if extra.size or miss.size:
            print(f"flush {i} {name}: gpu {g.size} oracle {o.size} extra {[(int(k>>32), int(k&0xffffffff)) for k in extra[:20]]} missing {[(int(k>>32), int(k&0xffffffff)) for k in miss[:20]]}")
            bad.append(i)
    w.collect_sync_infos()
with World(sc["n"], max_spaces=4, device=0) as w:
    SS.run_gpu(sc, w, on_flush, dev if devmode else None)
if bad:
    f = bad[0]
    slots = set()
    print("ops of flush", f)
    for op in sc["flushes"][f - 1]:
        if op[0] != "packet":
            print("  ", op[0], op[1])
print("bad flushes", sorted(set(bad)))
