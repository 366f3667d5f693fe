#!/usr/bin/env python3
"""Probe (GPU box): do two flushes on two streams overlap on this chip, and by how much?

Two config-3 worlds (1M entities each, own HIP stream each) run the bench's speculative tick loop
interleaved (world A finishes t and queues t+1, then world B), against world A alone.  If the pair
takes less than twice the single world's time per tick, kernels of one flush fill CUs the other
leaves idle (the combined pass's tail, the finish's serial blocks, the gap between flushes): the
bound on what overlapping a world's own consecutive flushes could win.
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from goworld_amd import World  # noqa: E402
from goworld_amd.workload import make_workload  # noqa: E402


def main():
    import torch
    ticks, warm = int(os.environ.get("OP_TICKS", "30")), 4
    wl = make_workload("cfg3")
    batches = [wl.tick(t) for t in range(ticks + warm)]
    d_s = torch.from_numpy(np.stack([b[0] for b in batches]).astype(np.int32)).to("cuda:0")
    d_x = torch.from_numpy(np.stack([b[1] for b in batches])).to("cuda:0")
    d_z = torch.from_numpy(np.stack([b[2] for b in batches])).to("cuda:0")
    rows = [(d_s[t].data_ptr(), d_x[t].data_ptr(), d_z[t].data_ptr(), batches[t][0].size) for t in range(ticks + warm)]
    init = make_workload("cfg3").initial()

    def world():
        w = World(wl.n, device=0, unique_moves=True)
        s = w.space_create(wl.D)
        w.enter_batch(s, init[0], init[1], init[2])
        w.tick_device()
        return w

    def run(ws):
        for w in ws:
            w.moved_batch_device(*rows[0])
            w.tick_begin()
        t0 = None
        for t in range(ticks + warm - 1):
            if t == warm:
                for w in ws:
                    w.sync()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            for w in ws:
                w.moved_batch_device(*rows[t + 1])
                w.tick_end_begin_device()
        for w in ws:
            w.tick_end_device()
            w.sync()
        return (time.perf_counter() - t0) / (ticks - 1) * 1e3

    a = world()
    one = run([a])
    b = world()
    two = run([a, b])
    one2 = run([a])
    print(f"one world: {one:.4f} / {one2:.4f} ms per tick; two worlds interleaved: {two:.4f} ms per tick "
          f"(both worlds' flushes), {two / 2:.4f} per flush; overlap gain {2 * min(one, one2) - two:.4f} ms per pair")


if __name__ == "__main__":
    main()
