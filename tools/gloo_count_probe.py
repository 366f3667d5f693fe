#!/usr/bin/env python3
"""Cost of strips.exchange's per-tick count all-gather over gloo (host tensors, no GPU):
`ws` processes on 127.0.0.1 all-gather the count row of an S=ws strip tick (7 S + 1 int64:
counts, teleports, ENTER / LEAVE counts, ENTER boxes) `iters` times; per iteration the time is
the slowest rank's.  Prints p50 / p90 / p99 / max in microseconds.

    python tools/gloo_count_probe.py [ws=8] [iters=3000]
"""
import json
import os
import socket
import sys
import time

import numpy as np


def worker(rank, ws, port, iters, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    row = torch.arange(7 * ws + 1, dtype=torch.int64) + rank
    rows = [torch.empty_like(row) for _ in range(ws)]
    for _ in range(50):  # warm the connections
        dist.all_gather(rows, row)
    dist.barrier()
    t = np.empty(iters)
    for i in range(iters):
        a = time.perf_counter()
        dist.all_gather(rows, row)
        t[i] = time.perf_counter() - a
    q.put((rank, t))
    dist.destroy_process_group()


def main():
    import multiprocessing as mp
    ws = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, ws, port, iters, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=600) for _ in range(ws))
    for p in procs:
        p.join()
    t = np.max(np.stack([res[r] for r in range(ws)]), axis=0) * 1e6  # slowest rank per iteration
    out = {"ws": ws, "iters": iters, "row_int64": 7 * ws + 1, "host_cpus": os.cpu_count(),
           "p50_us": round(float(np.percentile(t, 50)), 1), "p90_us": round(float(np.percentile(t, 90)), 1),
           "p99_us": round(float(np.percentile(t, 99)), 1), "max_us": round(float(t.max()), 1),
           "mean_us": round(float(t.mean()), 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
