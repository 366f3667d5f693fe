#!/usr/bin/env python3
"""Where the cfg5 input generation spends its time (GPU box): the ops of
DeviceUniformWorkload.strip_ops one by one with a synchronize after each, for one tick of 2^24
entities, in `procs` processes sharing the GPU at once (the gloo rehearsal's situation).

    python tools/cfg5_inputs_probe.py [procs=1] [n=16777216] [gloo=0]
"""
import multiprocessing as mp
import sys
import time


def worker(rank, procs, n, q, gloo=0, port=0):
    import os
    import torch
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    if gloo:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=procs)
        dist.barrier()
    t = {}

    def mark(name, t0):
        torch.cuda.synchronize()
        t[name] = round(time.perf_counter() - t0, 4)
        return time.perf_counter()

    a = time.perf_counter()
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    a = mark("generator", a)
    x = (torch.rand(n, generator=g, device=dev, dtype=torch.float64) * 1000).to(torch.float32)
    a = mark("rand_f64", a)
    for k in range(2):
        g2 = torch.Generator(device=dev)
        g2.manual_seed(7 + k)
        a = mark(f"generator_{k}", a)
        o2 = torch.randperm(n, generator=g2, device=dev)
        a = mark(f"randperm_{k}", a)
    sx = (2 * torch.rand(n, generator=g, device=dev, dtype=torch.float64) - 1).to(torch.float32)
    a = mark("rand_f64_2", a)
    order = torch.randperm(n, generator=g, device=dev)
    a = mark("randperm", a)
    pos = torch.empty_like(order)
    pos[order] = torch.arange(n, device=dev)
    a = mark("scatter_pos", a)
    edges = torch.tensor([-1e9, 250.0, 500.0, 750.0, 1e9], device=dev)
    own = torch.bucketize(x, edges, right=True) == (rank % 4)
    a = mark("bucketize", a)
    idx = torch.argsort((~own).to(torch.uint8), stable=True)
    a = mark("argsort_stable", a)
    r = torch.empty((n, 6), dtype=torch.int32, device=dev)
    r[:, 0] = idx.to(torch.int32)
    r[:, 1] = (x + sx)[idx].view(torch.int32)
    r[:, 3] = 0
    r[:, 4] = (pos[idx] & 0xFFFFFFFF).to(torch.int32)
    a = mark("records", a)
    c = int(own.sum())
    a = mark("count_sync", a)
    q.put((rank, t, c))


def main():
    procs = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 24
    gloo = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, procs, n, q, gloo, port)) for r in range(procs)]
    t0 = time.perf_counter()
    for p in ps:
        p.start()
    res = [q.get(timeout=600) for _ in ps]
    for p in ps:
        p.join()
    for rank, t, c in sorted(res):
        print(f"procs {procs} rank {rank}: {t} (owned {c})", flush=True)
    print(f"procs {procs}: wall {time.perf_counter() - t0:.1f} s", flush=True)


if __name__ == "__main__":
    main()
