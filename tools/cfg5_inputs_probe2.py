#!/usr/bin/env python3
"""DeviceUniformWorkload.strip_ops itself (GWAOI_INPUT_TRACE=1: per-tick times) in `procs`
processes sharing the GPU, without torch.distributed (diagnostics for the cfg5 rehearsal).

    python tools/cfg5_inputs_probe2.py [procs=1] [ticks=8] [gloo=0]
"""
import multiprocessing as mp
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def worker(rank, procs, ticks, gloo, port, q):
    os.environ["GWAOI_INPUT_TRACE"] = "1"
    import torch
    torch.cuda.set_device(0)
    if gloo:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=procs)
        dist.barrier()
    from goworld_amd.strips import even_edges
    from goworld_amd.workload import DeviceUniformWorkload
    dev = torch.device("cuda:0")
    t0 = time.perf_counter()
    wl = DeviceUniformWorkload(1 << 24, 0x5EED0005, dev)
    edges_t = torch.from_numpy(even_edges(procs, -wl.L / 2, wl.L / 2)).to(dev)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    ops = wl.strip_ops(edges_t, rank, ticks)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    q.put((rank, round(t1 - t0, 3), round(t2 - t1, 3), [int(o.shape[0]) for o in ops],
           round(torch.cuda.max_memory_allocated() / 2**30, 2)))


def main():
    procs = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    ticks = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    gloo = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, procs, ticks, gloo, port, q)) for r in range(procs)]
    for p in ps:
        p.start()
    res = [q.get(timeout=400) for _ in ps]
    for p in ps:
        p.join()
    for r in sorted(res):
        print(f"procs {procs} gloo {gloo}: rank {r[0]} positions {r[1]} s, strip_ops {r[2]} s, rows {r[3][:3]}..., "
              f"max mem {r[4]} GiB", flush=True)


if __name__ == "__main__":
    main()
