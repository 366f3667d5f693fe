"""PCIe copy rates on the GPU box for the host->host tick's two transfers (12 B per move in, 8 B per
directed event out at config 3): H2D alone, D2H alone, and both at once on two streams.
usage: python tools/pcie_probe.py [h2d_MB] [d2h_MB]"""
import sys
import time

import torch


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t = []
    for _ in range(reps):
        a = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        t.append(time.perf_counter() - a)
    t.sort()
    return t[len(t) // 2] * 1e3


def main():
    h_mb = float(sys.argv[1]) if len(sys.argv) > 1 else 12.0
    d_mb = float(sys.argv[2]) if len(sys.argv) > 2 else 8.9
    hn, dn = int(h_mb * 2**20) // 4, int(d_mb * 2**20) // 4
    hsrc = torch.empty(hn, dtype=torch.int32).pin_memory()
    ddst = torch.empty(hn, dtype=torch.int32, device="cuda")
    dsrc = torch.empty(dn, dtype=torch.int32, device="cuda")
    hdst = torch.empty(dn, dtype=torch.int32).pin_memory()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def h2d():
        with torch.cuda.stream(s1):
            ddst.copy_(hsrc, non_blocking=True)

    def d2h():
        with torch.cuda.stream(s2):
            hdst.copy_(dsrc, non_blocking=True)

    def both():
        h2d()
        d2h()

    th, td, tb = timed(h2d), timed(d2h), timed(both)
    print(f"H2D {h_mb:.1f} MB: {th:.3f} ms ({h_mb / 1024 / th * 1e3:.1f} GB/s)")
    print(f"D2H {d_mb:.1f} MB: {td:.3f} ms ({d_mb / 1024 / td * 1e3:.1f} GB/s)")
    print(f"both at once: {tb:.3f} ms (sum {th + td:.3f}, max {max(th, td):.3f})")


if __name__ == "__main__":
    main()
