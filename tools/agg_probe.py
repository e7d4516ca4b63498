"""Diagnostic: the 5000-wide aggregation A_hat . X against plain streaming kernels
(device copy, read-only reduction) on the same bytes, one bench pool batch.

    python tools/agg_probe.py [--iters 20]"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--graphs", default="self,chain,td,bu", help="comma list of self,chain,td,bu")
    ap.add_argument("--no-streams", action="store_true", help="skip the copy / colsum / fill lines")
    args = ap.parse_args()
    import bench
    from bigcn_amd import ops
    dev = torch.device("cuda", 0)
    wl = bench.WORKLOADS["twitter15"]
    b = bench.make_pool(wl, 0, 1, dev)[0]
    x = b.x
    N, F = x.shape
    nb = N * F * 4
    y = torch.empty_like(x)
    print(f"N={N} F={F} X={nb / 1e6:.0f} MB")
    if not args.no_streams:
        ms = timed(lambda: y.copy_(x), args.iters)
        print(f"copy      {ms * 1e3:8.1f} us  {2 * nb / ms / 1e6:7.0f} GB/s (read+write)")
        s = torch.empty(F, device=dev)
        ms = timed(lambda: torch.sum(x, 0, out=s), args.iters)
        print(f"colsum    {ms * 1e3:8.1f} us  {nb / ms / 1e6:7.0f} GB/s (read)")
        ms = timed(lambda: y.fill_(1.0), args.iters)
        print(f"fill      {ms * 1e3:8.1f} us  {nb / ms / 1e6:7.0f} GB/s (write)")
    # structure probes on the same X: self loops only (a copy through the kernel) and
    # chains (every parent re-read by the very next row: ideal reuse distance)
    ptr = b.ptr.tolist()
    ch_r = torch.cat([torch.arange(ptr[i], ptr[i + 1] - 1) for i in range(len(ptr) - 1)])
    probes = [("self", torch.zeros(2, 0, dtype=torch.int64, device=dev)),
              ("chain", torch.stack([ch_r, ch_r + 1]).to(dev))]
    want = set(args.graphs.split(","))
    for name, ei in probes + [("td", b.edge_index), ("bu", b.BU_edge_index)]:
        if name not in want:
            continue
        g = ops.build_graph(ei, N)
        ms = timed(lambda: ops.spmm(g, x, out=y), args.iters)
        alg = 2.0 * nb
        print(f"spmm {name}   {ms * 1e3:8.1f} us  {alg / ms / 1e6:7.0f} GB/s algorithmic "
              f"(E={ei.size(1)})")


if __name__ == "__main__":
    main()
