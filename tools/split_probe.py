"""Diagnostic: would splitting a 128-tree batch into P parts whose training chains run
concurrently on P streams shorten the step?  Each part has its own model copy, fused
step and prepared batch (reused, nothing on the side lane); before every iteration a
one-wave ALU spin holds stream 0 so the host has queued every chain before the first
kernel starts; the device span (spin end -> all chains done) is timed with events.

    python tools/split_probe.py [--steps 30]"""
from __future__ import annotations

import argparse
import ctypes
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--spin", type=int, default=60000)
    args = ap.parse_args()
    from bigcn_amd import BiGCN, FusedTrainStep
    from bigcn_amd.data import synth_batch, synth_tree_sizes
    from bigcn_amd.optim import bigcn_adam
    L = ctypes.CDLL(os.path.join(ROOT, "tools", "libinterfere.so"))
    dev = torch.device("cuda", 0)
    sizes = synth_tree_sizes(np.random.default_rng(5), 128, 256, 0.8)
    sink = torch.zeros(4, device=dev)
    for P in (1, 2, 4):
        parts = np.array_split(sizes, P)
        streams = [torch.cuda.Stream(dev) for _ in range(P)]
        chains = []
        for k in range(P):
            b = synth_batch(np.random.default_rng(7 + k), parts[k], 5000, 4, device=dev)
            m = BiGCN(5000, 64, 64, dev).to(dev)
            m.train()
            f = FusedTrainStep(m, bigcn_adam(m))
            with torch.cuda.stream(streams[k]):
                f(b, next_data=b)
                f(b, next_data=b)
            chains.append((f, b, f._pending))
        torch.cuda.synchronize()
        spans = []
        for it in range(args.steps):
            s0 = streams[0]
            L.ifr_alu(1, args.spin, ctypes.c_void_p(sink.data_ptr()), ctypes.c_void_p(s0.cuda_stream))
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(s0)
            for k in range(1, P):
                streams[k].wait_event(e0)
            for k, (f, b, pend) in enumerate(chains):
                with torch.cuda.stream(streams[k]):
                    f._pending = pend
                    f(b)
            for k in range(1, P):
                s0.wait_stream(streams[k])
            e1.record(s0)
            torch.cuda.synchronize()
            if it >= 3:
                spans.append(e0.elapsed_time(e1) * 1e3)
        print(f"P={P}: parts of {[int(p.sum()) for p in parts]} nodes: span median {statistics.median(spans):7.1f} us "
              f"(min {min(spans):7.1f})", flush=True)


if __name__ == "__main__":
    main()
