"""Diagnostic: the training chain alone (prepared batch reused, nothing on the side lane)
on batches of the same node count but different tree-size distributions - how much of
the chain's time follows the largest tree (per-tree readout blocks, long aggregation
rows of star roots) rather than the node count.

    python tools/shape_probe.py [--steps 100]"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--only", default=None, help="run only the shapes whose name contains this")
    args = ap.parse_args()
    from bigcn_amd import BiGCN, FusedTrainStep, ops
    from bigcn_amd.data import synth_batch, synth_tree_sizes
    from bigcn_amd.optim import bigcn_adam
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(5)
    ln = synth_tree_sizes(rng, 128, 256, 0.8)
    N = int(ln.sum())
    shapes = {
        "lognormal(0.8) mean 256": ln,
        "lognormal, 32 trees": ln[:32],
        "lognormal, 64 trees": ln[:64],
        "lognormal, 256 trees": np.concatenate([ln, synth_tree_sizes(np.random.default_rng(6), 128, 256, 0.8)]),
        "uniform 128 trees": np.full(128, N // 128),
        "lognormal, largest tree capped at 512": np.minimum(ln, 512),
        "one 4096-node tree + rest uniform": np.concatenate([[4096], np.full(127, (N - 4096) // 127)]),
    }
    model = BiGCN(5000, 64, 64, dev).to(dev)
    model.train()
    stream = torch.cuda.Stream(dev)
    for name, sizes in shapes.items():
        if args.only and args.only not in name:
            continue
        b = synth_batch(np.random.default_rng(7), sizes, 5000, 4, device=dev)
        fused = FusedTrainStep(model, bigcn_adam(model))
        with torch.cuda.stream(stream):
            fused(b, next_data=b)
            pend = fused._pending
            torch.cuda.synchronize()
            ops.set_kernel_timing(True, {9: "main"})
            for _ in range(args.steps):
                fused._pending = pend
                fused(b)
            torch.cuda.synchronize()
            ops.set_kernel_timing(False)
            ms, n = ops.kernel_timing(9)
        print(f"{name:40s} N={int(np.sum(sizes)):6d} max tree {int(np.max(sizes)):5d}: chain {ms / n * 1e3:7.1f} us",
              flush=True)


if __name__ == "__main__":
    main()
