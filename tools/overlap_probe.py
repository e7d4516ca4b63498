"""Diagnostic: the next-batch preparation alone, the training step alone (its batch
prepared beforehand), and both overlapped (the bench's steady state), in µs per step.

    python tools/overlap_probe.py [--iters 100]"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--workload", default="twitter15")
    args = ap.parse_args()
    import bench
    from bigcn_amd import BiGCN, FusedTrainStep, Net, _lib
    from bigcn_amd._lib import check, ptr, stream_handle
    from bigcn_amd.ops import _FEAT_MODES
    from bigcn_amd.optim import bigcn_adam
    dev = torch.device("cuda", 0)
    wl = bench.WORKLOADS[args.workload]
    pool = bench.make_pool(wl, 0, 4, dev)
    model = (BiGCN if wl["classes"] == 4 else Net)(wl["feats"], 64, 64, dev).to(dev)
    model.train()
    fused = FusedTrainStep(model, bigcn_adam(model))
    L = _lib.lib()
    stream = torch.cuda.Stream(dev)
    F = wl["feats"]

    def timed(fn, iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for i in range(iters):
            fn(i)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters * 1e3

    with torch.cuda.stream(stream):
        descs = [fused._desc(b) for b in pool]
        bufs = [fused._prep_buffer(d, F) for d, _ in descs]

        def prep(i):
            d, _ = descs[i % 4]
            check(L.bgcn_prepare_batch(d, F, 0, _FEAT_MODES["auto"], ptr(bufs[i % 4]), bufs[i % 4].numel(),
                                       stream_handle()))

        def step_alone_ready(iters):
            """the step on a batch prepared by the previous call, with no preparation of
            its own (events bracket only that call)"""
            tot = 0.0
            for i in range(iters):
                b, nb = pool[i % 4], pool[(i + 1) % 4]
                fused.forward_backward(b, seed=i, next_data=nb)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                fused.forward_backward(nb, seed=i)
                e1.record()
                torch.cuda.synchronize()
                tot += e0.elapsed_time(e1)
            return tot / iters * 1e3

        def step_inline(i):
            fused.forward_backward(pool[i % 4], seed=i)   # prepares its own batch, no next

        def step_overlapped(i):
            fused.forward_backward(pool[i % 4], seed=i, next_data=pool[(i + 1) % 4])

        for fn in (prep, step_inline, step_overlapped):
            fn(0)
        t_prep = timed(prep, args.iters)
        t_inline = timed(step_inline, args.iters)
        t_over = timed(step_overlapped, args.iters)
        t_ready = step_alone_ready(max(10, args.iters // 4))
    print(f"preparation alone {t_prep:.1f} us; step alone on a prepared batch {t_ready:.1f} us; "
          f"step preparing its own batch {t_inline:.1f} us; step + next-batch preparation "
          f"overlapped {t_over:.1f} us (no optimizer in any)")


if __name__ == "__main__":
    main()
