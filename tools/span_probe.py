"""Diagnostic: durations of the bgcn_train_step spans (timing classes 8-10): the next
batch's preparation on the auxiliary lane, the caller stream's own chain, the whole
call - averaged over K bench steps.  A preparation span close to the step span means the
side lane bounds the step.

    python tools/span_probe.py [--steps 200] [--dropedge host|device]"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--dropedge", default="host", choices=["device", "host"])
    ap.add_argument("--workload", default="twitter15")
    args = ap.parse_args()
    import bench
    from bigcn_amd import BiGCN, FusedTrainStep, ops
    from bigcn_amd.optim import bigcn_adam
    dev = torch.device("cuda", 0)
    wl = bench.WORKLOADS[args.workload]
    dd = args.dropedge == "device"
    pool = bench.make_pool(wl, 0, 4, dev, (0.0, 0.0) if dd else None)
    model = BiGCN(wl["feats"], 64, 64, dev).to(dev)
    model.train()
    opt = bigcn_adam(model)
    drops = wl["drop"] if dd else (0.0, 0.0)
    fused = FusedTrainStep(model, opt, tddroprate=drops[0], budroprate=drops[1], drop_seed=1)
    stream = torch.cuda.Stream(dev)
    with torch.cuda.stream(stream):
        for i in range(5):
            fused(pool[i % 4], next_data=pool[(i + 1) % 4])
        torch.cuda.synchronize()
        classes = {7: "compaction", 8: "prep span (side lane)", 9: "main chain span", 10: "whole call"}
        ops.set_kernel_timing(True, classes)
        for i in range(args.steps):
            fused(pool[i % 4], next_data=pool[(i + 1) % 4])
        torch.cuda.synchronize()
        ops.set_kernel_timing(False)
        for c, name in classes.items():
            ms, n = ops.kernel_timing(c)
            print(f"{name:24s} {ms / max(n, 1) * 1e3:8.1f} us  ({n} spans)")
        # host side: time spent inside the enqueueing call vs wall time per step (no
        # timing hook): a call time close to the step time means the step is host-bound
        import time
        torch.cuda.synchronize()
        host = 0.0
        t0 = time.perf_counter()
        for i in range(args.steps):
            h0 = time.perf_counter()
            fused(pool[i % 4], next_data=pool[(i + 1) % 4])
            host += time.perf_counter() - h0
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        print(f"{'host call (enqueue)':24s} {host / args.steps * 1e6:8.1f} us")
        print(f"{'wall per step':24s} {wall / args.steps * 1e6:8.1f} us")
        # the chain alone: batch 0 prepared once, every step reuses its prepared buffer
        # (no preparation on the side lane, so no HBM contention from the pass over X)
        fused(pool[3], next_data=pool[0])
        pend = fused._pending
        torch.cuda.synchronize()
        ops.set_kernel_timing(True, {9: "main", 10: "whole"})
        t0 = time.perf_counter()
        for i in range(args.steps):
            fused._pending = pend
            fused(pool[0])
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        ops.set_kernel_timing(False)
        for c, name in ((9, "chain alone: main span"), (10, "chain alone: whole call")):
            ms, n = ops.kernel_timing(c)
            print(f"{name:24s} {ms / max(n, 1) * 1e3:8.1f} us  ({n} spans)")
        print(f"{'chain alone: wall/step':24s} {wall / args.steps * 1e6:8.1f} us")
        # interference probes: the chain beside (a) a spin kernel (queue only, no memory),
        # (b) one big device copy of X (HBM only, one kernel) on another stream
        side = torch.cuda.Stream(dev)
        xs = pool[1].x
        ys = torch.empty_like(xs)
        small_x, small_y = xs[:1600].clone(), torch.empty_like(xs[:1600])    # 32 MB
        colsum = torch.empty(xs.size(1), device=dev)

        def small_copies():
            for _ in range(18):
                small_y.copy_(small_x)

        for name, job in (("spin", lambda: torch.cuda._sleep(600000)), ("copy X", lambda: ys.copy_(xs)),
                          ("read X", lambda: torch.sum(xs, 0, out=colsum)), ("fill Y", lambda: ys.fill_(1.0)),
                          ("32MB copy x18", small_copies)):
            torch.cuda.synchronize()
            ops.set_kernel_timing(True, {9: "main"})
            for i in range(args.steps):
                side.wait_stream(stream)
                with torch.cuda.stream(side):
                    job()
                fused._pending = pend
                fused(pool[0])
                stream.wait_stream(side)
            torch.cuda.synchronize()
            ops.set_kernel_timing(False)
            ms, n = ops.kernel_timing(9)
            print(f"{'chain beside ' + name:24s} {ms / max(n, 1) * 1e3:8.1f} us  ({n} spans)")


if __name__ == "__main__":
    main()
