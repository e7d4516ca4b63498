"""Host time of each piece of the drop-in loop body over feed.prepare_ahead (the bench's
dropin_path.prepared_ahead leg), unprofiled: perf_counter brackets only.

    python tools/dropin_parts.py [--steps 300] [--inline]

Pieces: next() of the prepare_ahead iterator (the next batch's bgcn_prepare_batch queued on
the side stream), model(data), F.nll_loss, zero_grad, loss.backward() (the autograd engine:
NllLossBackward, the net's backward node - timed on its own inside - and ten AccumulateGrad),
opt.step().  --inline: the same loop preparing each batch in its own forward.
"""
import argparse
import collections
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--inline", action="store_true")
    a = ap.parse_args()
    import bench
    from bigcn_amd import BiGCN, ops
    from bigcn_amd.feed import prepare_ahead
    from bigcn_amd.optim import bigcn_adam
    dev = torch.device("cuda", 0)
    wl = bench.WORKLOADS["twitter15"]
    pool = bench.make_pool(wl, 0, 4, dev, None)
    model = BiGCN(wl["feats"], 64, 64, dev).to(dev)
    model.train()
    opt = bigcn_adam(model)
    acc = collections.defaultdict(float)
    bw = ops._BiGCNNetFn.backward

    def timed_bw(ctx, *g):
        t = time.perf_counter()
        r = bw(ctx, *g)
        acc["  net backward node (autograd thread)"] += time.perf_counter() - t
        return r
    ops._BiGCNNetFn.backward = staticmethod(timed_bw)
    n = a.warmup + a.steps
    src = (pool[i % 4] for i in range(n + 1))
    it = iter(src if a.inline else prepare_ahead(src, model))
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        for i in range(n):
            if i == a.warmup:
                torch.cuda.synchronize()
                acc.clear()
                t_start = time.perf_counter()
            t0 = time.perf_counter()
            b = next(it)
            if a.inline:
                b.__dict__.pop("_bgcn_graphs", None)
            t1 = time.perf_counter()
            logp = model(b)
            t2 = time.perf_counter()
            loss = F.nll_loss(logp, b.y)
            t3 = time.perf_counter()
            opt.zero_grad()
            t4 = time.perf_counter()
            loss.backward()
            t5 = time.perf_counter()
            opt.step()
            t6 = time.perf_counter()
            for k, d in (("next(batches)", t1 - t0), ("model(data)", t2 - t1), ("nll_loss", t3 - t2),
                         ("zero_grad", t4 - t3), ("backward", t5 - t4), ("opt.step", t6 - t5), ("total", t6 - t0)):
                acc[k] += d
        th = time.perf_counter() - t_start
        torch.cuda.synchronize()
        tw = time.perf_counter() - t_start
    print(f"{'inline' if a.inline else 'prepare_ahead'}: host {th / a.steps * 1e6:.1f} us/step, "
          f"wall {tw / a.steps * 1e6:.1f} us/step")
    for k, v in acc.items():
        print(f"{k:40s} {v / a.steps * 1e6:8.1f} us")


if __name__ == "__main__":
    main()
