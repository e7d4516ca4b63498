"""Diagnostic: host enqueue time vs device time of the bench training step.

    python tools/step_probe.py [--steps 50] [--null-stream]

Prints, per step: the host time to enqueue one step (no sync) and the wall time of
K steps; a step whose enqueue time exceeds its device time is host-bound."""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--null-stream", action="store_true")
    ap.add_argument("--path", default="fused", choices=["fused", "autograd"])
    ap.add_argument("--prefetch", type=int, default=1)
    ap.add_argument("--dropedge", default="device", choices=["device", "host"])
    args = ap.parse_args()
    import bench
    from bigcn_amd import BiGCN, FusedTrainStep
    from bigcn_amd.optim import bigcn_adam
    dev = torch.device("cuda", 0)
    wl = bench.WORKLOADS["twitter15"]
    dd = args.path == "fused" and args.dropedge == "device"
    pool = bench.make_pool(wl, 0, 4, dev, (0.0, 0.0) if dd else None)
    model = BiGCN(wl["feats"], 64, 64, dev).to(dev)
    model.train()
    opt = bigcn_adam(model)
    stream = torch.cuda.current_stream() if args.null_stream else torch.cuda.Stream(dev)
    torch.cuda.synchronize()

    drops = wl["drop"] if dd else (0.0, 0.0)
    fused = FusedTrainStep(model, opt, tddroprate=drops[0], budroprate=drops[1], drop_seed=1)

    def step(i):
        b = pool[i % len(pool)]
        if args.path == "fused":
            fused(b, next_data=pool[(i + 1) % len(pool)] if args.prefetch else None)
            return
        b.__dict__.pop("_bgcn_graphs", None)
        logp = model(b)
        loss = F.nll_loss(logp, b.y)
        opt.zero_grad()
        loss.backward()
        opt.step()

    from bigcn_amd import _lib
    L = _lib.lib()
    native = {"t": 0.0, "n": 0}
    raw = L.bgcn_train_step

    def timed(*a):
        t = time.perf_counter()
        rc = raw(*a)
        native["t"] += time.perf_counter() - t
        native["n"] += 1
        return rc
    L.bgcn_train_step = timed

    with torch.cuda.stream(stream):
        for i in range(5):
            step(i)
        torch.cuda.synchronize()
        native["t"], native["n"] = 0.0, 0
        host = []
        t0 = time.perf_counter()
        for i in range(args.steps):
            h0 = time.perf_counter()
            step(i)
            host.append(time.perf_counter() - h0)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
    host.sort()
    print(f"host enqueue per step: median {host[len(host)//2]*1e6:.1f} us, "
          f"mean {sum(host)/len(host)*1e6:.1f} us; loop {((t1-t0)/args.steps)*1e6:.1f} us/step; "
          f"wall incl. drain {((t2-t0)/args.steps)*1e6:.1f} us/step; "
          f"inside bgcn_train_step {native['t'] / max(native['n'], 1) * 1e6:.1f} us/call")


if __name__ == "__main__":
    main()
