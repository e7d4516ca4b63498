"""Diagnostic: where the host time of one training step goes, on the GPU box.

    python tools/host_profile.py [--workload twitter15] [--steps 300] [--mode resident|host_fed|dropin]

resident: FusedTrainStep on a pool of resident batches (the bench's main loop); host_fed: the
same step fed by feed.host_fed_loader + DeviceFeeder (the bench's staging leg); dropin: the
reference loop body on the per-op modules.  Prints host us/step (enqueue only) and the wall
us/step, then cProfile's top functions by own time over the timed steps, with every native
libbgcn call wrapped so its host time shows as its own line."""
from __future__ import annotations

import argparse
import cProfile
import io
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def wrap_native():
    """Each libbgcn entry point behind a Python function of its own name (cProfile then
    reports the native host time per symbol)."""
    from bigcn_amd import _lib
    L = _lib.lib()
    for name in _lib.EXPORTED_SYMBOLS:
        f = getattr(L, name, None)
        if f is None:
            continue
        code = f"def {name}(*a, _f=_f):\n    return _f(*a)\n"
        ns = {"_f": f}
        exec(code, ns)
        setattr(L, name, ns[name])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="twitter15")
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--mode", default="resident", choices=["resident", "host_fed", "dropin"])
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--ahead", action="store_true", help="dropin: batches through feed.prepare_ahead")
    ap.add_argument("--loader", default="native", choices=["native", "dataloader"])
    ap.add_argument("--pre-timing", action="store_true", help="the kernel-timing hook on during the pre-fused steps")
    ap.add_argument("--reset", default="none", choices=["none", "alloc", "timing", "gc", "sync", "empty"],
                    help="dropin after --pre-fused: what runs between the two loops (the bench's "
                         "fresh_allocator = alloc; a kernel-timing enable/disable = timing)")
    ap.add_argument("--pre-fused", type=int, default=0,
                    help="dropin: first run this many fused steps on the same model / optimiser (as the bench does)")
    args = ap.parse_args()
    import bench
    import torch.nn.functional as F
    from bigcn_amd import BiGCN, FusedTrainStep, Net
    from bigcn_amd.optim import bigcn_adam
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    wl = bench.WORKLOADS[args.workload]
    model = (BiGCN if wl["classes"] == 4 else Net)(wl["feats"], 64, 64, dev).to(dev)
    model.train()
    opt = bigcn_adam(model)
    stream = torch.cuda.Stream(dev)
    wrap_native()
    if args.mode == "dropin":
        if args.pre_fused:
            fpool = bench.make_pool(wl, 0, 4, dev, (0.0, 0.0))
            fs = FusedTrainStep(model, opt, tddroprate=wl["drop"][0], budroprate=wl["drop"][1], drop_seed=7)
            from bigcn_amd import ops
            with torch.cuda.stream(stream):
                for i in range(args.pre_fused):
                    if args.pre_timing and i == 10:
                        torch.cuda.synchronize()
                        ops.set_kernel_timing(True, [7])
                    fs(fpool[i % 4], next_data=fpool[(i + 1) % 4])
                if args.pre_timing:
                    torch.cuda.synchronize()
                    ops.set_kernel_timing(False)
                    ops.kernel_timing(7)
                    ops.kernel_span(7)
                fs.discard_prefetch()
                torch.cuda.synchronize()
            del fs, fpool
            import gc
            if args.reset == "alloc":
                torch.cuda.synchronize(); gc.collect(); torch.cuda.empty_cache()
            elif args.reset == "empty":
                torch.cuda.synchronize(); torch.cuda.empty_cache()
            elif args.reset == "gc":
                gc.collect()
            elif args.reset == "sync":
                torch.cuda.synchronize()
            elif args.reset == "timing":
                ops.set_kernel_timing(True, [7]); ops.set_kernel_timing(False)
        pool = bench.make_pool(wl, 0, 4, dev, None)
        ahead = None
        if args.ahead:
            from bigcn_amd.feed import prepare_ahead
            ahead = iter(prepare_ahead((pool[i % 4] for i in range(args.warmup + 2 * args.steps + 1)), model))

        def step(i):
            b = next(ahead) if ahead is not None else pool[i % len(pool)]
            b.__dict__.pop("_bgcn_graphs", None)
            logp = model(b)
            loss = F.nll_loss(logp, b.y)
            opt.zero_grad()
            loss.backward()
            opt.step()
        it = None
    else:
        fused = FusedTrainStep(model, opt, tddroprate=wl["drop"][0], budroprate=wl["drop"][1], drop_seed=7)
        if args.mode == "resident":
            pool = bench.make_pool(wl, 0, 4, dev, (0.0, 0.0))

            def step(i):
                fused(pool[i % len(pool)], next_data=pool[(i + 1) % len(pool)])
            it = None
        else:
            from bigcn_amd import feed as FD
            store = FD.TreeStore.synthetic(2048, wl["mean"], seed=11, in_feats=wl["feats"],
                                           num_classes=wl["classes"])
            ep = (2 * args.steps + args.warmup) * wl["trees"] // 2048 + 3
            if args.loader == "native":
                loader = FD.NativeLoader(store, batch_size=wl["trees"], num_workers=5, seed=7, epochs=ep,
                                         bf16_values=wl.get("xdtype") == "bf16")
            else:
                loader = FD.host_fed_loader(store, batch_size=wl["trees"], num_workers=5, seed=7, epochs=ep,
                                            bf16_values=wl.get("xdtype") == "bf16")
            xdt = torch.bfloat16 if wl.get("xdtype") == "bf16" else torch.float32
            with torch.cuda.stream(stream):
                feeder = FD.DeviceFeeder(loader, dev, depth=3, x_dtype=xdt)
                it = iter(feeder)
                state = {"cur": next(it)}

            def step(i):
                nxt = next(it)
                fused(state["cur"], next_data=nxt)
                state["cur"] = nxt
    with torch.cuda.stream(stream):
        for i in range(args.warmup):
            step(i)
        torch.cuda.synchronize()
        prof = cProfile.Profile()
        t0 = time.perf_counter()
        prof.enable()
        for i in range(args.steps):
            step(i)
        prof.disable()
        th = time.perf_counter() - t0
        torch.cuda.synchronize()
        tw = time.perf_counter() - t0
        # the same loop without the profiler: the host's own rate
        t1 = time.perf_counter()
        for i in range(args.steps):
            step(i)
        th2 = time.perf_counter() - t1
        torch.cuda.synchronize()
        tw2 = time.perf_counter() - t1
    print(f"mode {args.mode} workload {args.workload}: unprofiled host {th2 / args.steps * 1e6:.1f} us/step, "
          f"wall {tw2 / args.steps * 1e6:.1f} us/step; profiled host {th / args.steps * 1e6:.1f}, "
          f"wall {tw / args.steps * 1e6:.1f}")
    s = io.StringIO()
    st = pstats.Stats(prof, stream=s)
    st.sort_stats("tottime").print_stats(args.top)
    print(s.getvalue())
    s = io.StringIO()
    st = pstats.Stats(prof, stream=s)
    st.sort_stats("cumulative").print_stats(args.top)
    print(s.getvalue())


if __name__ == "__main__":
    main()
