"""Where the host-fed leg's time goes (round 6): per batch, the host
time of the feeder's next() and the device time of its H2D copy, for the native loader
(feed.NativeLoader, its copy kernel and the DMA-engine hipMemcpyAsync) and the torch
DataLoader form, with and without the training step; plus raw H2D copies of one batch's bytes
from differently page-locked host buffers.

    python tools/loader_probe.py [--steps 40]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def raw_copies(nbytes, reps=20):
    """H2D copies of nbytes from: torch pinned (hipHostMalloc), a registered aligned buffer,
    pageable memory.  host us per call and device ms per copy."""
    dev = torch.device("cuda")
    dst = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream()
    out = {}
    libc = ctypes.CDLL(None)
    libc.aligned_alloc.restype = ctypes.c_void_p
    libc.aligned_alloc.argtypes = [ctypes.c_size_t, ctypes.c_size_t]
    p = libc.aligned_alloc(4096, (nbytes + 4095) // 4096 * 4096)
    reg = torch.frombuffer((ctypes.c_uint8 * nbytes).from_address(p), dtype=torch.uint8)
    reg.fill_(1)
    rt = torch.cuda.cudart()
    assert int(rt.cudaHostRegister(p, (nbytes + 4095) // 4096 * 4096, 0)) == 0
    srcs = {"torch_pinned": torch.ones(nbytes, dtype=torch.uint8).pin_memory(),
            "aligned_registered": reg, "pageable": torch.ones(nbytes, dtype=torch.uint8)}
    for name, src in srcs.items():
        host, devms = [], []
        with torch.cuda.stream(s):
            for r in range(reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                t = time.perf_counter()
                dst.copy_(src, non_blocking=True)
                host.append((time.perf_counter() - t) * 1e6)
                b.record(s)
                b.synchronize()
                devms.append(a.elapsed_time(b))
        out[name] = {"is_pinned": bool(src.is_pinned()), "host_us_med": round(float(np.median(host)), 1),
                     "host_us_first": round(host[0], 1), "dev_ms_med": round(float(np.median(devms)), 4),
                     "dev_ms_first": round(devms[0], 4),
                     "gbs_med": round(nbytes / (float(np.median(devms)) * 1e-3) / 1e9, 2)}
    rt.cudaHostUnregister(p)
    return out


def feeder_run(store, native, steps, warmup, train, wl_trees=128):
    from bigcn_amd import feed as FD
    from bigcn_amd import BiGCN, FusedTrainStep
    dev = torch.device("cuda")
    epochs = (steps + warmup + 8) // (len(store) // wl_trees) + 2
    if native:
        loader = FD.NativeLoader(store, batch_size=wl_trees, num_workers=5, seed=7, epochs=epochs)
    else:
        loader = FD.host_fed_loader(store, batch_size=wl_trees, num_workers=5, seed=7, epochs=epochs)
    stream = torch.cuda.Stream()
    fused = None
    if train:
        torch.manual_seed(0)
        m = BiGCN(5000, 64, 64).to(dev)
        m.train()
        fused = FusedTrainStep(m, tddroprate=0.2, budroprate=0.2, drop_seed=3)
    per = []
    detail = []
    with torch.cuda.stream(stream):
        feeder = FD.DeviceFeeder(loader, dev, depth=3, timing=True)
        if native:   # per-call host times of the feeder's pieces
            take0, nxt0, wait0 = feeder._take, loader.next_into, loader.wait

            def take(n, _f=take0):
                t = time.perf_counter()
                k = len(feeder._free)
                r = _f(n)
                detail.append(("take", round((time.perf_counter() - t) * 1e3, 3), k, r[1] is None))
                return r

            def next_into(*a, _f=nxt0):
                t = time.perf_counter()
                r = _f(*a)
                detail.append(("next_into", round((time.perf_counter() - t) * 1e3, 3)))
                return r

            def wait(_f=wait0):
                t = time.perf_counter()
                r = _f()
                detail.append(("wait", round((time.perf_counter() - t) * 1e3, 3)))
                return r
            feeder._take, loader.next_into, loader.wait = take, next_into, wait
        it = iter(feeder)
        t = time.perf_counter()
        cur = next(it)
        first = (time.perf_counter() - t) * 1e3
        for i in range(warmup + steps):
            t = time.perf_counter()
            nxt = next(it)
            tn = (time.perf_counter() - t) * 1e3
            t = time.perf_counter()
            if fused is not None:
                fused(cur, next_data=nxt)
            tc = (time.perf_counter() - t) * 1e3
            per.append((round(tn, 3), round(tc, 3)))
            cur = nxt
        torch.cuda.synchronize()
        if fused is not None:
            fused.discard_prefetch()
    copies = [round(a.elapsed_time(b), 4) for a, b in feeder._events]
    st = loader.stats() if native else None
    del cur, nxt, it, feeder
    if native:
        loader.close()
    else:
        loader.dataset.ring.close()
    return {"native": native, "train": train, "first_next_ms": round(first, 3), "next_ms": [p[0] for p in per],
            "step_call_ms": [p[1] for p in per], "copy_ms": copies, "loader_stats": st,
            "detail": [d for d in detail if d[0] != "take" or d[1] > 0.3 or not d[3]] if native else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--copies", default="kernel,sdma", help="the native loader's H2D copy forms (BGCN_LOADER_COPY)")
    args = ap.parse_args()
    from bigcn_amd import feed as FD
    store = FD.TreeStore.synthetic(2048, 256, seed=20250205 + 9, in_feats=5000, num_classes=4)
    res = {"raw": raw_copies(4_500_000)}
    for copy in args.copies.split(","):
        os.environ["BGCN_LOADER_COPY"] = copy            # read by bgcn_loader_create
        for train in (False, True):
            r = feeder_run(store, True, args.steps, args.warmup, train)
            r["copy"] = copy
            res[f"native_{copy}_{'train' if train else 'copyonly'}"] = r
    os.environ.pop("BGCN_LOADER_COPY", None)
    for train in (False, True):
        res[f"dataloader_{'train' if train else 'copyonly'}"] = feeder_run(store, False, args.steps, args.warmup, train)
    res["raw_after"] = raw_copies(4_500_000)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
