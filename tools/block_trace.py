"""Diagnostic: per-wave lifetimes of the training chain's kernels (chain alone, prepared
batch reused; --in-step: with the next batch's preparation beside it) from a -DBGCN_BLOCK_TRACE build of libbgcn (bgcn_trace.h):

    make -C bigcn_amd/csrc OUT=../../build/variants/libbgcn_bt.so OBJDIR=../../build/obj_bt \\
         EXTRA=-DBGCN_BLOCK_TRACE
    BGCN_LIB=build/variants/libbgcn_bt.so python tools/block_trace.py

Per instrumented kernel (id): waves recorded, the span from its first wave's start to its
last wave's end, when its last wave started, and wave lifetimes (p50 / p90 / max), all in
us of the device's constant-rate clock (100 MHz)."""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
NAMES = {1: "conv1_gather", 2: "conv2_sparse", 3: "spmm chunks", 4: "spmm long rows", 5: "readout_fwd",
         6: "readout_bwd", 70: "bwd_mid dW2 blk", 71: "bwd_mid root part", 72: "bwd_mid dH1",
         73: "bwd_mid db2", 80: "bwd_tail dW1", 81: "bwd_tail rootcols", 82: "bwd_tail dW2 red",
         83: "bwd_tail db1"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="twitter15")
    ap.add_argument("--mhz", type=float, default=100.0)
    ap.add_argument("--in-step", action="store_true",
                    help="record a step with the next batch's preparation running beside it")
    ap.add_argument("--spin", type=int, default=0,
                    help="ALU-spin iterations (tools/libinterfere.so) queued ahead of the recorded step, so the "
                         "whole step is enqueued before its first kernel starts (as tools/trace_probe.py)")
    args = ap.parse_args()
    import bench
    from bigcn_amd import BiGCN, FusedTrainStep, _lib
    from bigcn_amd.optim import bigcn_adam
    L = ctypes.CDLL(_lib.LIB_PATH)
    readers = [getattr(L, f"bgcn_bt_read_{tu}") for tu in ("sparse", "spmm", "bigcn")]
    for r in readers:
        r.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    wl = bench.WORKLOADS[args.workload]
    pool = bench.make_pool(wl, 0, 2, dev, (0.0, 0.0))
    model = BiGCN(wl["feats"], 64, 64, dev).to(dev)
    model.train()
    fused = FusedTrainStep(model, bigcn_adam(model), tddroprate=0.2, budroprate=0.2, drop_seed=1)
    stream = torch.cuda.Stream(dev)
    cap = 2 * 16 * (1 << 14)
    buf = np.zeros(cap * 4, dtype=np.uint64)
    with torch.cuda.stream(stream):
        for i in range(4):
            fused(pool[i % 2], next_data=pool[(i + 1) % 2])
        fused(pool[1], next_data=pool[0])
        pend = fused._pending
        for _ in range(5):
            fused._pending = pend
            fused(pool[0])
        torch.cuda.synchronize()
        for r in readers:
            r(None, 0, 1)           # reset + enable
        fused._pending = pend
        if args.spin:
            sink = torch.zeros(4, device=dev)
            Li = ctypes.CDLL(os.path.join(ROOT, "tools", "libinterfere.so"))
            Li.ifr_alu(1, args.spin, ctypes.c_void_p(sink.data_ptr()), ctypes.c_void_p(stream.cuda_stream))
        if args.in_step:
            fused(pool[0], next_data=pool[1])
            fused.discard_prefetch()
        else:
            fused(pool[0])
        torch.cuda.synchronize()
    recs, marks = [], []
    for r in readers:
        n = r(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), cap, 0)
        recs.append(buf[: 4 * max(n, 0)].reshape(-1, 4).copy())
        marks.append(buf[4 * max(n, 0): 8 * max(n, 0)].reshape(-1, 4).copy())
    rec = np.concatenate(recs)
    mk = np.concatenate(marks)
    keep = rec[:, 1] != 0
    rec, mk = rec[keep], mk[keep]
    kid = (rec[:, 0] >> 48).astype(int)
    t0 = rec[:, 1].astype(np.int64)
    t1 = rec[:, 2].astype(np.int64)
    cyc = (rec[:, 3] >> 32).astype(np.int64)
    xcc = ((rec[:, 3] >> 24) & 15).astype(int)
    wall = t1 - t0
    ok = wall > 0
    print(f"clock calibration: shader cycles per wall tick, median {np.median(cyc[ok] / wall[ok]):.2f} "
          f"(p10 {np.percentile(cyc[ok] / wall[ok], 10):.2f}, p90 {np.percentile(cyc[ok] / wall[ok], 90):.2f}); "
          f"XCCs seen {sorted(set(xcc))}")
    us = 1.0 / args.mhz
    cu = ((rec[:, 3] >> 8) & 0xffff).astype(np.int64) + 65536 * xcc

    def conc(m):   # largest number of this kernel's waves alive at once on one CU
        best = 0
        for c in set(cu[m]):
            mc = m & (cu == c)
            ev = sorted([(a, 1) for a in t0[mc]] + [(b, -1) for b in t1[mc]])
            cur = 0
            for _, dlt in ev:
                cur += dlt
                best = max(best, cur)
        return best
    # per-XCC clock offsets are unknown: spans are taken within each XCC, then the
    # longest reported
    print(f"{'kernel':20s} {'waves':>6s} {'span(max XCC)':>13s} {'last start':>10s}  "
          f"{'life p50':>8s} {'p90':>6s} {'max':>6s}  (us at {args.mhz:g} MHz)")
    for k in sorted(set(kid), key=lambda k: t0[kid == k].min()):
        m = kid == k
        life = (t1[m] - t0[m]) * us
        spans, lasts = [], []
        for x in sorted(set(xcc[m])):
            mx = m & (xcc == x)
            spans.append((t1[mx].max() - t0[mx].min()) * us)
            lasts.append((t0[mx].max() - t0[mx].min()) * us)
        print(f"{NAMES.get(k, str(k)):20s} {m.sum():6d} {max(spans):13.1f} {max(lasts):10.1f}  "
              f"{np.percentile(life, 50):8.1f} {np.percentile(life, 90):6.1f} {life.max():6.1f}")
        st = np.concatenate([(t0[m & (xcc == x)] - t0[m & (xcc == x)].min()) * us for x in sorted(set(xcc[m]))])
        print(f"{'':20s}   starts (per XCC) p10 {np.percentile(st, 10):5.1f} p50 {np.percentile(st, 50):5.1f} "
              f"p90 {np.percentile(st, 90):5.1f}; CUs {len(set(cu[m]))}, waves per CU max "
              f"{np.bincount(np.unique(cu[m], return_inverse=True)[1]).max()}; concurrent waves per CU max "
              f"{conc(m)}")
        for j in range(4):
            mj = mk[m, j].astype(np.int64)
            okj = mj != 0
            if okj.any():
                dt = (mj[okj] - t0[m][okj]) * us
                print(f"{'':20s}   mark {j}: +{np.percentile(dt, 50):6.1f} us p50, +{np.percentile(dt, 90):6.1f} p90 "
                      f"({okj.sum()} waves)")

if __name__ == "__main__":
    main()
