"""Diagnostic: the training chain (its prepared batch reused, nothing else on the side
lane) beside synthetic side-stream jobs of one kind each (tools/interfere.hip):
ALU-only (CU occupancy / clocks), L2-, Infinity-Cache- and HBM-resident streaming reads,
and page-hopping reads (address-translation pressure at little bandwidth).  Each job is
sized to last ~job_us alone.

    hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/interfere.hip -o tools/libinterfere.so
    python tools/interfere_probe.py [--steps 100]"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--job-us", type=float, default=300.0)
    ap.add_argument("--placement", action="store_true",
                    help="only the 590 MB HBM read from buffers of each allocation flag")
    ap.add_argument("--policies", action="store_true",
                    help="only the 590 MB HBM read under each buffer-load cache policy")
    args = ap.parse_args()
    import bench
    from bigcn_amd import BiGCN, FusedTrainStep, ops
    from bigcn_amd.optim import bigcn_adam
    L = ctypes.CDLL(os.path.join(ROOT, "tools", "libinterfere.so"))
    for f in (L.ifr_alu, L.ifr_read, L.ifr_pages, L.ifr_read_pol):
        f.restype = ctypes.c_int
    L.ifr_alloc.restype = ctypes.c_void_p
    dev = torch.device("cuda", 0)
    wl = bench.WORKLOADS["twitter15"]
    pool = bench.make_pool(wl, 0, 2, dev, (0.0, 0.0))
    model = BiGCN(wl["feats"], 64, 64, dev).to(dev)
    model.train()
    fused = FusedTrainStep(model, bigcn_adam(model), tddroprate=0.2, budroprate=0.2, drop_seed=1)
    stream = torch.cuda.Stream(dev)
    side = torch.cuda.Stream(dev)
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    big = torch.empty(590 << 20, dtype=torch.uint8, device=dev).fill_(1)
    mid = torch.empty(64 << 20, dtype=torch.uint8, device=dev).fill_(1)
    small = torch.empty(256 << 10, dtype=torch.uint8, device=dev).fill_(1)
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    sh = lambda: ctypes.c_void_p(side.cuda_stream)

    jobs = {
        "alu 1024 blocks": lambda r: L.ifr_alu(1024, 2000 * r, P(sink), sh()),
        "alu 64 blocks": lambda r: L.ifr_alu(64, 2000 * r, P(sink), sh()),
        "read 256KB (L2) 1024 blk": lambda r: L.ifr_read(P(small), ctypes.c_int64(small.numel()), 1024, r, P(sink), sh()),
        "read 64MB (MALL) 1024 blk": lambda r: L.ifr_read(P(mid), ctypes.c_int64(mid.numel()), 1024, r, P(sink), sh()),
        "read 590MB (HBM) 256 blk": lambda r: L.ifr_read(P(big), ctypes.c_int64(big.numel()), 256, r, P(sink), sh()),
        "read 590MB (HBM) 128 blk": lambda r: L.ifr_read(P(big), ctypes.c_int64(big.numel()), 128, r, P(sink), sh()),
        "read 590MB (HBM) 1024 blk": lambda r: L.ifr_read(P(big), ctypes.c_int64(big.numel()), 1024, r, P(sink), sh()),
        "read 590MB (HBM) 48 blk": lambda r: L.ifr_read(P(big), ctypes.c_int64(big.numel()), 48, r, P(sink), sh()),
        "pages 590MB 64 blk": lambda r: L.ifr_pages(P(big), ctypes.c_int64(big.numel()), 64, r, P(sink), sh()),
        "pages 590MB 1024 blk": lambda r: L.ifr_pages(P(big), ctypes.c_int64(big.numel()), 1024, r, P(sink), sh()),
    }

    if args.policies:
        jobs = {}
        for blk in (1024, 256):
            for aux in (0, 1, 2, 3, 16, 17, 18, 19):
                jobs[f"read 590MB pol {aux} {blk} blk"] = (
                    lambda r, aux=aux, blk=blk: L.ifr_read_pol(P(big), ctypes.c_int64(big.numel()), blk, r, aux,
                                                               P(sink), sh()))

    if args.placement:
        jobs = {}
        for flag, nm in ((0, "coarse"), (1, "fine"), (3, "uncached")):
            ptr = L.ifr_alloc(ctypes.c_int64(590 << 20), flag)
            if not ptr:
                print(f"alloc flag {flag} failed", flush=True)
                continue
            for blk in (1024, 256):
                jobs[f"read 590MB {nm} {blk} blk"] = (
                    lambda r, ptr=ptr, blk=blk: L.ifr_read(ctypes.c_void_p(ptr), ctypes.c_int64(590 << 20), blk, r,
                                                           P(sink), sh()))

    def time_job(job, reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(side)
        job(reps)
        e1.record(side)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3

    with torch.cuda.stream(stream):
        for i in range(4):
            fused(pool[i % 2], next_data=pool[(i + 1) % 2])
        fused(pool[1], next_data=pool[0])
        pend = fused._pending
        torch.cuda.synchronize()

        def chain(job=None, reps=0):
            torch.cuda.synchronize()
            ops.set_kernel_timing(True, {9: "main"})
            for i in range(args.steps):
                if job is not None:
                    side.wait_stream(stream)
                    job(reps)
                fused._pending = pend
                fused(pool[0])
                if job is not None:
                    stream.wait_stream(side)
            torch.cuda.synchronize()
            ops.set_kernel_timing(False)
            ms, n = ops.kernel_timing(9)
            return ms / max(n, 1) * 1e3

        print(f"{'chain alone':28s} {chain():8.1f} us", flush=True)
        for name, job in jobs.items():
            time_job(job, 1)
            t1 = max(time_job(job, 1), 1.0)
            reps = max(1, int(round(args.job_us / t1)))
            t = time_job(job, reps)
            print(f"{'beside ' + name:28s} {chain(job, reps):8.1f} us   (job alone {t:7.1f} us, reps {reps})",
                  flush=True)
        print(f"{'chain alone':28s} {chain():8.1f} us", flush=True)


if __name__ == "__main__":
    main()
