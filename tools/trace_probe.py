"""Diagnostic: device-side timeline of bgcn_train_step with the host enqueue out of the
picture.  Before every step a one-wave ALU spin (~1 ms, tools/libinterfere.so) holds the
step's stream, so the whole step is queued before its first kernel starts; under
rocprofv3 --kernel-trace the kernels then run exactly as the device schedules them.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python tools/trace_probe.py
    python tools/prof.py timeline OUT/.../run_kernel_trace.csv --after k_alu

--mode full: the normal step (next batch prepared on the side lane); --mode alone: the
prepared batch reused, nothing on the side lane (the chain alone)."""
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
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--mode", default="full", choices=["full", "alone", "both"])
    ap.add_argument("--workload", default="twitter15")
    ap.add_argument("--spin", type=int, default=60000)
    args = ap.parse_args()
    import bench
    from bigcn_amd import BiGCN, FusedTrainStep, Net
    from bigcn_amd.optim import bigcn_adam
    L = ctypes.CDLL(os.path.join(ROOT, "tools", "libinterfere.so"))
    dev = torch.device("cuda", 0)
    wl = bench.WORKLOADS[args.workload]
    dd = wl["drop"] != (0.0, 0.0)
    pool = bench.make_pool(wl, 0, 4, dev, (0.0, 0.0))
    model = (BiGCN if wl["classes"] == 4 else Net)(wl["feats"], 64, 64, dev).to(dev)
    model.train()
    fused = FusedTrainStep(model, bigcn_adam(model), tddroprate=wl["drop"][0], budroprate=wl["drop"][1],
                           drop_seed=1)
    stream = torch.cuda.Stream(dev)
    sink = torch.zeros(4, device=dev)
    modes = ["full", "alone"] if args.mode == "both" else [args.mode]
    with torch.cuda.stream(stream):
        for i in range(5):
            fused(pool[i % 4], next_data=pool[(i + 1) % 4])
        torch.cuda.synchronize()
        for mode in modes:
            if mode == "alone":
                fused(pool[3], next_data=pool[0])
                pend = fused._pending
            for i in range(args.steps):
                L.ifr_alu(1, args.spin, ctypes.c_void_p(sink.data_ptr()), ctypes.c_void_p(stream.cuda_stream))
                if mode == "full":
                    fused(pool[i % 4], next_data=pool[(i + 1) % 4])
                else:
                    fused._pending = pend
                    fused(pool[0])
                torch.cuda.synchronize()
            print(mode, "done", flush=True)


if __name__ == "__main__":
    main()
