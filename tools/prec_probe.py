"""Precision probe (CPU only): the fp32 oracle (the reference's own dtype) against the fp64
oracle on a bench workload's full-size batch - per-gradient (max-scaled, elementwise)
errors, and the relu' sign flips of H1 between the two (entries of H1 within fp32
rounding of zero take opposite relu' in the two precisions)."""
import argparse
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from oracle import bigcn_oracle as O  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="weibo_bf16")
ap.add_argument("--threads", type=int, default=16)
args = ap.parse_args()
torch.set_num_threads(args.threads)
wl = bench.WORKLOADS[args.workload]
b = bench.make_pool(wl, 0, 2, "cpu", drop=(0.0, 0.0))[1]
N, F, C = b.x.size(0), wl["feats"], wl["classes"]
g = torch.Generator().manual_seed(1)
m0 = torch.rand(N, 64 + F, generator=g) < 0.5
m1 = torch.rand(N, 64 + F, generator=g) < 0.5
p = O.make_params(F, 64, 64, C, seed=31)
res, st = {}, {}
for dt in (torch.float32, torch.float64):
    t = time.time()
    batch = {"x": b.x.to(dt), "edge_index": b.edge_index, "BU_edge_index": b.BU_edge_index,
             "batch": b.batch, "rootindex": b.rootindex, "y": b.y}
    stages = {}
    _, _, grads = O.reference_grads({k: v.to(dt) for k, v in p.items()}, batch, True, m0, m1, stages=stages)
    res[dt] = grads
    st[dt] = {k: stages[k] for k in ("TDrumorGCN.h1", "BUrumorGCN.h1")}
    print(f"{args.workload} N={N} {dt}: {time.time() - t:.1f} s", flush=True)
    del batch, stages
for d in ("TDrumorGCN", "BUrumorGCN"):
    h32, h64 = st[torch.float32][d + ".h1"].double(), st[torch.float64][d + ".h1"]
    flips = int(((h32 > 0) != (h64 > 0)).sum())
    print(f"{d}.h1: relu' flips fp32 vs fp64 = {flips}; min |h1| = {float(h64.abs().min()):.3e}, "
          f"max |h1| = {float(h64.abs().max()):.3e}")
for k in res[torch.float64]:
    a, r = res[torch.float32][k].double(), res[torch.float64][k]
    err = (a - r).abs()
    rms = r.pow(2).mean().sqrt()
    print(f"  {k:32s} {float(err.max() / r.abs().max()):.2e} {float((err / (r.abs() + rms)).max()):.2e}")
