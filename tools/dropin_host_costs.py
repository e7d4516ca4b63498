"""Per-call host costs of the drop-in (autograd) training step on the GPU box.

Runs the reference loop body (model(data) -> nll_loss -> backward -> opt.step) on
synthetic twitter15 batches and times each host-side piece (the native calls wrapped).
"""
import sys, time, collections, torch
import torch.nn.functional as F
import os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
from bigcn_amd import BiGCN, _lib, ops
from bigcn_amd.optim import bigcn_adam
dev = torch.device("cuda", 0)
wl = bench.WORKLOADS["twitter15"]
pool = bench.make_pool(wl, 0, 4, dev, None)
model = BiGCN(wl["feats"], 64, 64, dev).to(dev); model.train()
opt = bigcn_adam(model)
s = torch.cuda.Stream(dev)
acc = collections.defaultdict(float)
L = _lib.lib()
for name in ["bgcn_bigcn_forward", "bgcn_bigcn_backward", "bgcn_build_graph_pair", "bgcn_adam_step", "bgcn_head_forward", "bgcn_head_backward",
             "bgcn_bigcn_workspace_size", "bgcn_graph_pair_workspace_size"]:
    f = getattr(L, name)
    def w(*a, _f=f, _n=name):
        t = time.perf_counter(); r = _f(*a); acc["native " + _n] += time.perf_counter() - t; return r
    setattr(L, name, w)
def timed(key, fn):
    def w(*a, **k):
        t = time.perf_counter(); r = fn(*a, **k); acc[key] += time.perf_counter() - t; return r
    return w
ops._BiGCNNetFn.backward = staticmethod(timed("py net backward (incl native)", ops._BiGCNNetFn.backward))
ops._BiGCNNetFn.forward = staticmethod(timed("py net forward (incl native)", ops._BiGCNNetFn.forward))
import bigcn_amd.bigcn as bb
bb.build_graph_pair = timed("build_graph_pair (incl native)", bb.build_graph_pair)
bb._draw_seed = timed("draw_seed", bb._draw_seed)
def step(i, rec):
    b = pool[i % len(pool)]; b.__dict__.pop("_bgcn_graphs", None)
    t = time.perf_counter(); logp = model(b); t1 = time.perf_counter()
    t2 = t3 = t1
    loss = F.nll_loss(logp, b.y); t4 = time.perf_counter()
    opt.zero_grad(); loss.backward(); t5 = time.perf_counter(); opt.step(); t6 = time.perf_counter()
    if rec:
        for k, d in (("encode", t1 - t), ("fc", t2 - t1), ("log_softmax", t3 - t2), ("nll", t4 - t3),
                     ("zero_grad+backward", t5 - t4), ("opt.step", t6 - t5), ("total", t6 - t)):
            acc[k] += d
with torch.cuda.stream(s):
    for i in range(20): step(i, False)
    torch.cuda.synchronize(); acc.clear()
    t0 = time.perf_counter()
    for i in range(300): step(i, True)
    th = time.perf_counter() - t0; torch.cuda.synchronize(); dt = time.perf_counter() - t0
print(f"host {th/300*1e6:.1f} us/step, wall {dt/300*1e6:.1f} us/step")
with torch.cuda.stream(s):
    for burst in (10, 20):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        for i in range(burst): step(i, False)
        th = time.perf_counter() - t0; torch.cuda.synchronize(); dt = time.perf_counter() - t0
        print(f"burst {burst}: host {th/burst*1e6:.1f} us/step, wall {dt/burst*1e6:.1f} us/step")
for k, v in sorted(acc.items(), key=lambda x: -x[1]):
    print(f"{k:45s} {v/300*1e6:8.1f} us")
