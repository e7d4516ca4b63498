#!/usr/bin/env python
"""BiGCN training-step benchmark on MI355X (BASELINE.json metric: propagation-trees/s
fwd+bwd, batch = 128 trees per GPU, 5000-dim features).

    python bench.py [--gpus N --steps K --warmup W --workload twitter15]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step = one pass of the reference training loop body (``BiGCN_Twitter.py:183-189``) over
one batch of synthetic trees already resident in HBM: gcn_norm/CSR for TD and BU (K1),
the fused encoder forward, fc + log_softmax + NLL, backward, the DP gradient all-reduce
(N > 1) and the Adam step with the reference's three parameter groups.  Batches are
cycled from a pool of ``--pool`` distinct batches (each larger than the 256 MiB
Infinity Cache).  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import platform
import sys
import time


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv, dry_run: bool = False) -> int:
    """`python bench.py --gpus N` without a launcher (no WORLD_SIZE in the environment):
    start N fresh child processes of this script, one per GPU, with the torchrun
    environment (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT), relay
    rank 0's JSON line, and return non-zero if any child failed.  The parent makes no GPU
    call and imports nothing of bigcn_amd before (or after) spawning: only the children
    touch the device."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                                      stdout=subprocess.PIPE, text=True))
    outs, codes = [], []
    for p in procs:
        out, _ = p.communicate()
        outs.append(out or "")
        codes.append(p.returncode)
    # rank 0 prints the bench line; a dry run prints one environment line per rank
    for r, out in enumerate(outs):
        if r == 0 or dry_run:
            sys.stdout.write(out)
    sys.stdout.flush()
    bad = [(r, c) for r, c in enumerate(codes) if c != 0]
    for r, c in bad:
        print(f"rank {r} exited with status {c}", file=sys.stderr, flush=True)
    return next((c for _, c in bad if c > 0), 1) if bad else 0


if __name__ == "__main__":
    # `--gpus N` without torchrun: this process only launches the N ranks - decided before
    # torch (or anything that could touch the GPU) is imported
    _pre = argparse.ArgumentParser(add_help=False)
    _pre.add_argument("--gpus", type=int, default=1)
    _pre.add_argument("--launch-dry-run", action="store_true")
    _a, _ = _pre.parse_known_args()
    if _a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(_a.gpus, sys.argv[1:], _a.launch_dry_run))

import numpy as np
import torch
import torch.distributed as dist
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "propagation-trees/sec fwd+bwd, batch=128, 5000-dim feats @ 1/2/4/8 MI355X"
PEAK_FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix peak (dense)
PEAK_BF16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16 matrix peak (dense)
# the dense classes whose fp32-grade products run on the bf16 MFMA: products per fp32 product
# (conv1 / conv2: six-product splits; dW2: the keep bits exact, dZ2 split three ways - its
# 64 H1 columns of 5064 stay on the f32 MFMA)
# (bf16 X: X is exact in bf16, so conv1, dW1 and conv2's root block take three; fp32 X's
# dW1 stays on the f32 MFMA)
BF16_PRODUCTS = {("dense", 0, False): 6, ("dense", 2, False): 6, ("dense", 3, False): 3,
                 ("dense", 0, True): 3, ("dense", 1, True): 3, ("dense", 2, True): 3, ("dense", 3, True): 3}
PEAK_HBM_GBS = 8000.0

WORKLOADS = {
    # BASELINE.json configs[1]: Twitter15 training, batch 128, fp32, 1 x MI355X.  The real
    # trees are absent (.MISSING_LARGE_BLOBS), so the batch is synthetic in the reference's
    # format with the tree-size distribution of SURVEY.md 8(d).
    "twitter15": dict(trees=128, mean=256, sigma=0.8, feats=5000, classes=4, drop=(0.2, 0.2),
                      desc="Twitter15-shaped synthetic: 128 trees/GPU, LogNormal(0.8) sizes mean 256 "
                           "clamped [2,8192], 5000-dim BoW x, DropEdge 0.2/0.2 re-drawn every step, "
                           "dropout 0.5, fp32"),
    # twitter15 with a tail of long posts: 1 % of the rows hold 40-300 distinct words (the
    # reference caps no row, Process/getTwittergraph.py:16-24).  Rows past the 32-entry ELL
    # spill their tail to the batch's spill pool; the step stays on the sparse path.
    "twitter15_tail": dict(trees=128, mean=256, sigma=0.8, feats=5000, classes=4, drop=(0.2, 0.2),
                           long_rows=(0.01, 40, 300),
                           desc="twitter15 with 1% of the rows holding 40-300 non-zeros (uniform): "
                                "128 trees/GPU, LogNormal(0.8) sizes mean 256, 5000-dim BoW x, "
                                "DropEdge 0.2/0.2 re-drawn every step, dropout 0.5, fp32"),
    # BASELINE.json configs[2]: Weibo, 5000-dim BoW, batch 128, bf16.  Weibo trees average
    # ~816 nodes; the reference's Weibo script drops no edges
    # (BiGCN_Weibo.py:199-200) and has the 2-class head (Net, :76-89).  x is stored bf16
    # (the counts are exact); accumulation is fp32.
    "weibo_fp32": dict(trees=128, mean=816, sigma=0.8, feats=5000, classes=2, drop=(0.0, 0.0),
                       desc="Weibo-shaped synthetic as weibo_bf16 with x stored fp32"),
    "weibo_bf16": dict(trees=128, mean=816, sigma=0.8, feats=5000, classes=2, drop=(0.0, 0.0),
                       xdtype="bf16",
                       desc="Weibo-shaped synthetic: 128 trees/GPU, LogNormal(0.8) sizes mean 816 "
                            "clamped [2,8192], 5000-dim BoW x stored bf16 (exact counts), no "
                            "DropEdge, dropout 0.5, fp32 accumulation"),
    # BASELINE.json configs[4]: synthetic trees of mean 1024 nodes, 5000-dim, bf16 (the
    # HBM-roofline stress shape); per GPU one step = 128 such trees (weak scaling), the
    # training-run defaults of the Twitter script (DropEdge 0.2/0.2, 4 classes).
    # configs[3] (100k trees of mean 256) has the per-GPU step shape of "twitter15".
    # PHEME (BiGCN_Twitter.py:138-140,177-182: BiGCN(768, 64, 64), x = the tweets' 768-dim
    # BERT CLS embeddings): dense features, so the dense MFMA path; thread sizes from the
    # reference's own data/PHEME/*.json (1,982 threads: mean 10.5 posts, max 109)
    "pheme768": dict(trees=128, mean=10.5, sigma=0.8, feats=768, classes=4, drop=(0.2, 0.2), dense_x=True,
                     feat_mode="dense",
                     desc="PHEME-shaped synthetic: 128 threads/GPU, LogNormal(0.8) sizes mean 10.5 (the "
                          "reference's data/PHEME/*.json), 768-dim dense N(0,1) features (BERT CLS), "
                          "DropEdge 0.2/0.2 re-drawn every step, dropout 0.5, fp32, dense MFMA path"),
    "synth1024_bf16": dict(trees=128, mean=1024, sigma=0.8, feats=5000, classes=4, drop=(0.2, 0.2),
                           xdtype="bf16",
                           desc="synthetic stress: 128 trees/GPU, LogNormal(0.8) sizes mean 1024 "
                                "clamped [2,8192], 5000-dim BoW x stored bf16, DropEdge 0.2/0.2 "
                                "re-drawn every step, dropout 0.5, fp32 accumulation"),
}

# kernel classes timed by libbgcn's HIP-event hook (bgcn_set_kernel_timing)
KERNEL_CLASSES = {
    "dense": {0: "conv1 X.W1^T MFMA (TD+BU fused)", 1: "dW1 = dZ1^T X MFMA (TD+BU fused)",
              2: "conv2 A2.W2^T MFMA (generated A2)",
              3: "dW2 = dZ2^T A2 MFMA (root columns: k-tiles of one tree, keep bits x dZ2 on the bf16 MFMA, "
                 "the root factor per tile in fp32)"},
    "auto": {0: "conv1: k_compact_conv1 (X read + compaction + gather) or gather from prepared ELL",
             2: "conv2 (sparse root gather)", 3: "k_bwd_mid: dW2 partials + root partials + dH1",
             5: "k_bwd_tail: dW1 over CSC(X) + dW2 root columns + reductions",
             7: "k_prep_b: paced X read + BoW compaction of the next batch beside the training chain "
                "(+ its tree items; its DropEdge select and K1 run on a second lane)"},
}
SPARSE_CAP = 32
# rocprofv3 kernel symbol of each timed class (for the PMC traffic lookup)
ROCPROF_NAMES = {("auto", 0): "bgcn::k_compact_conv1<true, float>", ("auto", 2): "bgcn::k_conv2_sparse",
                 ("auto", 3): "bgcn::k_bwd_mid<float>", ("auto", 5): "bgcn::k_bwd_tail<0, 0>",
                 ("auto", 7): "bgcn::k_prep_b<float>",
                 ("dense", 0): "bgcn::k_gemm_xwt_x6p", ("dense", 1): "bgcn::k_gemm_tn_w",
                 ("dense", 2): "bgcn::k_conv2_fwd_bf16<float, true>", ("dense", 3): "bgcn::k_dw2_root<float>"}


def pmc_file(workload: str, mode: str = "auto") -> str:
    """The committed PMC passes of a workload's bench command (tools/profile_round.sh): the
    newest round's file for the workload (and the dense feature path's own passes)."""
    name = workload + ("_dense" if mode == "dense" else "")
    for r in ("r06", "r05"):
        f = os.path.join(ROOT, "profiles", f"{r}_pmc_traffic_{name}.json")
        if os.path.exists(f):
            return f
    return os.path.join(ROOT, "profiles", f"r06_pmc_traffic_{name}.json")


def pmc_traffic(mode: str, cls: int, workload: str = "twitter15", xbf16: bool = False):
    """HBM bytes per launch of a kernel class from the committed PMC passes
    (tools/prof.py traffic: FETCH_SIZE x2 + WRITE_SIZE, the same workload's bench), or None."""
    name = ROCPROF_NAMES.get((mode, cls))
    if name is None:
        return None
    if xbf16:   # the bf16-X instantiation of the templated kernels
        name = name.replace("<float>", "<unsigned short>")
    try:
        with open(pmc_file(workload, mode)) as f:
            k = json.load(f)["kernels"].get(name)
    except (OSError, ValueError):
        return None
    return None if k is None else round(float(k["hbm_bytes"]), 0)


def kernel_work(mode: str, cls: int, N: float, Fd: int, prefetch: bool = False, xbytes: int = 4):
    """(bound, algorithmic units per launch): FLOPs for MFMA kernels, bytes for HBM ones.
    xbytes: bytes per stored feature (4 fp32, 2 bf16)."""
    H = 64
    if mode == "auto":
        if cls == 0:   # dense X read once + Z1 [N,128] + the compacted lists written
            if prefetch:   # conv1 from the prepared ELL: lists read, Z1 written
                return "hbm", N * 2 * H * 4.0 + N * (SPARSE_CAP * 8.0 + 4.0)
            return "hbm", N * Fd * xbytes + N * 2 * H * 4.0 + N * (SPARSE_CAP * 8.0 + 4.0)
        if cls == 7:   # dense X read once + the compacted lists written
            return "hbm", N * Fd * xbytes + N * (SPARSE_CAP * 8.0 + 4.0)
        if cls == 2:   # H1 [N,128] read + Z2 [N,128] written (gathers of W2^T rows hit L2)
            return "hbm", N * 2 * H * 4.0 * 2
        if cls == 3:   # dZ2 read by three roles, H1 by two, dH1 written (the [N, 128] streams)
            return "hbm", N * 2 * H * 4.0 * 6
        if cls == 5:   # ELL + CSC slots + dZ1 [N,128] read once, dW1 [128, F] written
            return "hbm", N * SPARSE_CAP * 12.0 + N * 2 * H * 4.0 + 4.0 * Fd * 2 * H
        return None, 0.0
    if cls in (0, 1):
        return "mfma", 2.0 * N * Fd * 2 * H
    if cls in (2, 3):
        return "mfma", 2.0 * N * (Fd + H) * H * 2
    return None, 0.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_pool(wl, rank, pool, device, drop=None):
    """drop: (td, bu) rates applied on the host at synthesis (the reference's DataLoader
    does it per sample); (0, 0) when the step drops edges on the device."""
    from bigcn_amd.data import synth_batch, synth_tree_sizes
    drop = wl["drop"] if drop is None else drop
    out = []
    for i in range(pool):
        rng = np.random.default_rng(20250205 + 1 + 1000 * rank + i)
        sizes = synth_tree_sizes(rng, wl["trees"], wl["mean"], wl["sigma"])
        xdt = torch.bfloat16 if wl.get("xdtype") == "bf16" else torch.float32
        b = synth_batch(rng, sizes, wl["feats"], wl["classes"], *drop, device=device, dtype=xdt,
                        long_rows=wl.get("long_rows"))
        if wl.get("dense_x"):   # dense embeddings (PHEME's BERT CLS rows): no sparse hints
            g = torch.Generator(device=device).manual_seed(20250205 + i)
            b.x = torch.randn(b.x.shape, generator=g, device=device, dtype=xdt)
        out.append(b)
    return out


def cpu_threads() -> int:
    """Host threads for the CPU baseline: the affinity set (BASELINE.md protocol), capped
    by OMP_NUM_THREADS - the GPU box's CPU share is 16 per GPU (OMP_NUM_THREADS=16 there)
    while os.sched_getaffinity reports the whole machine's cores."""
    n = len(os.sched_getaffinity(0))
    try:
        cap = int(os.environ.get("OMP_NUM_THREADS", "16"))
    except ValueError:
        cap = 16
    return max(1, min(n, cap if cap > 0 else n))


def cpu_baseline(wl, trees: int, steps: int, warmup: int = 3, repeats: int = 3):
    """The oracle (op-for-op plain-PyTorch restatement of the reference step) on the
    host cores: Python root loops, materialised [N, 5064] concat, aten dropout, autograd,
    Adam with 3 groups.  BASELINE.md protocol (3 warm-up, >= 10 timed steps, the median of
    `repeats` repeats) on a bounded sample: batches of `trees` trees of the workload's
    distribution (32 by default, ~1 s per step; the line states it)."""
    from bigcn_amd.data import synth_batch, synth_tree_sizes
    from oracle import bigcn_oracle as O
    cores = cpu_threads()
    torch.set_num_threads(cores)
    rng = np.random.default_rng(777)
    sizes = synth_tree_sizes(rng, trees, wl["mean"], wl["sigma"])
    b = synth_batch(rng, sizes, wl["feats"], wl["classes"], *wl["drop"], device="cpu",
                    long_rows=wl.get("long_rows"))
    batch = {"x": b.x.float(), "edge_index": b.edge_index, "BU_edge_index": b.BU_edge_index,
             "batch": b.batch, "rootindex": b.rootindex, "y": b.y}
    p = {k: v.requires_grad_(True) for k, v in O.make_params(wl["feats"], 64, 64, wl["classes"]).items()}
    opt = O.make_optimizer(p)
    for _ in range(warmup):
        O.train_step(p, opt, batch, training=True)
    rates = []
    for _ in range(repeats):
        t0 = time.perf_counter()
        for _ in range(steps):
            O.train_step(p, opt, batch, training=True)
        rates.append(trees * steps / (time.perf_counter() - t0))
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": round(float(np.median(rates)), 3), "unit": "trees/s", "cores": cores, "kind": "port",
            "repeats": [round(r, 3) for r in rates],
            "sample": f"median of {repeats} repeats x {steps} timed steps (+{warmup} warm-up) of one "
                      f"{trees}-tree batch ({int(sizes.sum())} nodes), the workload's tree/feature "
                      f"distribution, fp32; oracle/bigcn_oracle.py train_step, torch {torch.__version__} "
                      f"on {cpu}, {cores} threads; baseline only.  BASELINE.md's protocol (3 warm-up, "
                      f">= 10 timed steps, median of 3 repeats) on batches of {trees} trees instead of 128 "
                      f"(the per-tree cost is linear in the nodes: dropout over [N, 5064] dominates), so the "
                      f"default bench run stays within minutes"}


def step_roofline(N_avg: float, wl, sec_per_step: float):
    """Whole-step HBM fraction: the algorithmic bytes of one step that no design can avoid -
    X read ONCE (N * F * s; the step's every other access is O(N * 128) or L2-served) - over
    the measured step time, against 8 TB/s.  BASELINE.md's per-tree figure counts X twice
    (forward and dW1, 2 * N * F * s), which this build's single pass does not need; both
    fractions are given."""
    xbytes = 2 if wl.get("xdtype") == "bf16" else 4
    once = N_avg * wl["feats"] * xbytes
    gbs = once / sec_per_step / 1e9
    return {"bytes_per_step": round(once), "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(gbs / PEAK_HBM_GBS, 4), "frac_baseline_md_bytes": round(2 * gbs / PEAK_HBM_GBS, 4),
            "what": "X read once per step / ms_per_step; frac_baseline_md_bytes counts 2*N*F*s (BASELINE.md)"}


def aggregation_bench(b, iters: int = 10):
    """BASELINE north_star's standalone aggregation target: out = A_hat . X at the full
    5000-dim width (the algebraically equivalent order of GCNConv's propagate; the fused
    step aggregates 64-wide rows).  Algorithmic bytes:
    2*N*F*4 + 4*(N+1) + 8*(E+N)  (inputs read once, outputs written once, CSR)."""
    from bigcn_amd import ops
    N, Fd = b.x.shape
    x = b.x.float()          # the aggregation runs in fp32 (a bf16 workload's x is converted)
    res = {}
    for name, ei in (("td", b.edge_index), ("bu", b.BU_edge_index)):
        g = ops.build_graph(ei, N)
        out = torch.empty(N, Fd, dtype=torch.float32, device=b.x.device)
        for _ in range(2):
            ops.spmm(g, x, out=out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(iters):
            ops.spmm(g, x, out=out)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / iters
        E = int(ei.size(1))
        nbytes = 2.0 * N * Fd * 4 + 4.0 * (N + 1) + 8.0 * (E + N)
        gbs = nbytes / (ms * 1e-3) / 1e9
        res[name] = {"avg_ms": round(ms, 4), "bytes": nbytes, "achieved": round(gbs, 1),
                     "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4)}
    return {"kernel": "bgcn_spmm F=5000 (A_hat . X), one pool batch", "N": N, "F": Fd, **res}


def compaction_standalone(fused, b, wl, iters: int = 10):
    """The preparation's pass over X (k_prep_b, timing class 7) alone on the GPU, paced
    (the step's grid) and unpaced (a wave per row over all rows, BGCN_PREP_BLOCKS=0): the
    kernel's capability next to the in-step (paced, beside the chain) figure of `roofline`."""
    import ctypes
    from bigcn_amd import _lib, ops
    from bigcn_amd._lib import ptr, stream_handle
    L = _lib.lib()
    F = int(b.x.size(1))
    d, keep = fused._desc(b)
    buf = fused._prep_buffer(d, F)
    mode = _lib.BGCN_FEAT_SPARSE
    N = int(b.x.size(0))
    xbytes = 2 if wl.get("xdtype") == "bf16" else 4
    nbytes = N * F * xbytes + N * (SPARSE_CAP * 8.0 + 4.0)
    out = {"kernel": "k_prep_b (X read + BoW compaction + tree items), alone on the GPU",
           "bytes_per_launch": nbytes}
    old = os.environ.get("BGCN_PREP_BLOCKS")
    try:
        for name, env in (("paced", old), ("unpaced", "0")):
            if env is None:
                os.environ.pop("BGCN_PREP_BLOCKS", None)
            else:
                os.environ["BGCN_PREP_BLOCKS"] = env
            for _ in range(2):
                _lib.check(L.bgcn_prepare_batch(ctypes.byref(d), F, fused.degree_on, mode, ptr(buf),
                                                buf.numel(), stream_handle()))
            torch.cuda.synchronize()
            ops.set_kernel_timing(True, [7])
            for _ in range(iters):
                _lib.check(L.bgcn_prepare_batch(ctypes.byref(d), F, fused.degree_on, mode, ptr(buf),
                                                buf.numel(), stream_handle()))
            torch.cuda.synchronize()
            ops.set_kernel_timing(False)
            ms, n = ops.kernel_span(7)        # the kernel's own device-side span
            if n == 0:
                ms, n = ops.kernel_timing(7)
            avg = ms / max(n, 1)
            gbs = nbytes / (avg * 1e-3) / 1e9
            out[name] = {"avg_ms": round(avg, 4), "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS,
                         "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4)}
    finally:
        if old is None:
            os.environ.pop("BGCN_PREP_BLOCKS", None)
        else:
            os.environ["BGCN_PREP_BLOCKS"] = old
    return out


def host_fed_bench(fused, wl, dev, stream, steps: int, warmup: int, workers: int, trees: int,
                   native: bool = True):
    """SURVEY.md 8(f) row 1 / 8(d) "staging reported separately": the same training step fed
    from the host the way the reference's loop is (BiGCN_Twitter.py:168,174-176:
    DataLoader(..., shuffle=True, num_workers=5) -> Batch_data.to(device)) over a packed store
    of synthetic trees of the workload's shape, each 128-tree batch collated with x as the CSR
    of its non-zeros into a page-locked slot, one H2D copy per batch on a dedicated stream
    issued `depth` batches ahead, the step preparing the next batch from the compacted lists
    (no pass over a dense x).  native: libbgcn's loader (C++ collating threads,
    feed.NativeLoader); else a torch.utils.data.DataLoader with worker processes packing into
    a shared slot ring (feed.host_fed_loader).  Timed: everything (loader, copies, steps,
    Adam)."""
    from bigcn_amd import feed as FD
    t0 = time.perf_counter()
    store = FD.TreeStore.synthetic(trees, wl["mean"], seed=20250205 + 9, in_feats=wl["feats"],
                                   num_classes=wl["classes"])
    t_store = time.perf_counter() - t0
    per_epoch = trees // wl["trees"]
    epochs = (steps + warmup + 4) // per_epoch + 2
    bf16 = wl.get("xdtype") == "bf16"
    if native:
        loader = FD.NativeLoader(store, batch_size=wl["trees"], num_workers=workers, seed=7, epochs=epochs,
                                 bf16_values=bf16)
    else:
        loader = FD.host_fed_loader(store, batch_size=wl["trees"], num_workers=workers, seed=7, epochs=epochs,
                                    bf16_values=bf16)
    xdt = torch.bfloat16 if bf16 else torch.float32
    with torch.cuda.stream(stream):
        feeder = FD.DeviceFeeder(loader, dev, depth=3, x_dtype=xdt, timing=True)
        it = iter(feeder)
        cur = next(it)
        for _ in range(warmup):
            nxt = next(it)
            fused(cur, next_data=nxt)
            cur = nxt
        torch.cuda.synchronize()
        feeder.copy_stats(reset=True)
        fused.run_report(reset=True)
        if native:
            loader.stats(reset=True)
        nodes = 0
        t_next = t_call = 0.0
        t0 = time.perf_counter()
        for _ in range(steps):
            ta = time.perf_counter()
            nxt = next(it)
            tb = time.perf_counter()
            fused(cur, next_data=nxt)
            t_call += time.perf_counter() - tb
            t_next += tb - ta
            nodes += cur.num_nodes
            cur = nxt
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        lstats = loader.stats() if native else None
        fused.discard_prefetch()
        res = None
        if native:
            # the same compacted batches resident on the device (no loader, no copies): the
            # device-side rate of the compacted-input step
            pool = [next(it) for _ in range(4)]
            for k in range(6):
                fused(pool[k % 4], next_data=pool[(k + 1) % 4])
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for k in range(steps):
                fused(pool[k % 4], next_data=pool[(k + 1) % 4])
            torch.cuda.synchronize()
            dt_res = time.perf_counter() - t1
            fused.discard_prefetch()
            res = {"value": round(wl["trees"] * steps / dt_res, 2), "unit": "trees/s",
                   "ms_per_step": round(dt_res / steps * 1e3, 4),
                   "what": "4 compacted batches resident in HBM, cycled (no loader, no H2D): "
                           "the step without the pass over a dense x"}
            del pool
    n, mean_bytes, copy_ms = feeder.copy_stats()
    report = fused.run_report()
    del cur, nxt, it, feeder
    if native:
        loader.close()
    else:
        loader.dataset.ring.close()
    del loader
    dense_bytes = nodes / steps * wl["feats"] * (2 if xdt == torch.bfloat16 else 4)
    leg = {"value": round(wl["trees"] * steps / dt, 2), "unit": "trees/s",
           "ms_per_step": round(dt / steps * 1e3, 4), "steps": steps, "warmup": warmup,
           "status": report["status"], "invalid_steps": report["invalid_steps"],
           "host_ms_per_step_in_loader": round(t_next / steps * 1e3, 4),
           "host_ms_per_step_in_step_call": round(t_call / steps * 1e3, 4),
           "loader": ({"kind": "native (feed.NativeLoader: libbgcn bgcn_loader_*, C++ collating threads)",
                       "threads": workers} if native else
                      {"kind": "torch.utils.data.DataLoader, worker processes, shared slot ring "
                               "(feed.host_fed_loader)", "num_workers": workers}),
           "h2d_bytes_per_batch": round(mean_bytes), "h2d_ms_per_batch": round(copy_ms, 4),
           "h2d_gbs": round(mean_bytes / (copy_ms * 1e-3) / 1e9, 2) if copy_ms > 0 else None}
    if lstats is not None:
        leg["loader_stats"] = lstats
    out = {"leg": leg, "store_build_s": round(t_store, 2), "avg_nodes_per_batch": round(nodes / steps, 1),
           "dense_x_bytes_per_batch": round(dense_bytes),
           "dense_x_h2d_ms_at_measured_rate": (round(dense_bytes / (mean_bytes / copy_ms), 3)
                                               if mean_bytes > 0 and copy_ms > 0 else None)}
    if res is not None:
        out["compacted_resident"] = res
    return out


def staging_bench(fused, wl, dev, stream, steps: int, warmup: int, workers: int, trees: int):
    """The host-fed legs: libbgcn's native loader (the "host_fed" figure) and the torch
    DataLoader with worker processes beside it (the reference's loader form)."""
    nat = host_fed_bench(fused, wl, dev, stream, steps, warmup, workers, trees, native=True)
    dl = host_fed_bench(fused, wl, dev, stream, steps, warmup, workers, trees, native=False)
    out = {"host_fed": nat["leg"], "host_fed_dataloader": dl["leg"],
           "compacted_resident": nat["compacted_resident"],
           "h2d_bytes_per_batch": nat["leg"]["h2d_bytes_per_batch"],
           "h2d_ms_per_batch": nat["leg"]["h2d_ms_per_batch"], "h2d_gbs": nat["leg"]["h2d_gbs"],
           "dense_x_bytes_per_batch": nat["dense_x_bytes_per_batch"],
           "dense_x_h2d_ms_at_measured_rate": nat["dense_x_h2d_ms_at_measured_rate"],
           "store": {"trees": trees, "build_s": nat["store_build_s"],
                     "avg_nodes_per_batch": nat["avg_nodes_per_batch"], "batch_size": wl["trees"],
                     "copy_depth": 3},
           "what": "a packed tree store -> each batch collated (x as CSR of its non-zeros) into a page-locked "
                   "slot by loader threads / worker processes -> one H2D copy per batch on a copy stream, "
                   "3 batches ahead -> FusedTrainStep with next-batch prefetch and device DropEdge; whole "
                   "loop timed (BiGCN_Twitter.py:168,174-176)"}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--launch-dry-run", action="store_true",
                    help="test hook: each rank prints its launcher environment and exits before any device work")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="twitter15", choices=sorted(WORKLOADS))
    ap.add_argument("--pool", type=int, default=4)
    ap.add_argument("--cpu-trees", type=int, default=32,
                    help="CPU baseline: trees per step (a bounded sample of the workload, ~1 s per step)")
    ap.add_argument("--cpu-steps", type=int, default=10, help="CPU baseline: timed steps per repeat")
    ap.add_argument("--cpu-warmup", type=int, default=3)
    ap.add_argument("--cpu-repeats", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--feat-mode", default="auto", choices=["auto", "dense"],
                    help="auto: sparse feature path with device-side dense fallback; dense: MFMA only")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: 128 trees per GPU (the metric); strong: the global batch of 128 trees "
                         "split over the ranks (SURVEY 8(e)'s secondary report)")
    ap.add_argument("--path", default="fused", choices=["fused", "autograd"],
                    help="fused: FusedTrainStep (one native call per step); autograd: per-op "
                         "drop-in modules + loss.backward()")
    ap.add_argument("--prefetch", type=int, default=1,
                    help="fused path: prepare the next batch (K1, ELL/CSC of X) during each step")
    ap.add_argument("--aggregation", type=int, default=1,
                    help="at N=1 also time the standalone 5000-wide aggregation A_hat . X")
    ap.add_argument("--compare-dense", type=int, default=1,
                    help="at N=1 also time the dense MFMA path and report it beside the main line")
    ap.add_argument("--dropedge", default="device", choices=["device", "host"],
                    help="fused path: DropEdge (dataset.py:68-90) drawn afresh for every step "
                         "inside the step's batch preparation on the device (default, timed), "
                         "or pre-applied ONCE per pool batch at synthesis on the host (the "
                         "draw is then neither repeated nor timed)")
    ap.add_argument("--compare-dropedge", type=int, default=1,
                    help="at N=1 also time the other DropEdge placement and report it beside the main line")
    ap.add_argument("--host-fed", type=int, default=1,
                    help="at N=1 also run the step host-fed through a DataLoader with worker processes "
                         "(the staging object)")
    ap.add_argument("--host-fed-workers", type=int, default=5,
                    help="DataLoader worker processes of the host-fed run (the reference's num_workers=5)")
    ap.add_argument("--host-fed-trees", type=int, default=2048, help="trees in the host-fed run's store")
    ap.add_argument("--eval-path", type=int, default=1,
                    help="at N=1 also time the fused evaluation step (the reference's test loop body)")
    ap.add_argument("--dropin-ahead", type=int, default=1,
                    help="1: also time the drop-in loop over feed.prepare_ahead (batches prepared one "
                         "step ahead on a side stream)")
    ap.add_argument("--dropin", type=int, default=1,
                    help="at N=1 also time the drop-in path (model(data), loss.backward(), the "
                         "optimiser: --path autograd) and report it beside the main line")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no torchrun around us (bench imported and main() called): launch the N ranks
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], args.launch_dry_run))
    if args.launch_dry_run:
        print(json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                          "MASTER_PORT", "BGCN_DIST_BACKEND")}), flush=True)
        return

    from bigcn_amd import BiGCN, FusedTrainStep, Net
    from bigcn_amd import ops
    from bigcn_amd.dp import GradBucket, init_from_env
    from bigcn_amd.optim import bigcn_adam

    rank, world, local = init_from_env("nccl")
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    wl = WORKLOADS[args.workload]
    if wl.get("feat_mode") and args.feat_mode == "auto":
        args.feat_mode = wl["feat_mode"]         # dense-feature workloads run the dense path
    if args.scaling == "strong":   # the workload's global batch split over the ranks
        wl = dict(wl, trees=max(1, wl["trees"] // world))
    torch.manual_seed(1234 + rank)
    device_drop = args.path == "fused" and args.dropedge == "device"
    pool = make_pool(wl, rank, args.pool, dev, (0.0, 0.0) if device_drop else None)
    nodes = [b.x.size(0) for b in pool]
    model = (BiGCN if wl["classes"] == 4 else Net)(wl["feats"], 64, 64, dev).to(dev)
    if world > 1:   # identical initial parameters on every rank
        for p in model.parameters():
            dist.broadcast(p.data, 0)
    model.train()
    # the step runs on its own stream: the fused encoder forks independent branches onto
    # libbgcn's auxiliary stream, which needs a non-default stream to wait on the device
    stream = torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    opt = bigcn_adam(model)                             # reference groups, one fused launch
    bucket = GradBucket(opt.params())                   # same parameter order as opt

    drops = wl["drop"] if device_drop else (0.0, 0.0)
    fused = FusedTrainStep(model, opt, tddroprate=drops[0], budroprate=drops[1],
                           drop_seed=4242 + rank)       # bgcn_train_step + all-reduce + Adam

    ctx = {"pool": pool, "fused": fused, "path": args.path}   # swapped for the comparison runs

    def step(i):
        pool, fused = ctx["pool"], ctx["fused"]
        b = next(ctx["ahead"]) if ctx.get("ahead") is not None else pool[i % len(pool)]
        if ctx["path"] == "fused":                      # K1 + fwd + head + loss + bwd in one call;
            nxt = pool[(i + 1) % len(pool)] if args.prefetch else None   # the next batch's
            return fused(b, next_data=nxt)              # preparation overlaps this step
        b.__dict__.pop("_bgcn_graphs", None)          # gcn_norm/CSR rebuilt every step (as GCNConv does)
        logp = model(b)
        loss = F.nll_loss(logp, b.y)
        opt.zero_grad()
        loss.backward()
        if world > 1:                                   # RCCL sum of the flat bucket, mean folded in
            opt.step(grads=bucket.reduce_sum(), grad_scale=1.0 / world)
        else:
            opt.step()
        return loss

    def run(mode: str, steps: int, warmup: int, timing: bool = True):
        with torch.cuda.stream(stream):
            return run_on_stream(mode, steps, warmup, timing)

    def run_on_stream(mode: str, steps: int, warmup: int, timing: bool = True):
        model.feat_mode = mode
        # the kernel-timing hook records HIP events around the timed class: on the per-op
        # path those land on the caller's stream, each a queue-draining barrier (~6 us), so
        # the drop-in leg runs without it (it reports no roofline)
        timing = timing and not args.no_kernel_timing
        # warm-up: every kernel class timed (after the first step, which pays one-time
        # code-object loading), to find the dominant one; the timed loop then records
        # events only around that class (2 events per step)
        for i in range(warmup):
            if timing and i == min(1, warmup - 1):
                torch.cuda.synchronize()
                ops.set_kernel_timing(True)
            step(i)
        torch.cuda.synchronize()
        warm = {}
        if timing:
            ops.set_kernel_timing(False)
            for c in KERNEL_CLASSES[mode]:
                ms, n = ops.kernel_timing(c)
                if n:
                    warm[c] = ms / n
        if world > 1:
            dist.barrier()
        dominant = [max(warm, key=warm.get)] if warm else []
        # the sparse step's roofline kernel is the pass over X (class 7) whenever it runs:
        # a warm-up ranking can flip on a noisy box (two ranks sharing one GPU in a rehearsal)
        if mode == "auto" and 7 in warm:
            dominant = [7]
        if timing and dominant:
            ops.set_kernel_timing(True, dominant)
        torch.cuda.synchronize()
        if ctx["path"] == "fused":
            ctx["fused"].run_report(reset=True)         # validity of the timed steps only
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for i in range(steps):
            loss = step(warmup + i)
            if rank == 0 and (i + 1) % max(1, steps // 4) == 0:
                log(f"[{mode}] step {i + 1}/{steps}")
        t_host = time.perf_counter() - t0               # host enqueue time of the K steps
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        kern, span = {}, None
        if timing and dominant:
            ops.set_kernel_timing(False)
            kern[dominant[0]] = ops.kernel_timing(dominant[0])
            if dominant[0] == 7:   # the pass over X stamps its own device-side span
                span = ops.kernel_span(7)
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        N_avg = float(np.mean([nodes[(warmup + i) % len(nodes)] for i in range(steps)]))
        N_warm = float(np.mean([nodes[i % len(nodes)] for i in range(max(warmup, 1))]))
        roof, kernels, best = None, {}, None
        per_class = {c: (ms, n, "timed loop") for c, (ms, n) in kern.items()}
        for c, avg in warm.items():
            if c not in per_class:
                per_class[c] = (avg, 1, "warm-up")
        for c, (ms, n, where) in per_class.items():
            if n == 0:
                continue
            avg_ms = ms / n
            n_nodes = N_avg if where == "timed loop" else N_warm
            bound, work = kernel_work(mode, c, n_nodes, wl["feats"], args.prefetch and ctx["path"] == "fused",
                                      2 if wl.get("xdtype") == "bf16" else 4)
            ent = {"avg_ms": round(avg_ms, 4), "launches": n, "measured": where}
            if bound == "mfma":
                ent["tflops"] = round(work / (avg_ms * 1e-3) / 1e12, 2)
            elif bound == "hbm":
                ent["gbs"] = round(work / (avg_ms * 1e-3) / 1e9, 1)
            kernels[KERNEL_CLASSES[mode][c]] = ent
            if bound is not None and where == "timed loop":
                best = (c, avg_ms, bound, work, n_nodes)
        if best is not None:
            c, avg_ms, bound, work, n_nodes = best
            if bound == "mfma":
                ach = work / (avg_ms * 1e-3) / 1e12
                roof = {"bound": "mfma", "achieved": round(ach, 2), "peak": PEAK_FP32_MFMA_TFLOPS,
                        "unit": "TFLOP/s", "frac": round(ach / PEAK_FP32_MFMA_TFLOPS, 4),
                        "traffic": pmc_traffic(mode, c, args.workload, wl.get("xdtype") == "bf16"), "kernel": KERNEL_CLASSES[mode][c], "flops_per_launch": work,
                        "avg_ms": round(avg_ms, 4)}
                xb = wl.get("xdtype") == "bf16"
                k3 = BF16_PRODUCTS.get((mode, c, xb))
                # the library's own size rules (bgcn_internal.h kX6MinRows = 8192 rows for the
                # fp32 six-product kernels; dW2's tree-run tiles need >= 32 nodes per tree)
                if k3 and not xb and c in (0, 2) and n_nodes < 8192:
                    k3 = None
                if k3 and c == 3 and n_nodes < 32 * wl["trees"]:
                    k3 = None if not xb else k3
                if k3:   # the hardware the class runs on: fp32-grade products as k bf16 products
                    roof["bf16_products"] = k3
                    roof["peak_bf16_emulated"] = round(PEAK_BF16_MFMA_TFLOPS / k3, 1)
                    roof["frac_of_bf16_emulated_peak"] = round(ach * k3 / PEAK_BF16_MFMA_TFLOPS, 4)
            else:
                event_ms = avg_ms
                timer = "HIP events on the launch stream"
                if c == 7 and span is not None and span[1] > 0:
                    # device-side span: first block start -> last block end on the constant
                    # wall clock, the duration rocprofv3 reports for the dispatch
                    avg_ms = span[0] / span[1]
                    timer = "device wall-clock span (first block start to last block end, in-kernel stamps)"
                ach = work / (avg_ms * 1e-3) / 1e9
                roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                        "frac": round(ach / PEAK_HBM_GBS, 4), "traffic": pmc_traffic(mode, c, args.workload, wl.get("xdtype") == "bf16"),
                        "kernel": KERNEL_CLASSES[mode][c], "bytes_per_launch": work,
                        "avg_ms": round(avg_ms, 4), "timer": timer, "event_avg_ms": round(event_ms, 4),
                        "frac_by_event_bracket": round(work / (event_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)}
                if mode == "auto" and c == 7 and args.prefetch:
                    roof["note"] = ("frac uses the kernel's own span (comparable with the rocprofv3 kernel "
                                    "average under profiles/); the HIP-event bracket on the side lane also "
                                    "holds the pass's dispatch delay behind the second preparation lane "
                                    "(frac_by_event_bracket)")
        value = wl["trees"] * world * steps / dt
        # the step's validity (one host read after the timed region): the OR of the timed
        # steps' status words and the optimiser updates skipped as invalid, max over ranks
        report = ctx["fused"].run_report() if ctx["path"] == "fused" else {"status": 0, "invalid_steps": 0}
        v = torch.tensor([report["status"], report["invalid_steps"]], dtype=torch.int64, device=dev)
        if world > 1:
            dist.all_reduce(v, op=dist.ReduceOp.MAX)
        return {"value": value, "dt": dt, "t_host": t_host, "N_avg": N_avg, "roof": roof, "kernels": kernels,
                "loss": float(loss.item()), "status": int(v[0]), "invalid_steps": int(v[1])}

    main_res = run(args.feat_mode, args.steps, args.warmup)

    def fresh_allocator():
        # each comparison leg starts from the caching allocator state a fresh process would
        # have: the blocks earlier legs cached (and their pending stream uses) made the
        # per-op leg's ~40 allocations per step slower (host enqueue 0.47 vs 0.28 ms per step)
        torch.cuda.synchronize()
        gc.collect()
        torch.cuda.empty_cache()
    dense_res = None
    if world == 1 and args.feat_mode != "dense" and args.compare_dense:
        fresh_allocator()
        dense_res = run("dense", max(3, args.steps // 2), 2)
    drop_res = None
    if world == 1 and args.path == "fused" and args.compare_dropedge:
        fresh_allocator()
        other = not device_drop                         # the other DropEdge placement
        ctx["pool"] = make_pool(wl, rank, args.pool, dev, (0.0, 0.0) if other else None)
        d2 = wl["drop"] if other else (0.0, 0.0)
        ctx["fused"] = FusedTrainStep(model, opt, tddroprate=d2[0], budroprate=d2[1], drop_seed=4242)
        drop_res = run(args.feat_mode, max(3, args.steps // 2), 2)
        drop_res["where"] = "device" if other else "host_once_untimed"
        ctx["pool"], ctx["fused"] = pool, fused
    dropin_res = None
    if world == 1 and args.path == "fused" and args.dropin:
        # the north_star drop-in form: the reference's loop body verbatim on the per-op
        # modules (gcn_norm/CSR rebuilt every step as GCNConv does), DropEdge applied by the
        # host DataLoader as in the reference (once per pool batch here, untimed)
        fresh_allocator()
        ctx["pool"] = make_pool(wl, rank, args.pool, dev, None)
        ctx["path"] = "autograd"
        # (a sixty-step window after ten warm-up steps: the per-op loop's host enqueue jitters
        # by tens of us per step, so a ten-step window after three read 8-25 % low,
        # DESIGN.md 7)
        dropin_steps = max(60, args.steps)
        dropin_warm = int(os.environ.get("BGCN_BENCH_DROPIN_WARMUP", "10"))
        dropin_res = run(args.feat_mode, dropin_steps, dropin_warm, timing=False)
        # the same loop body over the batches as feed.prepare_ahead hands them out (each
        # batch's K1 and pass over X queued on a side stream one step ahead, beside the
        # previous step - the data pipeline's stage, the loop body untouched)
        dropin_ahead_res = None
        if args.dropin_ahead:
            from bigcn_amd.feed import prepare_ahead
            fresh_allocator()
            dp = ctx["pool"]
            ctx["ahead"] = iter(prepare_ahead((dp[i % len(dp)] for i in range(dropin_steps + dropin_warm + 1)),
                                              model))
            dropin_ahead_res = run(args.feat_mode, dropin_steps, dropin_warm, timing=False)
            ctx["ahead"] = None
        ctx["pool"], ctx["path"] = pool, args.path
    eval_res = None
    if world == 1 and args.path == "fused" and args.eval_path:
        # the reference's per-epoch test loop (BiGCN_Twitter.py:207-222) in the fused form:
        # eval-mode forward + head + NLL mean + argmax / correct count per batch, the next
        # batch prepared on the side lane, no host sync inside the timed loop
        n_eval = max(5, args.steps // 2)
        model.eval()
        with torch.cuda.stream(stream):
            for i in range(3):
                fused.evaluate(pool[i % len(pool)], next_data=pool[(i + 1) % len(pool)])
            fused.discard_prefetch()
            torch.cuda.synchronize()
            fused.run_report(reset=True)
            t0 = time.perf_counter()
            for i in range(n_eval):
                ev_loss, ev_correct = fused.evaluate(pool[i % len(pool)],
                                                     next_data=pool[(i + 1) % len(pool)] if i + 1 < n_eval else None)
            torch.cuda.synchronize()
            dt_eval = time.perf_counter() - t0
        rep = fused.run_report(reset=True)
        model.train()
        eval_res = {"value": round(wl["trees"] * n_eval / dt_eval, 2), "unit": "trees/s",
                    "ms_per_step": round(dt_eval / n_eval * 1e3, 4), "steps": n_eval, "status": rep["status"],
                    "last_loss": round(float(ev_loss), 5), "last_correct": int(ev_correct),
                    "what": "FusedTrainStep.evaluate: the test loop body (BiGCN_Twitter.py:207-222: model.eval(), "
                            "model(data), nll_loss, argmax, correct count) per pool batch, the next batch "
                            "prepared beside it; no DropEdge, no dropout"}
    agg = None
    if world == 1 and args.aggregation:
        agg = aggregation_bench(pool[0])
    comp = None
    if world == 1 and args.path == "fused" and args.feat_mode == "auto":
        with torch.cuda.stream(stream):
            comp = compaction_standalone(fused, pool[0], wl)
    staging = None
    if world == 1 and args.path == "fused" and args.host_fed and args.feat_mode == "auto":
        # same model / optimiser / DropEdge as the headline step (its state continues)
        staging = staging_bench(fused, wl, dev, stream, max(20, args.steps), min(args.warmup, 10),
                                args.host_fed_workers, args.host_fed_trees)
    if rank == 0:
        value, dt, N_avg = main_res["value"], main_res["dt"], main_res["N_avg"]
        roof, kernels, final_loss = main_res["roof"], main_res["kernels"], main_res["loss"]
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            log("cpu baseline ...")
            cpu = cpu_baseline(wl, args.cpu_trees, args.cpu_steps, args.cpu_warmup, args.cpu_repeats)
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "trees/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
            "host_enqueue_ms_per_step": round(main_res["t_host"] / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None,
            "dtype": "bf16 x, f32 accumulate" if wl.get("xdtype") == "bf16" else "f32",
            "data": "synthetic (reference npz/Batch layout; real Twitter15 trees absent)",
            "config": {"workload": wl["desc"], "trees_per_gpu": wl["trees"], "feat_path": args.feat_mode,
                       "global_batch": wl["trees"] * world, "avg_nodes_per_batch": round(N_avg, 1),
                       "in_feats": wl["feats"], "parallelism": f"dp{world}"},
            "roofline": roof, "cpu_baseline": cpu,
            "invalid_steps": main_res["invalid_steps"], "status": main_res["status"],
            "step_roofline": step_roofline(N_avg, wl, dt / args.steps),
            "kernels": kernels, "final_loss": round(final_loss, 5),
            "feat_mode": args.feat_mode, "step_path": args.path, "prefetch_next_batch": bool(args.prefetch),
            "dropedge": ("device, re-drawn every step (timed)" if device_drop
                         else "host, applied once per pool batch at synthesis (not timed)"),
        }
        if staging is not None:
            staging["host_fed_over_headline"] = round(staging["host_fed"]["value"] / value, 4)
            out["staging"] = staging
        if agg is not None:
            out["aggregation_5000"] = agg
        if comp is not None:
            out["compaction_standalone"] = comp
        if drop_res is not None:
            out["dropedge_" + drop_res["where"]] = {
                "value": round(drop_res["value"], 2), "unit": "trees/s",
                "ms_per_step": round(drop_res["dt"] / max(3, args.steps // 2) * 1e3, 4)}
        if eval_res is not None:
            out["eval_path"] = eval_res
        if dropin_res is not None:
            n = dropin_steps
            out["dropin_path"] = {
                "value": round(dropin_res["value"], 2), "unit": "trees/s",
                "ms_per_step": round(dropin_res["dt"] / n * 1e3, 4), "steps": n,
                "host_enqueue_ms_per_step": round(dropin_res["t_host"] / n * 1e3, 4),
                "what": "--path autograd: model(data) -> F.nll_loss -> loss.backward() -> optimiser "
                        "step per batch (BiGCN_Twitter.py:183-189 verbatim on the drop-in GCNConv / "
                        "scatter_mean modules), host DropEdge once per pool batch (untimed)",
                "prepared_ahead": None if dropin_ahead_res is None else {
                    "value": round(dropin_ahead_res["value"], 2), "unit": "trees/s",
                    "ms_per_step": round(dropin_ahead_res["dt"] / n * 1e3, 4),
                    "host_enqueue_ms_per_step": round(dropin_ahead_res["t_host"] / n * 1e3, 4),
                    "what": "the same loop over feed.prepare_ahead(batches, model): each batch's K1 and "
                            "pass over X queued on a side stream one step ahead"}}
        if dense_res is not None:
            out["dense_path"] = {"value": round(dense_res["value"], 2), "unit": "trees/s",
                                 "ms_per_step": round(dense_res["dt"] / max(3, args.steps // 2) * 1e3, 4),
                                 "roofline": dense_res["roof"], "kernels": dense_res["kernels"]}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if main_res["invalid_steps"] or main_res["status"]:
        log(f"INVALID: {main_res['invalid_steps']} timed step(s) skipped by the optimiser, "
            f"status bits {main_res['status']:#x}")
        sys.exit(3)


if __name__ == "__main__":
    main()
