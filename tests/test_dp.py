"""Data-parallel path on CPU (gloo, world size 2): sharding trees across ranks and one
all-reduce of the flat gradient bucket reproduces the full-batch gradient
(bigcn_amd/dp.py).  Gradients come from the oracle, so no GPU is needed;
the GPU path uses the same GradBucket over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import bigcn_oracle as O

F_SMALL = 48


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batch(seed):
    """Four trees, identical for every caller (seeded)."""
    from bigcn_amd.data import synth_batch
    return synth_batch(np.random.default_rng(seed), [5, 9, 3, 7], vocab=F_SMALL, num_classes=4)


def _shard(full, trees):
    """Sub-batch of the given tree ids (re-offset, as a rank's own collation would be)."""
    ptr = full.ptr.tolist()
    xs, td, bu, roots, ys, bt = [], [], [], [], [], []
    off = 0
    for k, t in enumerate(trees):
        lo, hi = ptr[t], ptr[t + 1]
        xs.append(full.x[lo:hi])
        for src, dst in ((full.edge_index, td), (full.BU_edge_index, bu)):
            m = (src[0] >= lo) & (src[0] < hi)
            dst.append(src[:, m] - lo + off)
        roots.append(int(full.rootindex[t]) - lo + off)
        ys.append(int(full.y[t]))
        bt += [k] * (hi - lo)
        off += hi - lo
    return {"x": torch.cat(xs).double(), "edge_index": torch.cat(td, 1), "BU_edge_index": torch.cat(bu, 1),
            "batch": torch.tensor(bt), "rootindex": torch.tensor(roots), "y": torch.tensor(ys)}


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from bigcn_amd.dp import GradBucket, init_from_env
    r, w, _ = init_from_env("gloo")
    assert (r, w) == (rank, world)
    full = _batch(11)
    p = {k: v.double() for k, v in O.make_params(F_SMALL, 64, 64, 4, seed=3).items()}
    mine = _shard(full, [2 * rank, 2 * rank + 1])
    _, _, grads = O.reference_grads(p, mine, False)
    params = [torch.nn.Parameter(v.clone()) for v in p.values()]
    for prm, k in zip(params, p):
        prm.grad = grads[k].clone()
    bucket = GradBucket(params)
    views = bucket.reduce_sum()
    res = {k: (v / world).clone() for k, v in zip(p, views)}
    # the two-part order of the fused step (everything but the conv1 weights + the status
    # slot first, then the conv1 weights) reduces to the same bits as one all-reduce
    split = GradBucket(params, status_slot=True, late=[params[0], params[4]])
    for v, prm in zip(split.views(), params):
        v.copy_(prm.grad)
    split.flag.fill_(float(rank))
    works = [split.allreduce_part_async("a"), split.allreduce_part_async("b")]
    for wk in works:
        wk.wait()
    for k, v, ref in zip(p, split.views(), views):
        assert torch.equal(v, ref), k
    assert float(split.flag) == float(sum(range(world)))
    # in-place mean for torch optimisers
    bucket.allreduce_mean()
    res_mean = {k: prm.grad.clone() for k, prm in zip(p, params)}
    out.put((rank, {k: v.numpy() for k, v in res.items()},     # plain arrays: no shared-
             {k: v.numpy() for k, v in res_mean.items()}))      # memory handles across exit
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gradient_mean_equals_full_batch():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    got = []
    import queue
    while len(got) < world:
        try:
            got.append(q.get(timeout=5))
        except queue.Empty:
            dead = [pr for pr in procs if pr.exitcode not in (None, 0)]
            assert not dead, "a rank failed"
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    full = _batch(11)
    p = {k: v.double() for k, v in O.make_params(F_SMALL, 64, 64, 4, seed=3).items()}
    _, _, ref = O.reference_grads(p, _shard(full, [0, 1, 2, 3]), False)
    for rank, res, res_mean in got:
        for k in ref:
            # the bucket is fp32 (the device path's dtype); fp64 oracle grads on each rank
            scale = float(ref[k].abs().max())
            for got_k in (res[k], res_mean[k]):
                err = float((torch.from_numpy(got_k).double() - ref[k]).abs().max())
                assert err <= 1e-6 * max(scale, 1e-12), (k, err, scale)


def test_single_process_bucket_is_identity():
    from bigcn_amd.dp import GradBucket, init_from_env
    for k in ("WORLD_SIZE", "RANK"):
        os.environ.pop(k, None)
    assert init_from_env("gloo") == (0, 1, 0)
    a = torch.nn.Parameter(torch.zeros(3, 2))
    b = torch.nn.Parameter(torch.zeros(5))
    a.grad = torch.arange(6.).view(3, 2)
    b.grad = None
    bk = GradBucket([a, b])
    v = bk.reduce_sum()
    assert torch.equal(v[0], a.grad) and torch.equal(v[1], torch.zeros(5))
    assert v[0].data_ptr() == bk.views()[0].data_ptr()              # persistent views
    bk.allreduce_mean()                                              # no-op at world 1
    assert torch.equal(a.grad, torch.arange(6.).view(3, 2))
