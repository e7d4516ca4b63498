"""Data-parallel training with the HIP step on the GPU: two ranks (separate processes on
the box's one GPU, gloo all-reduce of the flat gradient bucket) stay bitwise identical
over training steps with per-rank dropout and device DropEdge, and their averaged
gradients equal one process training on the concatenated shards (1e-5 of each
gradient's max magnitude: fp32 sums in a different order).  bench.py runs the same
FusedTrainStep + GradBucket over RCCL at N > 1."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _concat(batches):
    from bigcn_amd.data import Batch
    xs, td, bu, roots, ys, bt, ptr = [], [], [], [], [], [], [0]
    off, goff = 0, 0
    for b in batches:
        n = b.x.size(0)
        xs.append(b.x)
        td.append(b.edge_index + off)
        bu.append(b.BU_edge_index + off)
        roots.append(b.rootindex + off)
        ys.append(b.y)
        bt.append(b.batch + goff)
        ptr += [p + off for p in b.ptr.tolist()[1:]]
        off += n
        goff += b.num_graphs
    out = Batch(x=torch.cat(xs), edge_index=torch.cat(td, 1), BU_edge_index=torch.cat(bu, 1),
                rootindex=torch.cat(roots), y=torch.cat(ys), batch=torch.cat(bt),
                ptr=torch.tensor(ptr), num_graphs=goff)
    out.set_x_nnz_max(max(b.x_nnz_hint() for b in batches))
    return out


def _run_ranks(out_dir, world, overlap):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                   LOCAL_RANK=str(r), WORLD_SIZE=str(world), BGCN_DIST_BACKEND="gloo",
                   BGCN_DP_OVERLAP=overlap)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dp_gpu_worker.py"),
                                       str(out_dir)], env=env))
    try:
        for p in procs:
            assert p.wait(timeout=100) == 0
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return [np.load(out_dir / f"rank{r}.npz") for r in range(world)]


def test_two_ranks_on_the_hip_step(tmp_path):
    """Two ranks with the overlapped two-part all-reduce (the default at world > 1: the
    bucket minus the conv1 weight gradients reduced while bgcn_train_step_dw1 computes
    them) and with one all-reduce after the step (BGCN_DP_OVERLAP=0): the ranks stay
    bitwise equal, and both schedules train to bitwise-identical parameters."""
    world = 2
    (tmp_path / "ov").mkdir()
    (tmp_path / "one").mkdir()
    r0, r1 = _run_ranks(tmp_path / "ov", world, "1")
    s0, _ = _run_ranks(tmp_path / "one", world, "0")
    params = [k for k in r0.files if k.startswith("param:")]
    assert len(params) == 10
    for k in params:
        assert np.array_equal(r0[k], r1[k]), f"ranks diverged on {k}"
        assert np.array_equal(r0[k], s0[k]), f"overlapped and single all-reduce differ on {k}"
    assert np.array_equal(r0["grads0"], r1["grads0"])
    assert np.array_equal(r0["grads0"], s0["grads0"])

    # one process on the concatenation of both shards (loss mean over 2B trees = the
    # mean of the two ranks' means): same gradients
    sys.path.insert(0, HERE)
    from dp_gpu_worker import make_model, shard_batches
    from bigcn_amd import FusedTrainStep
    dev = torch.device("cuda", 0)
    m = make_model(dev)
    m.eval()
    step = FusedTrainStep(m)
    full = _concat([shard_batches(r, 1, dev)[0] for r in range(world)])
    step.forward_backward(full)
    torch.cuda.synchronize()
    step.check_status()
    off = 0
    for v in step.bucket.views():
        n = v.numel()
        a, b = r0["grads0"][off:off + n], v.reshape(-1).cpu().numpy()
        scale = float(np.abs(b).max())
        assert float(np.abs(a - b).max()) <= 1e-5 * max(scale, 1e-12), (tuple(v.shape), scale)
        off += n                    # grads0: the views concatenated in parameter order


def test_rccl_deferred_dw1_one_rank():
    """The RCCL (`nccl` backend) path of the overlapped two-part all-reduce through
    FusedTrainStep.__call__ itself (its world > 1 branch forced on a one-rank group), in a
    fresh process (the box has one GPU; RCCL refuses two ranks on one device): three steps
    train to the bits of the world-1 step."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0",
               LOCAL_RANK="0", WORLD_SIZE="1")
    env.pop("BGCN_DIST_BACKEND", None)
    r = subprocess.run([sys.executable, os.path.join(HERE, "nccl_gpu_worker.py")], env=env,
                       capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "rccl ok" in r.stdout
