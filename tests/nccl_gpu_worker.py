"""Worker of tests/test_gpu_dp.py::test_rccl_deferred_dw1_one_rank (a fresh process: the
process group is initialised before any other GPU call).  A one-rank `nccl` (RCCL) group runs
FusedTrainStep.__call__ down its world > 1 branch (the test hook ``_force_dp_overlap``): the
step with defer_dw1, flat_a (everything but dW1 + the status slot) all-reduced asynchronously
on RCCL's stream while bgcn_train_step_dw1 computes dW1 on the caller's stream, then flat_b,
both waited for, then the fused Adam - the code an 8-GPU bench run executes.  Over three steps
with next-batch prefetch and device DropEdge, the reduced buckets and the parameters must be
bitwise those of the one-call world-1 step (a sum over one rank)."""
import copy
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"
    from bigcn_amd import BiGCN, FusedTrainStep
    from bigcn_amd.data import synth_batch, synth_tree_sizes
    rng = np.random.default_rng(3)
    batches = [synth_batch(rng, synth_tree_sizes(rng, 32, 60), 5000, 4, device=dev) for _ in range(3)]
    torch.manual_seed(0)
    base = BiGCN(5000, 64, 64).to(dev)
    base.train()
    out = {}
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for overlapped in (True, False):
            model = copy.deepcopy(base)
            st = FusedTrainStep(model, tddroprate=0.2, budroprate=0.2, drop_seed=5)
            st._force_dp_overlap = overlapped
            issued = []
            orig = st.bucket.allreduce_part_async

            def rec(*a, _orig=orig, _issued=issued, **kw):
                w = _orig(*a, **kw)
                _issued.append(w is not None)
                return w
            st.bucket.allreduce_part_async = rec
            buckets = []
            for k in range(3):
                st(batches[k], seed=11 + k, next_data=batches[k + 1] if k + 1 < 3 else None)
                buckets.append(st.bucket.flat.clone())
            # the overlapped branch issued both RCCL all-reduces every step; the plain one none
            assert issued == ([True] * 6 if overlapped else []), issued
            st.check_status()
            assert st.run_report() == {"status": 0, "invalid_steps": 0}
            out[overlapped] = (buckets, [p.detach().clone() for p in model.parameters()])
    torch.cuda.synchronize()
    (ba, pa), (bb, pb) = out[True], out[False]
    for k, (x, y) in enumerate(zip(ba, bb)):
        assert x.numel() == y.numel() and x.abs().sum() > 0
        assert torch.equal(x, y), (k, float((x - y).abs().max()))
    for x, y in zip(pa, pb):
        assert torch.equal(x, y), float((x - y).abs().max())
    # the bucket's own helper without the hook: world 1 issues no collective
    assert st.bucket.allreduce_part_async("a") is None
    dist.barrier()
    dist.destroy_process_group()
    print("rccl ok")


if __name__ == "__main__":
    main()
