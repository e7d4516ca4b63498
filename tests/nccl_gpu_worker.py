"""Worker of tests/test_gpu_dp.py::test_rccl_deferred_dw1_one_rank (a fresh process: the
process group is initialised before any other GPU call).  A one-rank `nccl` (RCCL) group runs
the fused step's two-part overlapped all-reduce exactly as FusedTrainStep.__call__ does at
world > 1 - flat_a (everything but dW1 + the status slot) all-reduced asynchronously on
RCCL's stream while bgcn_train_step_dw1 computes dW1 on the caller's stream, then flat_b -
and checks the reduced bucket is bitwise the one-call step's (a sum over one rank)."""
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
    b = synth_batch(rng, synth_tree_sizes(rng, 32, 60), 5000, 4, device=dev)
    torch.manual_seed(0)
    model = BiGCN(5000, 64, 64).to(dev)
    model.train()
    out = {}
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        for split in (True, False):
            st = FusedTrainStep(model, tddroprate=0.2, budroprate=0.2, drop_seed=5)
            if split:
                st.forward_backward(b, seed=11, defer_dw1=True)
                wa = dist.all_reduce(st.bucket.flat_a, op=dist.ReduceOp.SUM, async_op=True)
                st.finish_dw1()
                wb = dist.all_reduce(st.bucket.flat_b, op=dist.ReduceOp.SUM, async_op=True)
                wa.wait()
                wb.wait()
            else:
                st.forward_backward(b, seed=11)
                dist.all_reduce(st.bucket.flat, op=dist.ReduceOp.SUM)
            out[split] = st.bucket.flat.clone()
            st.check_status()
    torch.cuda.synchronize()
    assert out[True].numel() == out[False].numel() and out[True].abs().sum() > 0
    assert torch.equal(out[True], out[False]), float((out[True] - out[False]).abs().max())
    # the bucket's own RCCL helpers on the same group (world 1: a no-op, as documented)
    assert st.bucket.allreduce_part_async("a") is None
    dist.barrier()
    dist.destroy_process_group()
    print("rccl ok")


if __name__ == "__main__":
    main()
