"""One rank of the GPU data-parallel test (tests/test_gpu_dp.py): the fused HIP training
step on this rank's shard, the gradient bucket all-reduced over torch.distributed
(gloo here: several ranks share the box's single GPU, which RCCL does not allow), the
fused Adam.  Writes the first step's reduced gradients and the final parameters."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def shard_batches(rank: int, steps: int, dev):
    """The batches rank ``rank`` trains on (step-indexed, seeded)."""
    from bigcn_amd.data import synth_batch, synth_tree_sizes
    out = []
    for it in range(steps):
        rng = np.random.default_rng(9000 + 100 * it + rank)
        sizes = synth_tree_sizes(rng, 8, 90)
        out.append(synth_batch(rng, sizes, 5000, 4, device=dev))
    return out


def make_model(dev):
    from bigcn_amd import BiGCN
    from oracle import bigcn_oracle as O
    m = BiGCN(5000, 64, 64).to(dev)
    m.load_state_dict({k: v.float() for k, v in O.make_params(5000, 64, 64, 4, seed=31).items()})
    return m


def main():
    out_dir = sys.argv[1]
    from bigcn_amd import FusedTrainStep
    from bigcn_amd.dp import init_from_env
    rank, world, _ = init_from_env("gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    m = make_model(dev)
    res = {}
    # phase 1: eval mode (no dropout), 3 steps; the first step's reduced gradients are
    # compared with a single process training on the concatenation of the shards
    m.eval()
    step = FusedTrainStep(m)
    for it, b in enumerate(shard_batches(rank, 3, dev)):
        step(b)
        if it == 0:
            res["grads0"] = (torch.cat([v.reshape(-1) for v in step.bucket.views()]) / world).cpu().numpy()
    # phase 2: training mode, dropout drawn per rank, DropEdge on the device, prefetch
    m.train()
    step2 = FusedTrainStep(m, step.opt, tddroprate=0.2, budroprate=0.2, drop_seed=77 + rank)
    bs = shard_batches(rank, 3, dev)
    for it, b in enumerate(bs):
        step2(b, seed=1000 * rank + it, next_data=bs[it + 1] if it + 1 < len(bs) else None)
    torch.cuda.synchronize()
    step.check_status()
    step2.check_status()
    for k, v in m.state_dict().items():
        res["param:" + k] = v.cpu().numpy()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **res)
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
