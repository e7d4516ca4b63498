"""Data-parallel training over propagation trees (one process per GPU).

The reference is single-device (``BiGCN_Twitter.py:367``).  Trees are independent,
so the batch shards with no halo exchange: each rank builds its own graphs and runs
the fused encoder on its own 128 trees; the only exchange is one all-reduce of the
flat fp32 gradient bucket (1,289,476 params = 5.16 MB for the Twitter model) per
step over RCCL (torch.distributed backend "nccl" on ROCm) / gloo on CPU, followed by
the same Adam step on every rank.
"""
from __future__ import annotations

import os
from typing import Iterable, List

import torch
import torch.distributed as dist


def init_from_env(backend: str = "nccl"):
    """Initialise the process group from torchrun's env (RANK, WORLD_SIZE, MASTER_*).
    Returns (rank, world_size, local_rank); (0, 1, 0) without a launcher."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 0, 1, 0
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    if not dist.is_initialized():
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


class GradBucket:
    """One flat gradient bucket for all parameters (fixed order)."""

    def __init__(self, params: Iterable[torch.nn.Parameter]):
        self.params: List[torch.nn.Parameter] = [p for p in params if p.requires_grad]
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)

    def allreduce_mean(self, group=None) -> None:
        """grads <- mean over ranks of grads (sum all-reduce, then / world)."""
        if not dist.is_initialized() or dist.get_world_size(group) == 1:
            return
        world = dist.get_world_size(group)
        off = 0
        for p in self.params:
            n = p.numel()
            if p.grad is None:
                self.flat[off:off + n].zero_()
            else:
                self.flat[off:off + n].copy_(p.grad.view(-1))
            off += n
        dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group)
        self.flat.div_(world)
        off = 0
        for p in self.params:
            n = p.numel()
            if p.grad is None:
                p.grad = torch.empty_like(p)
            p.grad.view(-1).copy_(self.flat[off:off + n])
            off += n
