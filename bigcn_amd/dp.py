"""Data-parallel training over propagation trees (one process per GPU).

The reference is single-device (``BiGCN_Twitter.py:367``).  Trees are independent,
so the batch shards with no halo exchange: each rank builds its own graphs and runs
the fused encoder on its own 128 trees; the only exchange is one all-reduce (sum) of
the flat fp32 gradient bucket (1,289,476 params = 5.16 MB for the Twitter model) per
step over RCCL (torch.distributed backend "nccl" on ROCm) / gloo on CPU.  The mean
(÷ world) is folded into the fused Adam step (``grad_scale``), which reads the reduced
bucket in place, so every rank applies the identical update.  The fused step all-reduces
the bucket in two parts: everything but the conv1 weight gradients while those are still
being computed (overlap the conv1 dW with communication), then the conv1
weights.
"""
from __future__ import annotations

import os
from typing import Iterable, List, Optional

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
    # BGCN_DIST_BACKEND overrides the backend (e.g. gloo to rehearse several ranks on one
    # GPU; ranks then share devices round-robin)
    backend = os.environ.get("BGCN_DIST_BACKEND", backend)
    if backend != "nccl" and torch.cuda.is_available() and torch.cuda.device_count() > 0:
        local = local % torch.cuda.device_count()
    if not dist.is_initialized():
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


class GradBucket:
    """One flat gradient bucket for all parameters (fixed order).

    ``status_slot``: one extra fp32 element after the gradients (``self.flag``).  The
    fused step writes its validity flag there, so the same all-reduce that sums the
    gradients also tells every rank whether any rank's step was invalid (the fused Adam
    then skips the update everywhere, keeping the replicas identical)."""

    def __init__(self, params: Iterable[torch.nn.Parameter], status_slot: bool = False,
                 late: Iterable[torch.nn.Parameter] = ()):
        self.params: List[torch.nn.Parameter] = [p for p in params if p.requires_grad]
        self.numels = [p.numel() for p in self.params]
        dev = self.params[0].device
        # Layout: [early gradients | status slot | late gradients].  ``late`` parameters
        # (the conv1 weights of the deferred-dW1 step) sit at the end, so the bucket
        # all-reduces in two contiguous parts: ``flat_a`` (every other gradient and the
        # status slot) while the late gradients are still being computed, then ``flat_b``.
        # Every view starts on a 16-byte boundary (the kernels' float4 paths; a Weibo head
        # bias of 2 elements would otherwise misalign every parameter after it); the gaps
        # stay zero through the all-reduce.
        late_ids = {id(p) for p in late}
        order = [i for i, p in enumerate(self.params) if id(p) not in late_ids] + \
                [i for i, p in enumerate(self.params) if id(p) in late_ids]
        self.late = [self.params[i] for i in order if id(self.params[i]) in late_ids]
        offs, n = [0] * len(self.params), 0
        n_a = None
        for i in order:
            if n_a is None and id(self.params[i]) in late_ids:
                n_a = n + (4 if status_slot else 0)
                n = n_a
            offs[i] = n
            n += (self.numels[i] + 3) // 4 * 4
        flag_at = n_a - 4 if (n_a is not None and status_slot) else n
        if n_a is None:
            n_a = n + (1 if status_slot else 0)
        total = max(n_a, n) if self.late else n_a
        self._packed = all(k % 4 == 0 for k in self.numels) and not self.late   # one cat fills it
        self.flat = torch.zeros(total, dtype=torch.float32, device=dev)
        self.flag = self.flat[flag_at:flag_at + 1] if status_slot else None
        self.flat_a = self.flat[:n_a]        # early gradients + the status slot
        self.flat_b = self.flat[n_a:]        # the late gradients (empty without late params)
        self._views = [self.flat[o:o + k].view_as(p) for o, k, p in zip(offs, self.numels, self.params)]

    def views(self) -> List[torch.Tensor]:
        """Persistent per-parameter views of the flat bucket (parameter order): kernels
        can write gradients straight into them (bgcn_train_step)."""
        return self._views

    def allreduce_sum_(self, group=None) -> None:
        """In-place SUM of the bucket over ranks (one RCCL all-reduce; no-op at world 1)."""
        if dist.is_initialized() and self.world(group) > 1:
            dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group)

    def allreduce_part_async(self, part: str, group=None, force: bool = False):
        """Start the in-place SUM of one part ("a": early gradients + status slot, "b": the
        late gradients) and return the work handle (None at world 1 or for an empty part):
        ``work.wait()`` orders the current stream behind the collective.  ``force``: issue
        the collective on a one-rank group too (test hook)."""
        t = self.flat_a if part == "a" else self.flat_b
        if t.numel() == 0 or not dist.is_initialized() or (self.world(group) <= 1 and not force):
            return None
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=True)

    def world(self, group=None) -> int:
        return dist.get_world_size(group) if dist.is_initialized() else 1

    def reduce_sum(self, group=None) -> List[torch.Tensor]:
        """Concatenate the grads (one copy kernel), all-reduce SUM in place, and return
        views of the reduced bucket in parameter order (the caller divides by world)."""
        grads = [p.grad.reshape(-1) if p.grad is not None else torch.zeros(n, device=self.flat.device)
                 for p, n in zip(self.params, self.numels)]
        if self._packed:
            torch.cat(grads, out=self.flat[:sum(self.numels)])
        else:
            for v, g in zip(self._views, grads):
                v.view(-1).copy_(g)
        self.allreduce_sum_(group)
        return self._views

    def allreduce_mean(self, group=None) -> None:
        """In-place mean of p.grad over ranks (for torch optimisers)."""
        world = self.world(group)
        if world == 1:
            return
        views = self.reduce_sum(group)
        for p, v in zip(self.params, views):
            if p.grad is None:
                p.grad = torch.empty_like(p)
            p.grad.copy_(v).div_(world)
