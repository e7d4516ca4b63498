"""One-call training step: ``bgcn_train_step`` + the data-parallel bucket + fused Adam.

The reference's loop body (``model/Twitter/BiGCN_Twitter.py:183-189``)::

    out_labels = model(Batch_data)                      # K1 + encoder + fc + log_softmax
    loss = F.nll_loss(out_labels, Batch_data.y)
    optimizer.zero_grad(); loss.backward(); optimizer.step()

as three device calls and no host sync: ``bgcn_train_step`` (graphs, forward, head,
loss and the complete backward, gradients written straight into the flat gradient
bucket), one RCCL all-reduce of the bucket when ``world > 1``, and ``bgcn_adam_step``
(the mean over ranks folded in as ``grad_scale``).  The per-op autograd path
(``BiGCN.forward`` + ``loss.backward()``) computes the same step; this is the
launch-lean form for training loops, where Python/autograd overhead would otherwise
exceed the device time of a 128-tree step.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _lib
from ._lib import StepArgs, check, ptr, stream_handle, workspace
from .bigcn import BiGCN, _draw_seed, _num_graphs
from .dp import GradBucket
from .ops import _FEAT_MODES
from .optim import FusedAdam, bigcn_adam


def _need(t: torch.Tensor, dtype, name: str) -> torch.Tensor:
    if t.dtype != dtype:
        t = t.to(dtype)
    if not t.is_contiguous():
        t = t.contiguous()
    return t


class FusedTrainStep:
    """``step = FusedTrainStep(model)``; ``loss = step(batch)`` per training batch.

    ``model``: :class:`bigcn_amd.BiGCN` / :class:`bigcn_amd.Net` (hid = out = 64).
    ``optimizer``: a :class:`FusedAdam` over the model's parameters (default: the
    reference's three groups, :func:`bigcn_amd.optim.bigcn_adam`).  Gradients live in
    ``self.bucket`` (``grads()`` maps them back to the parameters)."""

    def __init__(self, model: BiGCN, optimizer: Optional[FusedAdam] = None, degree_on: str = "col",
                 group=None):
        self.model = model
        self.opt = optimizer if optimizer is not None else bigcn_adam(model)
        self.group = group
        self.bucket = GradBucket(self.opt.params())
        by_id = {id(p): v for p, v in zip(self.bucket.params, self.bucket.views())}
        self.step_params = list(model.encoder_params()) + [model.fc.weight, model.fc.bias]
        missing = [i for i, p in enumerate(self.step_params) if id(p) not in by_id]
        if missing:
            raise ValueError("optimizer must manage every encoder and fc parameter")
        self.step_grads = [by_id[id(p)] for p in self.step_params]
        for p in self.step_params:
            if p.dtype != torch.float32 or not p.is_contiguous():
                raise ValueError("parameters must be contiguous fp32")
        self.num_classes = model.fc.out_features
        self.degree_on = 0 if degree_on == "col" else 1
        a = StepArgs()
        for k, (p, g) in enumerate(zip(self.step_params, self.step_grads)):
            a.params[k], a.grads[k] = ptr(p), ptr(g)
        a.num_classes = self.num_classes
        a.degree_on = self.degree_on
        self._args = a
        self.status = torch.zeros(1, dtype=torch.int32, device=model.fc.weight.device)

    def grads(self):
        """{parameter: gradient view} of the last step (before the DP all-reduce)."""
        return dict(zip(self.step_params, self.step_grads))

    def forward_backward(self, data, seed: Optional[int] = None, logp: Optional[torch.Tensor] = None):
        """bgcn_train_step only (no all-reduce, no optimiser step); returns the loss."""
        m = self.model
        x = _need(data.x, torch.float32, "x")
        N, F = x.shape
        B = _num_graphs(data)
        td_ei = _need(data.edge_index, torch.int64, "edge_index")
        bu_ei = _need(data.BU_edge_index, torch.int64, "BU_edge_index")
        batch = _need(data.batch, torch.int64, "batch")
        root = _need(data.rootindex, torch.int64, "rootindex")
        y = _need(data.y, torch.int64, "y")
        if seed is None:
            seed = _draw_seed() if m.training else 0
        a = self._args
        a.x, a.ldx, a.num_nodes, a.num_graphs, a.in_feats = ptr(x), x.stride(0), N, B, F
        a.batch, a.rootindex, a.y = ptr(batch), ptr(root), ptr(y)
        a.td_edge_index, a.td_num_edges = ptr(td_ei), td_ei.size(1)
        a.bu_edge_index, a.bu_num_edges = ptr(bu_ei), bu_ei.size(1)
        a.training, a.seed = int(m.training), int(seed) & (2**64 - 1)
        a.feat_mode = _FEAT_MODES[m.feat_mode]
        loss = torch.empty(1, dtype=torch.float32, device=x.device)
        a.loss, a.logp, a.status = ptr(loss), ptr(logp), ptr(self.status)
        L = _lib.lib()
        ws = workspace(L.bgcn_train_step_workspace_size(N, B, F, self.num_classes, a.td_num_edges,
                                                        a.bu_num_edges), x.device)
        # every auxiliary-lane branch joins back into the caller's stream inside the call,
        # so the workspace and converted inputs can return to the allocator afterwards
        check(L.bgcn_train_step(ctypes.addressof(a), ptr(ws), ws.numel(), stream_handle()))
        return loss.view(())

    def __call__(self, data, seed: Optional[int] = None, logp: Optional[torch.Tensor] = None):
        loss = self.forward_backward(data, seed, logp)
        world = self.bucket.world(self.group)
        self.bucket.allreduce_sum_(self.group)
        self.opt.step(grads=self.bucket.views(), grad_scale=1.0 / world)
        return loss

    def check_status(self) -> None:
        """Host sync: raise on a bad edge index / label seen by the last step."""
        s = int(self.status.item())
        if s & 1:
            raise IndexError("edge_index contains an index out of range [0, num_nodes)")
        if s & 2:
            raise IndexError("label out of range [0, num_classes)")
