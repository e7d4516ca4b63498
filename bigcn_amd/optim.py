"""Fused Adam for the BiGCN training loop (one HIP launch per step).

Mirrors ``torch.optim.Adam([{base}, {BU conv1, lr/5}, {BU conv2, lr/5}], lr=5e-4,
weight_decay=1e-4)`` of ``model/Twitter/BiGCN_Twitter.py:146-153`` (step at ``:189``):
same update rule (amsgrad off, weight decay as L2 in the gradient), same parameter
groups and learning rates, kernel ``bgcn_adam_step`` in ``csrc/bgcn_optim.hip``.
"""
from __future__ import annotations

import ctypes
import math
from typing import Iterable, List, Optional, Sequence

import torch

from . import _lib
from ._lib import check, ptr, stream_handle

MAX_TENSORS = 16


class _AdamTensor(ctypes.Structure):
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
                ("exp_avg_sq", ctypes.c_void_p), ("numel", ctypes.c_int64), ("lr", ctypes.c_float)]


class AdamArgs(ctypes.Structure):
    _fields_ = [("t", _AdamTensor * MAX_TENSORS), ("block_start", ctypes.c_int64 * MAX_TENSORS),
                ("count", ctypes.c_int), ("beta1", ctypes.c_float), ("beta2", ctypes.c_float),
                ("eps", ctypes.c_float), ("weight_decay", ctypes.c_float),
                ("bias_correction1", ctypes.c_float), ("bias_correction2_sqrt", ctypes.c_float),
                ("grad_scale", ctypes.c_float), ("skip_flag", ctypes.c_void_p),
                ("images", ctypes.c_void_p), ("images_in_feats", ctypes.c_int64),
                ("image_role", ctypes.c_int32 * MAX_TENSORS), ("skip_count", ctypes.c_void_p)]

# BGCN_IMAGE_* (include/bgcn.h): which weight image a conv weight's update also writes
IMAGE_TD_W1, IMAGE_BU_W1, IMAGE_TD_W2, IMAGE_BU_W2 = 1, 2, 3, 4


class FusedAdam:
    """``param_groups``: list of dicts {"params": [...], "lr": float} (torch layout)."""

    def __init__(self, param_groups: Sequence[dict], lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0):
        self.param_groups = []
        for g in param_groups:
            ps = [p for p in g["params"]]
            self.param_groups.append({"params": ps, "lr": g.get("lr", lr)})
        self.betas, self.eps, self.weight_decay = betas, eps, weight_decay
        self.step_count = 0
        self.state = {}
        self._cache = None
        n = sum(len(g["params"]) for g in self.param_groups)
        if n > MAX_TENSORS:
            raise ValueError(f"FusedAdam handles at most {MAX_TENSORS} tensors")
        for g in self.param_groups:
            for p in g["params"]:
                if p.dtype != torch.float32 or not p.is_contiguous():
                    raise ValueError("FusedAdam: contiguous fp32 parameters only")
                self.state[p] = (torch.zeros_like(p), torch.zeros_like(p))

    def params(self) -> List[torch.nn.Parameter]:
        return [p for g in self.param_groups for p in g["params"]]

    def zero_grad(self, set_to_none: bool = True) -> None:
        for p in self.params():
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()

    def step(self, grads: Optional[Sequence[torch.Tensor]] = None, grad_scale: float = 1.0,
             skip_flag: Optional[torch.Tensor] = None, images=None,
             skip_count: Optional[torch.Tensor] = None) -> None:
        a = self.prepare(grads, grad_scale, skip_flag, images, skip_count)
        self.step_count += 1
        if a is not None:
            check(_lib.lib().bgcn_adam_step(ctypes.addressof(a), stream_handle()))

    def prepare(self, grads: Optional[Sequence[torch.Tensor]] = None, grad_scale: float = 1.0,
                skip_flag: Optional[torch.Tensor] = None, images=None,
                skip_count: Optional[torch.Tensor] = None):
        """The ``bgcn_adam_args`` of the next :meth:`step` (step count + 1) without launching it
        - for a caller that hands them to the training step (``bgcn_step_args.adam``, which
        performs the update inside the step) and then advances ``step_count`` itself; None when
        no parameter has a gradient.

        ``grads`` overrides ``p.grad`` (e.g. views of a reduced flat DP bucket).
        ``skip_flag``: a one-element fp32 device tensor; when it holds a non-zero value at
        execution time the launch updates nothing (an invalid training step, decided on
        the device without a host sync; the step counter still advances).
        ``skip_count``: a one-element int32 device tensor incremented on the device by
        every skipped update (the number of invalid steps of a run, read once).
        ``images``: ``(buffer, in_feats, {id(param): IMAGE_*})`` - the updates of those
        conv weights also write the weight images a :class:`FusedTrainStep` reads
        (``bgcn_weight_images_size``), so its next step derives nothing from the weights.

        Learning rates are read from ``param_groups`` on every call, so schedulers that
        edit ``group['lr']`` (as with torch.optim.Adam) take effect."""
        t = self.step_count + 1
        b1, b2 = self.betas
        ps = self.params()
        gs = list(grads) if grads is not None else [p.grad for p in ps]
        # the tensor table (parameter / moment pointers, sizes, groups) is built once per
        # set of present gradients and parameter / moment storage; only the gradient
        # pointers are written per step (autograd hands out fresh gradient tensors every
        # step).  The key holds every pointer the table captures, so reassigning p.data,
        # swapping a parameter in param_groups or replacing a moment rebuilds it.
        if len(ps) > MAX_TENSORS:
            raise ValueError(f"FusedAdam handles at most {MAX_TENSORS} tensors")
        for p in ps:
            if p not in self.state:   # a parameter added to param_groups after construction
                self.state[p] = (torch.zeros_like(p), torch.zeros_like(p))
        key = (tuple(g is None for g in gs),
               tuple((p.data_ptr(), p.numel(), self.state[p][0].data_ptr(), self.state[p][1].data_ptr())
                     for p in ps),
               tuple(len(g["params"]) for g in self.param_groups))
        cached = self._cache if getattr(self, "_cache", None) is not None and self._cache[0] == key else None
        if cached is None:
            a = AdamArgs()
            groups = []         # param_groups index of each table entry (lr refreshed per step)
            entries = []        # params() index of each table entry
            k = 0
            for gi, p in enumerate(ps):
                if gs[gi] is None:
                    continue
                entries.append(gi)
                m, v = self.state[p]
                e = a.t[k]
                e.param, e.exp_avg, e.exp_avg_sq = ptr(p), ptr(m), ptr(v)
                e.numel = p.numel()
                groups.append(self._group_of(p))
                k += 1
            a.count = k
            a.beta1, a.beta2, a.eps, a.weight_decay = b1, b2, self.eps, self.weight_decay
            cached = (key, a, [a.t[k] for k in range(k)], groups, entries)   # entry proxies
            self._cache = cached
        keep = []   # non-contiguous gradients: contiguous copies, alive through the launch
        a, ents, groups = cached[1], cached[2], cached[3]
        if a.count == 0:
            return None
        for e, gi, gj in zip(ents, cached[4], groups):
            gr = gs[gi]
            if not gr.is_contiguous():
                gr = gr.contiguous()
                keep.append(gr)
            e.grad = gr.data_ptr()
            e.lr = float(self.param_groups[gj]["lr"])
        if skip_flag is not None:
            if skip_flag.dtype != torch.float32 or skip_flag.numel() != 1 or skip_flag.device != ps[0].device:
                raise ValueError("skip_flag must be a one-element fp32 tensor on the parameters' device")
        a.skip_flag = ptr(skip_flag)
        if skip_count is not None and (skip_count.dtype != torch.int32 or skip_count.numel() != 1):
            raise ValueError("skip_count must be a one-element int32 tensor")
        a.skip_count = ptr(skip_count)
        a.bias_correction1 = 1.0 - b1 ** t
        a.bias_correction2_sqrt = math.sqrt(1.0 - b2 ** t)
        a.grad_scale = grad_scale
        if images is not None:
            buf, F, roles = images
            a.images, a.images_in_feats = ptr(buf), int(F)
            for k, gi in enumerate(self._entries(cached)):
                a.image_role[k] = roles.get(id(ps[gi]), 0)
        else:
            a.images, a.images_in_feats = None, 0
        self._keep = keep
        return a

    def _entries(self, cached):
        """params() index of each table entry (gradients that are None have no entry)."""
        return cached[4]

    def _group_of(self, p) -> int:
        for gi, g in enumerate(self.param_groups):
            if any(q is p for q in g["params"]):
                return gi
        raise KeyError("parameter not managed by this optimiser")


def bigcn_adam(model, lr: float = 5e-4, weight_decay: float = 1e-4) -> FusedAdam:
    """The reference's optimiser (``BiGCN_Twitter.py:146-153``) on FusedAdam."""
    bu_ids = {id(p) for p in model.BUrumorGCN.conv1.parameters()}
    bu_ids |= {id(p) for p in model.BUrumorGCN.conv2.parameters()}
    base = [p for p in model.parameters() if id(p) not in bu_ids]
    return FusedAdam([
        {"params": base},
        {"params": list(model.BUrumorGCN.conv1.parameters()), "lr": lr / 5},
        {"params": list(model.BUrumorGCN.conv2.parameters()), "lr": lr / 5},
    ], lr=lr, weight_decay=weight_decay)
