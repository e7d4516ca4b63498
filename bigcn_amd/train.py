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
import os
from typing import Optional

import torch

from . import _lib
from ._lib import BatchDesc, StepArgs, check, ptr, stream_handle, workspace
from .bigcn import BiGCN, _draw_seed, _num_graphs
from .dp import GradBucket
from .feed import PackedBatch
from .ops import HID, _FEAT_MODES, check_encoder_shapes, degree_code, feat_path, features, x_dtype_code
from .optim import IMAGE_BU_W1, IMAGE_BU_W2, IMAGE_TD_W1, IMAGE_TD_W2, FusedAdam, bigcn_adam


def _compacted(data) -> bool:
    """A host-fed batch whose features stay compacted (x never materialised): every
    PackedBatch whose rows fit the sparse path; one that overflows the spill pool is
    trained from its dense x (expanded on the device) like any collated batch."""
    return isinstance(data, PackedBatch) and data.fits_sparse


def _in_feats(data) -> int:
    return int(data.in_feats) if isinstance(data, PackedBatch) else int(data.x.size(1))


def _device(data):
    return data.device if isinstance(data, PackedBatch) else data.x.device


def _step_feat_mode(feat_mode: str, data) -> int:
    if _compacted(data):
        if feat_mode == "dense":
            raise ValueError("feat_mode 'dense' needs the dense x; this batch's features are compacted "
                             "(read batch.x to expand them)")
        return _lib.BGCN_FEAT_SPARSE
    return feat_path(feat_mode, data)


def _need(t: torch.Tensor, dtype, name: str) -> torch.Tensor:
    if t.dtype != dtype:
        t = t.to(dtype)
    if not t.is_contiguous():
        t = t.contiguous()
    return t


class FusedTrainStep:
    """``step = FusedTrainStep(model)``; ``loss = step(batch)`` per training batch.

    ``model``: :class:`bigcn_amd.BiGCN` / :class:`bigcn_amd.Net` (hid = out = 64).
    The loss a step returns is a 0-dim device tensor that keeps its value for the next
    4095 steps (a ring of loss slots: no allocation per step).
    ``optimizer``: a :class:`FusedAdam` over the model's parameters (default: the
    reference's three groups, :func:`bigcn_amd.optim.bigcn_adam`).  Gradients live in
    ``self.bucket`` (``grads()`` maps them back to the parameters)."""

    def __init__(self, model: BiGCN, optimizer: Optional[FusedAdam] = None, degree_on: Optional[str] = None,
                 group=None, tddroprate: float = 0.0, budroprate: float = 0.0,
                 drop_seed: Optional[int] = None, fuse_optimizer: Optional[bool] = None):
        self.model = model
        # DropEdge on the device (dataset.py:68-90): batches are then passed UNDROPPED
        # (BiGraphDataset(tddroprate=0, budroprate=0)) and each preparation draws its own
        # kept subsets; batch k prepared by this object uses drop seed drop_seed + k
        if not (0.0 <= tddroprate < 1.0 and 0.0 <= budroprate < 1.0):
            raise ValueError("droprates must be in [0, 1)")
        self.tddroprate, self.budroprate = float(tddroprate), float(budroprate)
        self._drop_seed = _draw_seed() if drop_seed is None else int(drop_seed)
        self._drop_count = 0
        self.last_drop_seed = None
        self.opt = optimizer if optimizer is not None else bigcn_adam(model)
        self.group = group
        # fuse_optimizer (single process): the optimiser step inside the training step's last
        # launch (bgcn_step_args.adam; bit-identical to the separate bgcn_adam_step, which the
        # library falls back to when the step cannot take it).  Off by default: its ~36 MB of
        # parameter / moment traffic lengthens the tail by as much as the separate launch
        # costs.  BGCN_FUSED_OPTIMIZER=1 turns it on when not given.
        if fuse_optimizer is None:
            fuse_optimizer = os.environ.get("BGCN_FUSED_OPTIMIZER", "0") == "1"
        self.fuse_optimizer = bool(fuse_optimizer)
        # the conv1 weight gradients (the step's last, bgcn_train_step_dw1) at the bucket's
        # end: with world > 1 the rest of the bucket is all-reduced while they compute
        enc = list(model.encoder_params())
        self.bucket = GradBucket(self.opt.params(), status_slot=True, late=[enc[0], enc[4]])
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
        # the gcn_norm convention is the model's (BiGCN.degree_on), so the fused step
        # trains with the normalisation model(data) evaluates with
        if degree_on is not None and degree_on != model.degree_on:
            raise ValueError(f"degree_on={degree_on!r} differs from the model's "
                             f"{model.degree_on!r}; set model.degree_on instead")
        self.degree_on = degree_code(model.degree_on)
        a = StepArgs()
        for k, (p, g) in enumerate(zip(self.step_params, self.step_grads)):
            a.params[k], a.grads[k] = ptr(p), ptr(g)
        a.num_classes = self.num_classes
        a.degree_on = self.degree_on
        self._args = a
        self.status = torch.zeros(1, dtype=torch.int32, device=model.fc.weight.device)
        # validity over many steps without a host sync per step: the OR of every step's
        # status (bgcn_step_args.status_seen) and the number of updates the fused Adam
        # skipped (bgcn_adam_args.skip_count); read by run_report()
        self.status_seen = torch.zeros(1, dtype=torch.int32, device=model.fc.weight.device)
        self.skipped = torch.zeros(1, dtype=torch.int32, device=model.fc.weight.device)
        self._pending = None       # (batch, prepared buffer, feat_mode, tensors) from next_data
        self._dw1_pending = None   # buffers of a defer_dw1 step until finish_dw1()
        self._stream = None
        self._next_desc = None
        # Weight images (W1^T, W2^T, the bf16 splits of W2[:, :64]) in a persistent buffer:
        # the fused Adam writes them with every update, so a step whose weights are those the
        # last update wrote launches no prologue.  They count as current while the weights'
        # version counters, storage and the optimiser's step count are what they were right
        # after that update (any torch in-place edit - load_state_dict, copy_ under no_grad -
        # or an optimiser step without the images makes the next step re-derive them).
        # Edits through ``p.data`` bypass the version counter: call invalidate_images().
        w = self.step_params
        self._img_params = (w[0], w[4], w[2], w[6])
        self._img_roles = {id(w[0]): IMAGE_TD_W1, id(w[4]): IMAGE_BU_W1,
                           id(w[2]): IMAGE_TD_W2, id(w[6]): IMAGE_BU_W2}
        self._images = None
        self._images_F = None
        self._images_key = None
        # Per-step device buffers are kept and reused (a torch.empty per buffer and step cost
        # ~9 us of host time each in the host-fed loop, tools/host_profile.py): the step
        # workspace, two prepared-batch buffers taken in turn (the batch a step trains on and
        # the next one its side lane prepares) and a ring of loss slots.  A buffer is kept per
        # stream (a call on another stream allocates afresh).
        self._bufs = {}
        self._loss_ring = None
        self._loss_at = 0
        # test hook: take the world > 1 branch of __call__ (defer_dw1 + the two async
        # all-reduces) on a one-rank process group, so the code an 8-GPU run executes is
        # exercised over RCCL on a one-GPU box (tests/nccl_gpu_worker.py)
        self._force_dp_overlap = False

    def _image_key(self):
        return (self.opt.step_count, tuple(p._version for p in self._img_params),
                tuple(p.data_ptr() for p in self._img_params))

    def invalidate_images(self) -> None:
        """Make the next step re-derive the weight images from the parameters (needed only
        after writing parameters behind torch's version counters, e.g. via ``p.data``)."""
        self._images_key = None

    def _image_buffer(self, F: int):
        if self._images is None or self._images_F != F:
            n = _lib.lib().bgcn_weight_images_size(F)
            # zeroed once: the rows' padding words are never written, so two steps' buffers
            # compare equal word for word when their images do
            self._images = workspace(n, self.status.device).zero_()
            self._images_F = F
            self._images_key = None
        return self._images

    def grads(self):
        """{parameter: gradient view} of the last step (before the DP all-reduce)."""
        return dict(zip(self.step_params, self.step_grads))

    def _desc(self, data, drop: bool = True):
        """bgcn_batch of a collated batch (+ the tensors it points into, kept alive);
        ``drop=False``: no DropEdge whatever the model's mode (evaluation batches)."""
        if _compacted(data):
            F = _in_feats(data)
            want = [(HID, F), (HID,), (HID, HID + F), (HID,)] * 2
            for p, shp in zip(self.step_params[:8], want):
                if tuple(p.shape) != shp:
                    raise ValueError(f"parameter of shape {tuple(p.shape)}, expected {shp} for in_feats={F}")
            d = BatchDesc()
            data.fill_desc(d)
            if drop:
                self._drop_fields(d)
            return d, (data,)
        x = features(data.x)                         # fp32, or bf16 kept as is
        check_encoder_shapes(x, data.batch, data.rootindex, self.step_params[:8])
        if data.rootindex.numel() != _num_graphs(data) or data.y.numel() != _num_graphs(data):
            raise ValueError("rootindex and y must have one entry per tree")
        td_ei = _need(data.edge_index, torch.int64, "edge_index")
        bu_ei = _need(data.BU_edge_index, torch.int64, "BU_edge_index")
        batch = _need(data.batch, torch.int64, "batch")
        root = _need(data.rootindex, torch.int64, "rootindex")
        d = BatchDesc()
        d.x, d.ldx, d.num_nodes, d.num_graphs = ptr(x), x.stride(0), x.size(0), _num_graphs(data)
        d.x_dtype = x_dtype_code(x)
        d.batch, d.rootindex = ptr(batch), ptr(root)
        d.td_edge_index, d.td_num_edges = ptr(td_ei), td_ei.size(1)
        d.bu_edge_index, d.bu_num_edges = ptr(bu_ei), bu_ei.size(1)
        if drop:
            self._drop_fields(d)
        return d, (x, td_ei, bu_ei, batch, root)

    def _drop_fields(self, d) -> None:
        if self.model.training and (self.tddroprate > 0 or self.budroprate > 0):
            d.td_droprate, d.bu_droprate = self.tddroprate, self.budroprate
            d.drop_seed = (self._drop_seed + self._drop_count) & (2**64 - 1)
            self._drop_count += 1

    def _buffer(self, key, nbytes: int) -> torch.Tensor:
        dev = self.status.device
        stream = stream_handle()
        b = self._bufs.get(key)
        if b is None or b[0].numel() < nbytes or b[1] != stream:
            # headroom: batches of one workload vary in size around their mean
            self._bufs[key] = b = (workspace(int(nbytes * 1.25) + 4096, dev), stream)
        return b[0]

    def _prep_buffer(self, d, F, avoid=None):
        """One of the two prepared-batch buffers, not ``avoid`` (the buffer of the batch the
        call trains on, while the other receives the next batch's preparation)."""
        L = _lib.lib()
        n = L.bgcn_prepare_workspace_size(d.num_nodes, d.num_graphs, F, d.td_num_edges, d.bu_num_edges)
        for k in (0, 1):
            b = self._bufs.get(("prep", k))
            if avoid is not None and b is not None and b[0] is avoid:
                continue
            return self._buffer(("prep", k), n)
        raise AssertionError("unreachable")

    def _loss_slot(self, dev) -> torch.Tensor:
        """A 0-dim fp32 device slot for the step's loss, from a ring of 4096: a returned loss
        tensor holds its value for the next 4095 calls."""
        if self._loss_ring is None or self._loss_ring.device != dev:
            self._loss_ring = torch.empty(4096, dtype=torch.float32, device=dev)
            self._loss_at = 0
        k = self._loss_at
        self._loss_at = (k + 1) % 4096
        return self._loss_ring[k]

    def forward_backward(self, data, seed: Optional[int] = None, logp: Optional[torch.Tensor] = None,
                         next_data=None, defer_dw1: bool = False, adam=None):
        """bgcn_train_step only (no all-reduce, no optimiser step); returns the loss.

        ``next_data``: the batch the next call will train on.  Its weight-independent
        preparation (K1, ELL and CSC of X) then runs inside this call on the auxiliary
        lane, overlapped with this step's latency-bound chain; the next call finds it
        ready (matched by identity - do not mutate the batch in between).  Every call
        still does exactly one preparation's worth of work.

        ``defer_dw1``: return before the conv1 weight gradients are written (every other
        gradient and the status slot are final); ``finish_dw1()`` writes them."""
        if self._dw1_pending is not None:
            # the previous step's conv1 weight gradients are not written yet: a new step
            # would reuse its workspace and the bucket would keep stale dW1 values
            raise RuntimeError("a step run with defer_dw1=True is pending: call finish_dw1() first")
        m = self.model
        F = _in_feats(data)
        dev = _device(data)
        y = _need(data.y, torch.int64, "y")
        if seed is None:
            seed = _draw_seed() if m.training else 0
        mode = _step_feat_mode(m.feat_mode, data)
        pend = self._pending
        if pend is not None and pend[0] is data and pend[2] == (mode == _lib.BGCN_FEAT_DENSE, m.training):
            # prepared by the previous call (its descriptor, drop seed and inputs)
            prep, keep, d = pend[1], pend[3], pend[4]
            ready = 1
        else:
            if pend is not None:   # a preparation no step consumes: order its end before
                self._join_side()   # its buffer returns to the allocator
            d, keep = self._desc(data)
            prep = self._prep_buffer(d, F)
            ready = 0
        a = self._args
        a.cur = d
        a.in_feats = F
        a.y = ptr(y)
        a.training, a.seed = int(m.training), int(seed) & (2**64 - 1)
        a.feat_mode = mode
        a.prepared_ready = ready
        a.prepared, a.prepared_bytes = ptr(prep), prep.numel()
        a.defer_dw1 = 1 if defer_dw1 else 0
        a.adam = ctypes.addressof(adam) if adam is not None else None   # (the optimiser's own struct)
        self._pending = None
        nxt = None
        if next_data is not None:
            nd, nkeep = self._desc(next_data)
            nbuf = self._prep_buffer(nd, F, avoid=prep)
            self._next_desc = nd                     # the struct must outlive the call
            a.next = ctypes.pointer(self._next_desc)
            a.next_prepared, a.next_prepared_bytes = ptr(nbuf), nbuf.numel()
            nxt = (next_data, nbuf, (mode == _lib.BGCN_FEAT_DENSE, m.training), nkeep, nd)
        else:
            a.next = None
            a.next_prepared, a.next_prepared_bytes = 0, 0
        self.last_drop_seed = int(a.cur.drop_seed) if a.cur.td_droprate > 0 or a.cur.bu_droprate > 0 else None
        loss = self._loss_slot(dev)
        a.loss, a.logp, a.status = ptr(loss), ptr(logp), ptr(self.status)
        a.status_flag = ptr(self.bucket.flag)
        a.status_seen = ptr(self.status_seen)
        img = self._image_buffer(F)
        a.images = ptr(img)
        a.images_current = int(self._images_key is not None and self._images_key == self._image_key())
        L = _lib.lib()
        N, B = d.num_nodes, d.num_graphs
        ws = self._buffer("ws", L.bgcn_train_step_workspace_size(N, B, F, self.num_classes, d.td_num_edges,
                                                                 d.bu_num_edges))
        # every branch the step forks joins back into the caller's stream inside the call
        # (the workspace can return to the allocator afterwards), except the next batch's
        # preparation, which outlives the call: its buffer is held in self._pending until
        # the next call (or _join_side()) has ordered a stream behind it
        self._stream = stream_handle()   # the prepared buffers belong to this stream
        self._last = (ws, N, B, F)       # the saved activations of this step (saved_activations)
        self._dw1_pending = (ws, prep, keep, y, img) if defer_dw1 else None
        self._pending = nxt              # held before the call: a failure below may leave
        try:                             # the preparation queued on the side lane
            check(L.bgcn_train_step(ctypes.addressof(a), ptr(ws), ws.numel(), self._stream))
        except Exception:
            self._dw1_pending = None     # the failed step wrote no gradients to finish
            if nxt is not None:
                self._join_side()        # nothing may still write the buffer once it is freed
                self._pending = None
            raise
        return loss

    def evaluate(self, data, next_data=None, logp: Optional[torch.Tensor] = None, pred: bool = False):
        """One evaluation batch of the reference's test loop (``BiGCN_Twitter.py:207-222``:
        ``model.eval(); val_out = model(Batch_data); val_loss = F.nll_loss(val_out, y);
        _, val_pred = val_out.max(dim=1); correct = val_pred.eq(y).sum()``) as one call
        (``bgcn_eval_step``): the forward in eval mode whatever ``model.training`` says (no
        dropout; no DropEdge, as the test set's ``BiGraphDataset``), the head, and the mean
        NLL, the argmax predictions and the correct count on the device - no host sync.

        Returns ``(loss, correct)`` (0-dim fp32 / int32 device tensors), plus ``pred`` ([B]
        int64 device tensor) when ``pred=True``.  ``logp``: an optional [B, C] fp32 output
        for the log-probabilities.  ``next_data``: the next evaluation batch, prepared on the
        side lane during this call.  Validity: ``check_status()`` / ``run_report()``."""
        if self._dw1_pending is not None:
            raise RuntimeError("a step run with defer_dw1=True is pending: call finish_dw1() first")
        m = self.model
        F = _in_feats(data)
        dev = _device(data)
        y = _need(data.y, torch.int64, "y")
        mode = _step_feat_mode(m.feat_mode, data)
        key = (mode == _lib.BGCN_FEAT_DENSE, False)
        pend = self._pending
        if pend is not None and pend[0] is data and pend[2] == key:
            prep, keep, d = pend[1], pend[3], pend[4]
            ready = 1
        else:
            if pend is not None:
                self._join_side()
            d, keep = self._desc(data, drop=False)
            prep = self._prep_buffer(d, F)
            ready = 0
        if logp is not None and (logp.dtype != torch.float32 or not logp.is_contiguous()
                                 or logp.numel() != d.num_graphs * self.num_classes):
            raise ValueError("logp must be a contiguous fp32 [B, C] tensor")
        a = self._args
        a.cur = d
        a.in_feats = F
        a.y = ptr(y)
        a.training, a.seed = 0, 0
        a.feat_mode = mode
        a.prepared_ready = ready
        a.prepared, a.prepared_bytes = ptr(prep), prep.numel()
        a.defer_dw1 = 0
        self._pending = None
        nxt = None
        if next_data is not None:
            nd, nkeep = self._desc(next_data, drop=False)
            nbuf = self._prep_buffer(nd, F, avoid=prep)
            self._next_desc = nd
            a.next = ctypes.pointer(self._next_desc)
            a.next_prepared, a.next_prepared_bytes = ptr(nbuf), nbuf.numel()
            nxt = (next_data, nbuf, key, nkeep, nd)
        else:
            a.next = None
            a.next_prepared, a.next_prepared_bytes = 0, 0
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        correct = torch.empty(1, dtype=torch.int32, device=dev)
        pr = torch.empty(d.num_graphs, dtype=torch.int64, device=dev) if pred else None
        a.loss, a.logp, a.status = ptr(loss), ptr(logp), ptr(self.status)
        a.status_flag = None
        a.status_seen = ptr(self.status_seen)
        img = self._image_buffer(F)
        a.images = ptr(img)
        current = self._images_key is not None and self._images_key == self._image_key()
        a.images_current = int(current)
        L = _lib.lib()
        N, B = d.num_nodes, d.num_graphs
        ws = self._buffer("ws", L.bgcn_train_step_workspace_size(N, B, F, self.num_classes, d.td_num_edges,
                                                                 d.bu_num_edges))
        self._stream = stream_handle()
        self._pending = nxt
        try:
            check(L.bgcn_eval_step(ctypes.addressof(a), ptr(correct), ptr(pr), ptr(ws), ws.numel(), self._stream))
        except Exception:
            if nxt is not None:
                self._join_side()
                self._pending = None
            raise
        # (stale images were re-derived into the buffer on the sparse path only, so the key
        # is left as it was: after a training step's Adam they are current anyway)
        out = (loss.view(()), correct.view(()))
        return out + (pr,) if pred else out

    def finish_dw1(self) -> None:
        """The conv1 weight gradients of a step run with ``defer_dw1`` (bgcn_train_step_dw1:
        same arguments and buffers, on the current stream)."""
        pend = getattr(self, "_dw1_pending", None)
        if pend is None:
            raise RuntimeError("no step with a deferred dW1 is pending")
        ws = pend[0]
        self._dw1_pending = None
        check(_lib.lib().bgcn_train_step_dw1(ctypes.addressof(self._args), ptr(ws), ws.numel(), stream_handle()))

    def __call__(self, data, seed: Optional[int] = None, logp: Optional[torch.Tensor] = None,
                 next_data=None):
        """One training step (the step, the all-reduce at world > 1, the optimiser update).

        Returns the loss as a 0-dim fp32 device tensor that is a VIEW into a ring of 4096
        loss slots: it keeps its value for the next 4095 calls and is then overwritten
        (no allocation per step).  Keep ``loss.item()`` or ``loss.clone()`` to hold a loss
        longer.  ``next_data``: see :meth:`forward_backward`."""
        world = self.bucket.world(self.group)
        overlap = (world > 1 or self._force_dp_overlap) and os.environ.get("BGCN_DP_OVERLAP", "1") != "0"
        if overlap:
            # the bucket in two all-reduces: everything but the conv1 weight gradients (and
            # the status slot) while the tail computes dW1, then dW1
            loss = self.forward_backward(data, seed, logp, next_data, defer_dw1=True)
            force = self._force_dp_overlap
            work_a = self.bucket.allreduce_part_async("a", self.group, force=force)
            self.finish_dw1()
            work_b = self.bucket.allreduce_part_async("b", self.group, force=force)
            for w in (work_a, work_b):
                if w is not None:
                    w.wait()
        elif world == 1 and self.fuse_optimizer:
            # the update inside the step (an invalid step skips it there, as below)
            F = _in_feats(data)
            adam = self.opt.prepare(grads=self.bucket.views(), grad_scale=1.0, skip_flag=self.bucket.flag,
                                    images=(self._image_buffer(F), F, self._img_roles), skip_count=self.skipped)
            loss = self.forward_backward(data, seed, logp, next_data, adam=adam)
            self.opt.step_count += 1
            self._images_key = self._image_key()
            return loss
        else:
            loss = self.forward_backward(data, seed, logp, next_data)
            self.bucket.allreduce_sum_(self.group)
        # an invalid step (status bits, any rank: the flag is summed by the all-reduce)
        # updates nothing; check_status() reports why
        self.opt.step(grads=self.bucket.views(), grad_scale=1.0 / world, skip_flag=self.bucket.flag,
                      images=(self._images, self._images_F, self._img_roles), skip_count=self.skipped)
        # the images now hold the updated weights (or, after an invalid step, the unchanged
        # ones: the launch skipped params and images alike)
        self._images_key = self._image_key()
        return loss

    def _join_side(self) -> None:
        """The current stream waits for the library's auxiliary lane (a next-batch
        preparation may still be running there when a step returns)."""
        check(_lib.lib().bgcn_join_side(self._stream))

    def discard_prefetch(self) -> None:
        """Drop a prepared next batch that will not be trained on (after ordering the
        current stream behind its preparation)."""
        if self._pending is not None:
            self._join_side()
            self._pending = None

    def __del__(self):
        try:
            if getattr(self, "_pending", None) is not None:
                self._join_side()
        except Exception:   # interpreter shutdown: nothing left to order
            pass

    def saved_activations(self):
        """(H1, H2) of the last step: the pre-relu conv1 / conv2 outputs, [N, 128] fp32
        device tensors (TD columns [0, 64), BU [64, 128)), views of the step's workspace
        (valid until the next step or evaluation call) - the per-stage intermediates the reference's
        explain_PHEME.py:91-162 dumps."""
        if getattr(self, "_last", None) is None:
            raise RuntimeError("no step has run yet")
        ws, N, B, F = self._last
        h1, h2 = ctypes.c_void_p(), ctypes.c_void_p()
        check(_lib.lib().bgcn_train_step_saved(ptr(ws), ws.numel(), N, B, F, self.num_classes,
                                               ctypes.byref(h1), ctypes.byref(h2)))
        base = ws.data_ptr()
        n = N * 128
        out = []
        for p_ in (h1.value, h2.value):
            off = p_ - base
            if off % 4 or off < 0 or off + 4 * n > ws.numel():
                raise RuntimeError("activation view outside the step workspace")
            out.append(ws[off:off + 4 * n].view(torch.float32).view(N, 128))
        return tuple(out)

    def run_report(self, reset: bool = False) -> dict:
        """Host sync: validity of every step since construction (or the last reset):
        ``status`` = the OR of the steps' status words (0: every step valid) and
        ``invalid_steps`` = the optimiser updates skipped because a step was invalid (on
        any rank).  Steps run through forward_backward() alone count in ``status`` only."""
        out = {"status": int(self.status_seen.item()), "invalid_steps": int(self.skipped.item())}
        if reset:
            self.status_seen.zero_()
            self.skipped.zero_()
        return out

    def check_status(self) -> None:
        """Host sync: raise on a bad edge index / batch id / label / (feat_mode "sparse")
        an over-full feature row / an internal time-out seen by the last step.  Any of them
        makes the step invalid: __call__'s optimiser update was skipped."""
        s = int(self.status.item())
        if s & 1:
            raise IndexError("edge_index or batch contains an index out of range "
                             "([0, num_nodes) / [0, num_graphs)), or a host-fed feature row a column "
                             "outside [0, in_feats) or out of ascending order")
        if s & 2:
            raise IndexError("label out of range [0, num_classes)")
        if s & 4:
            raise ValueError(f"feat_mode 'sparse': the batch's feature rows hold more non-zeros "
                             f"than the sparse path's ELL + spill pool ({_lib.BGCN_SPARSE_CAP} + "
                             f"{_lib.BGCN_SPARSE_SPILL_PER_ROW} per row of the batch; the step's "
                             f"results are invalid); use 'auto' or 'dense'")
        if s & 8:
            raise RuntimeError("libbgcn: an internal cross-workgroup hand-off timed out "
                               "(the step's results are invalid)")
