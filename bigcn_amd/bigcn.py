"""BiGCN model classes with the reference's module structure and state_dict.

Mirrors ``model/Twitter/BiGCN_Twitter.py:19-131`` (``TDrumorGCN``, ``BUrumorGCN``,
``BiGCN``; 4 classes) and ``model/Weibo/BiGCN_Weibo.py:16-89`` (``Net``; 2 classes).
Attribute names (``conv1``, ``conv2``, ``fc``, ``TDrumorGCN``, ``BUrumorGCN``) and the
parameter layout are identical, so reference checkpoints load with ``load_state_dict``.

``BiGCN.forward`` runs the fused bidirectional encoder (:func:`bigcn_amd.ops.bigcn_encoder`:
both directions, conv1 for TD and BU in one pass over ``x``, the root extension /
relu / dropout generated inside the conv2 GEMM) and the ``fc`` + ``log_softmax`` head
(the K9 kernels) as one autograd node (:func:`bigcn_amd.ops.bigcn_net`).  ``TDrumorGCN.forward`` /
``BUrumorGCN.forward`` called on their own follow the reference op sequence with the
drop-in :class:`GCNConv` and :func:`scatter_mean`.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .conv import GCNConv
from .ops import (Graph, _feat_code, bigcn_encoder, bigcn_net, build_graph_pair, degree_code, feat_path,
                  head_fits, scatter_mean)


def _graphs(data, degree_on: str = "col"):
    """Build (once per batch object) the TD and BU graphs: gcn_norm + CSR (K1)."""
    cache = getattr(data, "_bgcn_graphs", None)
    if cache is not None and cache[0] == degree_on:
        return cache[1], cache[2]
    n = data.x.size(0)
    # with the batch vector K1 also checks that every edge stays inside its tree (the
    # encoder's fast readout backward relies on knowing it)
    batch = getattr(data, "batch", None)
    td, bu = build_graph_pair(data.edge_index, data.BU_edge_index, n, degree_on=degree_on,
                              batch=batch if batch is not None and batch.numel() == n else None)
    try:
        data._bgcn_graphs = (degree_on, td, bu)
    except AttributeError:
        pass
    return td, bu


def _num_graphs(data) -> int:
    ng = getattr(data, "num_graphs", None)
    if ng is None:
        ng = int(data.batch.max().item()) + 1  # the reference's max(data.batch)+1 (:47)
    return int(ng)


class _RumorGCN(torch.nn.Module):
    """Shared body of TDrumorGCN (``BiGCN_Twitter.py:19-67``) / BUrumorGCN (``:70-114``)."""

    edge_key = "edge_index"

    def __init__(self, in_feats, hid_feats, out_feats, device=None, degree_on: str = "col"):
        super().__init__()
        self.conv1 = GCNConv(in_feats, hid_feats, degree_on=degree_on)
        self.conv2 = GCNConv(hid_feats + in_feats, out_feats, degree_on=degree_on)
        self.device = device

    def forward(self, data):
        x = data.x.float()
        if self.conv1.degree_on != self.conv2.degree_on:
            raise ValueError("conv1 and conv2 must use the same degree_on convention")
        td, bu = _graphs(data, self.conv1.degree_on)
        g = td if self.edge_key == "edge_index" else bu
        batch, rootindex = data.batch, data.rootindex
        root_of_node = rootindex[batch]                       # :46-50 as one gather
        h1 = self.conv1(x, g)                                 # :42
        x2 = h1.detach()                                      # :44 copy.copy -> new leaf
        h = torch.cat((h1, x.index_select(0, root_of_node)), 1)  # :51
        h = F.relu(h)                                         # :53
        h = F.dropout(h, training=self.training)              # :54
        h = self.conv2(h, g)                                  # :56
        h = F.relu(h)                                         # :57
        h = torch.cat((h, x2.index_select(0, root_of_node)), 1)  # :59-63
        return scatter_mean(h, batch, dim=0, dim_size=_num_graphs(data))  # :65


class TDrumorGCN(_RumorGCN):
    edge_key = "edge_index"


class BUrumorGCN(_RumorGCN):
    edge_key = "BU_edge_index"


def _draw_seed() -> int:
    # host-side draw from torch's default generator: reproducible under torch.manual_seed,
    # no device sync
    return int(torch.randint(0, 2**62, (1,), dtype=torch.int64).item())


class BiGCN(torch.nn.Module):
    """``BiGCN(in_feats, hid_feats, out_feats, device)`` (``BiGCN_Twitter.py:117-131``).

    ``degree_on``: gcn_norm degree convention of every GCNConv of the model - ``'col'``
    (PyG >= 1.6, target degree; the fork's) or ``'row'`` (PyG 1.3.2, source degree).  It
    is one model-wide setting (the ``degree_on`` property sets all four convolutions), so
    the per-op path, the fused encoder and :class:`FusedTrainStep` always agree."""

    num_classes = 4

    def __init__(self, in_feats, hid_feats, out_feats, device=None, degree_on: str = "col"):
        super().__init__()
        if hid_feats != 64 or out_feats != 64:
            raise ValueError("the fused MI355X encoder is specialised for hid = out = 64 "
                             "(the reference configuration, BiGCN_Twitter.py:144)")
        degree_code(degree_on)
        self.TDrumorGCN = TDrumorGCN(in_feats, hid_feats, out_feats, device, degree_on)
        self.BUrumorGCN = BUrumorGCN(in_feats, hid_feats, out_feats, device, degree_on)
        self.fc = torch.nn.Linear((out_feats + hid_feats) * 2, self.num_classes)
        self.device = device
        self.keep_words = None  # optional injected dropout draw (tests)
        self.feat_mode = "auto"  # "auto": sparse feature path with device-side dense fallback
        # True: fc + log_softmax run as the K9 head kernels inside the encoder's autograd
        # node (bigcn_net) whenever fc fits them; False: torch's Linear + log_softmax
        self.fused_head = True

    def _convs(self):
        return (self.TDrumorGCN.conv1, self.TDrumorGCN.conv2, self.BUrumorGCN.conv1, self.BUrumorGCN.conv2)

    @property
    def degree_on(self) -> str:
        conv = {c.degree_on for c in self._convs()}
        if len(conv) != 1:
            raise ValueError(f"the model's GCNConvs disagree on degree_on: {sorted(conv)}")
        return conv.pop()

    @degree_on.setter
    def degree_on(self, value: str) -> None:
        degree_code(value)
        for c in self._convs():
            c.degree_on = value

    def _feat(self, data):
        # "auto" with the batch's hints (bound to x's identity and version) saying its rows
        # fit: BGCN_FEAT_SPARSE, the dense fallback kernels are not launched at all; every
        # other case keeps the device-gated fallback (the encoder entry points have no
        # status word to report a batch that does not fit)
        return feat_path("auto", data) if self.feat_mode == "auto" else self.feat_mode

    def encoder_params(self):
        t, b = self.TDrumorGCN, self.BUrumorGCN
        return (t.conv1.lin.weight, t.conv1.bias, t.conv2.lin.weight, t.conv2.bias,
                b.conv1.lin.weight, b.conv1.bias, b.conv2.lin.weight, b.conv2.bias)

    def _inputs(self, data):
        """(td, bu, prep, feat code): the batch's preparation when a data pipeline attached
        one that is still of this batch (``feed.prepare_ahead``: no K1 and no pass over X in
        the forward), else its graphs (built once per batch object)."""
        feat = self._feat(data)
        prep = getattr(data, "_bgcn_prep", None)
        if prep is not None and prep.matches(data, self.degree_on, _feat_code(feat)):
            return None, None, prep, feat
        td, bu = _graphs(data, self.degree_on)
        return td, bu, None, feat

    def encode(self, data, seed=None):
        td, bu, prep, feat = self._inputs(data)
        if seed is None:
            seed = _draw_seed() if self.training else 0
        return bigcn_encoder(data.x, data.batch, data.rootindex, td, bu, _num_graphs(data),
                             self.encoder_params(), training=self.training, seed=seed,
                             keep_words=self.keep_words, feat_mode=feat, prep=prep)

    def forward(self, data, seed=None):
        if self.fused_head and head_fits(self.fc):
            # :126-130 as one autograd node (encoder + the K9 fc / log_softmax kernels)
            td, bu, prep, feat = self._inputs(data)
            if seed is None:
                seed = _draw_seed() if self.training else 0
            return bigcn_net(data.x, data.batch, data.rootindex, td, bu, _num_graphs(data),
                             self.encoder_params(), self.fc.weight, self.fc.bias, training=self.training,
                             seed=seed, keep_words=self.keep_words, feat_mode=feat, prep=prep)
        x = self.encode(data, seed)            # cat(BU_x, TD_x)  (:126-128)
        x = self.fc(x)                         # :129
        return F.log_softmax(x, dim=1)         # :130


class Net(BiGCN):
    """Weibo head: ``Net(in_feats, hid_feats, out_feats)`` with ``fc(256 -> 2)``
    (``model/Weibo/BiGCN_Weibo.py:76-89``)."""

    num_classes = 2

    def __init__(self, in_feats, hid_feats, out_feats, device=None, degree_on: str = "col"):
        super().__init__(in_feats, hid_feats, out_feats, device, degree_on)


def make_optimizer(model: BiGCN, lr: float = 5e-4, weight_decay: float = 1e-4, fused: bool = False):
    """Adam with the reference's three groups (``BiGCN_Twitter.py:146-153``)."""
    bu_ids = {id(p) for p in model.BUrumorGCN.conv1.parameters()}
    bu_ids |= {id(p) for p in model.BUrumorGCN.conv2.parameters()}
    base = [p for p in model.parameters() if id(p) not in bu_ids]
    kw = {"fused": True} if fused else {}
    return torch.optim.Adam([
        {"params": base},
        {"params": list(model.BUrumorGCN.conv1.parameters()), "lr": lr / 5},
        {"params": list(model.BUrumorGCN.conv2.parameters()), "lr": lr / 5},
    ], lr=lr, weight_decay=weight_decay, **kw)
