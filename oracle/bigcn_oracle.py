"""CPU oracle for the BiGCN bidirectional message-passing path.

TEST INFRASTRUCTURE ONLY.  Nothing under ``bigcn_amd/`` imports this module; only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
use it, and only as the checker / the timed CPU baseline.

What it restates (plain PyTorch, CPU, op for op):

* ``model/Twitter/BiGCN_Twitter.py:19-131`` (TDrumorGCN / BUrumorGCN / BiGCN) and
  ``model/Weibo/BiGCN_Weibo.py:16-89`` (same math, 2-class ``Net`` head), including
  the five semantic traps listed in SURVEY.md section 0:
  detached ``x2 = copy.copy(h1)`` (``BiGCN_Twitter.py:44``), dropout over the whole
  ``[N, 64+F]`` concat (``:51-54``), global ``rootindex`` (PyG collation), target-degree
  normalisation with self loops appended after the edges, lin -> propagate -> +bias.
* The third-party operators the reference calls but does not vendor:
  ``torch_geometric.nn.GCNConv`` (PyG >= 2.0 semantics, ``gcn_norm`` +
  ``add_remaining_self_loops`` + ``MessagePassing(aggr='add')``; the PyG 1.x
  source-degree convention is selectable with ``degree_on='row'``) and
  ``torch_scatter.scatter_mean`` (sum / count.clamp(min=1), dim_size = index.max()+1).
* The optimiser of ``BiGCN_Twitter.py:146-153`` / ``:186-189`` (Adam, three groups,
  BU convs at lr/5, weight_decay as L2 in the gradient).

PARITY PINNING.  torch_geometric / torch_scatter are not installed in this image
and the reference ships no tests or golden vectors for this arithmetic, so the
GCNConv / scatter_mean arithmetic here is **parity unpinned** by the reference
itself: it follows the published PyG-2.x / torch_scatter algorithms (cited per
function) and is cross-checked against hand-derived closed forms in
``tests/test_oracle.py``.  The on-disk / in-memory data format IS pinned: the
fixtures in ``tests/golden/format_*.npz`` were produced by the reference's own
``Process/getTwittergraph.py:constructMat/getfeature`` (``oracle/gen_golden.py``).
"""
from __future__ import annotations

import copy
from typing import Dict, List, Optional, Sequence

import torch
import torch.nn.functional as F

__all__ = [
    "add_remaining_self_loops", "gcn_norm", "gcn_conv", "scatter_mean",
    "root_extend", "BiGCNParams", "direction_forward", "bigcn_forward",
    "bigcn_loss", "make_params", "make_optimizer", "train_step",
]


# ----------------------------------------------------------------------------
# torch_geometric (>= 2.0) operators, restated
# ----------------------------------------------------------------------------
def add_remaining_self_loops(edge_index: torch.Tensor, edge_weight: Optional[torch.Tensor],
                             num_nodes: int, fill_value: float = 1.0, dtype=torch.float32):
    """PyG ``utils.add_remaining_self_loops`` (called from ``gcn_norm``; the reference
    reaches it through every ``GCNConv`` call, ``BiGCN_Twitter.py:42,56,92,105``, and
    names it explicitly at ``explain_PHEME.py:62-63``).

    Existing self loops are removed from the edge list (their weight becomes the
    loop weight), then one loop ``(i, i)`` per node is appended AFTER the edges.
    """
    row, col = edge_index[0], edge_index[1]
    mask = row != col
    if edge_weight is None:
        edge_weight = torch.ones(edge_index.size(1), dtype=dtype)
    loop_index = torch.arange(num_nodes, dtype=torch.long)
    loop_weight = torch.full((num_nodes,), fill_value, dtype=edge_weight.dtype)
    inv = ~mask
    if bool(inv.any()):
        loop_weight[row[inv]] = edge_weight[inv]
    ei = torch.cat([edge_index[:, mask], torch.stack([loop_index, loop_index])], dim=1)
    ew = torch.cat([edge_weight[mask], loop_weight])
    return ei, ew


def gcn_norm(edge_index: torch.Tensor, edge_weight: Optional[torch.Tensor], num_nodes: int,
             degree_on: str = "col", dtype=torch.float32):
    """PyG ``nn.conv.gcn_conv.gcn_norm(improved=False, add_self_loops=True,
    flow='source_to_target')``.  ``degree_on='col'`` is PyG >= 1.6 (target degree);
    ``'row'`` is PyG 1.3.2 (source degree, the version ``readme.md:28`` pins)."""
    ei, ew = add_remaining_self_loops(edge_index, edge_weight, num_nodes, dtype=dtype)
    row, col = ei[0], ei[1]
    idx = col if degree_on == "col" else row
    deg = torch.zeros(num_nodes, dtype=ew.dtype).scatter_add_(0, idx, ew)
    dinv = deg.pow(-0.5)
    dinv = dinv.masked_fill(dinv == float("inf"), 0.0)
    norm = dinv[row] * ew * dinv[col]
    return ei, norm


def gcn_conv(x: torch.Tensor, edge_index: torch.Tensor, weight: torch.Tensor,
             bias: Optional[torch.Tensor], edge_weight: Optional[torch.Tensor] = None,
             degree_on: str = "col") -> torch.Tensor:
    """PyG ``GCNConv.forward`` (2.x): ``h = lin(x)`` (``lin.weight [out,in]``, no bias),
    ``out[i] = sum_{e: col_e = i} norm_e * h[row_e]`` (message = norm * x_j, aggr add,
    edges in order, self loops last), then ``+ bias``."""
    n = x.size(0)
    ei, norm = gcn_norm(edge_index, edge_weight, n, degree_on, dtype=x.dtype)  # PyG passes x.dtype
    h = x @ weight.t()
    msg = norm.view(-1, 1) * h.index_select(0, ei[0])
    out = torch.zeros(n, h.size(1), dtype=h.dtype).index_add_(0, ei[1], msg)
    if bias is not None:
        out = out + bias
    return out


# ----------------------------------------------------------------------------
# torch_scatter.scatter_mean, restated
# ----------------------------------------------------------------------------
def scatter_mean(src: torch.Tensor, index: torch.Tensor, dim: int = 0,
                 dim_size: Optional[int] = None) -> torch.Tensor:
    """torch_scatter ``scatter_mean(src, index, dim=0)`` (called at
    ``BiGCN_Twitter.py:65,113``): ``sum / count.clamp(min=1)``, output rows =
    ``index.max()+1`` unless ``dim_size`` is given."""
    assert dim == 0
    if dim_size is None:
        dim_size = int(index.max()) + 1 if index.numel() else 0
    out = torch.zeros(dim_size, *src.shape[1:], dtype=src.dtype)
    out = out.index_add(0, index, src)
    cnt = torch.zeros(dim_size, dtype=src.dtype).index_add_(0, index, torch.ones(index.numel(), dtype=src.dtype))
    cnt = cnt.clamp(min=1)
    return out / cnt.view(-1, *([1] * (src.dim() - 1)))


# ----------------------------------------------------------------------------
# The BiGCN model (BiGCN_Twitter.py:19-131)
# ----------------------------------------------------------------------------
def root_extend(src: torch.Tensor, batch: torch.Tensor, rootindex: torch.Tensor) -> torch.Tensor:
    """The Python loop of ``BiGCN_Twitter.py:46-50`` / ``:59-63``, kept as a loop."""
    out = torch.zeros(len(batch), src.size(1), dtype=src.dtype)
    batch_size = int(batch.max()) + 1                # the reference's max(batch)
    for b in range(batch_size):
        index = torch.eq(batch, b)
        out[index] = src[rootindex[b]]
    return out


class BiGCNParams(dict):
    """Parameters keyed exactly like the reference ``state_dict`` (PyG-2.x layout)."""


def make_params(in_feats: int = 5000, hid: int = 64, out: int = 64, num_classes: int = 4,
                seed: int = 0, dtype=torch.float32) -> Dict[str, torch.Tensor]:
    """glorot-uniform ``lin.weight`` and zero ``bias`` (PyG GCNConv.reset_parameters);
    ``fc`` as ``torch.nn.Linear`` default init (``BiGCN_Twitter.py:122``).  Biases get
    small random values so that parity tests exercise the bias path."""
    g = torch.Generator().manual_seed(seed)

    def glorot(o, i):
        a = (6.0 / (i + o)) ** 0.5
        return (torch.rand(o, i, generator=g, dtype=torch.float64) * 2 * a - a).to(dtype)

    p = {}
    for d in ("TDrumorGCN", "BUrumorGCN"):
        p[f"{d}.conv1.lin.weight"] = glorot(hid, in_feats)
        p[f"{d}.conv1.bias"] = (torch.rand(hid, generator=g, dtype=torch.float64) * 0.2 - 0.1).to(dtype)
        p[f"{d}.conv2.lin.weight"] = glorot(out, hid + in_feats)
        p[f"{d}.conv2.bias"] = (torch.rand(out, generator=g, dtype=torch.float64) * 0.2 - 0.1).to(dtype)
    fin = (out + hid) * 2
    k = 1.0 / fin ** 0.5
    p["fc.weight"] = ((torch.rand(num_classes, fin, generator=g, dtype=torch.float64) * 2 - 1) * k).to(dtype)
    p["fc.bias"] = ((torch.rand(num_classes, generator=g, dtype=torch.float64) * 2 - 1) * k).to(dtype)
    return p


def _relu(h: torch.Tensor, mask: Optional[torch.Tensor]) -> torch.Tensor:
    """``F.relu``; with ``mask`` (bool, h's shape) the relu' decision is injected: h * mask.
    Only entries where h is within rounding of zero (a tie: +-1e-9 where the value is O(1))
    can differ from relu(h) - by at most that entry's magnitude in the forward value - but
    their gradient flips from 0 to 1 or back.  Parity tests at full size pass the kernel's
    own decisions so the comparison measures arithmetic error, not ties (test_gpu_fullsize)."""
    if mask is None:
        return F.relu(h)
    return h * mask.to(h.dtype)


def direction_forward(p: Dict[str, torch.Tensor], prefix: str, x: torch.Tensor,
                      edge_index: torch.Tensor, batch: torch.Tensor, rootindex: torch.Tensor,
                      training: bool = False, keep_mask: Optional[torch.Tensor] = None,
                      degree_on: str = "col", stages: Optional[dict] = None,
                      relu_masks=None) -> torch.Tensor:
    """``TDrumorGCN.forward`` (``BiGCN_Twitter.py:26-67``) == ``BUrumorGCN.forward``
    (``:77-114``) with the direction's edge_index.  ``keep_mask`` ([N, hid+F] bool)
    injects the dropout draw of ``:54`` (``F.dropout(p=0.5)`` keeps with prob 0.5 and
    scales by 2); ``None`` in training mode uses torch's own RNG like the reference.
    ``relu_masks`` (optional ``(m1 [N, hid], m2 [N, out])`` bool): the relu' decisions of
    the relu over conv1's columns of the concat (``:53``) and of the relu after conv2
    (``:57``), see ``_relu``."""
    w1, b1 = p[f"{prefix}.conv1.lin.weight"], p[f"{prefix}.conv1.bias"]
    w2, b2 = p[f"{prefix}.conv2.lin.weight"], p[f"{prefix}.conv2.bias"]
    m1, m2 = relu_masks if relu_masks is not None else (None, None)
    x1 = copy.copy(x.float())                                            # :28
    h = gcn_conv(x, edge_index, w1, b1, degree_on=degree_on)             # :42
    x2 = copy.copy(h)                                                    # :44  detached leaf
    # :46-54 - cat((h, root_extend(x1))), relu, dropout - evaluated per column block:
    # relu and the dropout are elementwise, so applying them to conv1's columns and to
    # the root-extend columns apart is the same tensor.  The root-extend block is a
    # constant (no parameter reaches it), so autograd's buffers stay 64 wide instead of
    # hid + F wide (the full-size parity tests run this at N > 100k, F = 5000).
    hid = h.size(1)
    root = F.relu(root_extend(x1, batch, rootindex).to(h.dtype))        # :46-51, :53
    h = F.relu(h) if m1 is None else _relu(h, m1)                        # :53 (decision injectable)
    if training:                                                         # :54
        if keep_mask is None:
            h = F.dropout(torch.cat((h, root), 1), training=True)
        else:
            h = torch.cat((h * keep_mask[:, :hid] * 2.0, root.mul_(keep_mask[:, hid:]).mul_(2.0)), 1)
    else:
        h = torch.cat((h, root), 1)
    del root
    if stages is not None:
        stages[f"{prefix}.h1"] = x2.detach().clone()
        stages[f"{prefix}.a2"] = h.detach()
    h = gcn_conv(h, edge_index, w2, b2, degree_on=degree_on)             # :56
    if stages is not None:
        stages[f"{prefix}.h2"] = h.detach().clone()
    h = _relu(h, m2)                                                     # :57
    if stages is not None:
        stages[f"{prefix}.r1"] = h.detach().clone()
    h = torch.cat((h, root_extend(x2, batch, rootindex)), 1)             # :59-63
    out = scatter_mean(h, batch, dim=0)                                  # :65
    if stages is not None:
        stages[f"{prefix}.out"] = out.detach().clone()
    return out


def bigcn_forward(p: Dict[str, torch.Tensor], x, td_edge_index, bu_edge_index, batch, rootindex,
                  training: bool = False, td_mask=None, bu_mask=None, degree_on: str = "col",
                  stages: Optional[dict] = None, relu_masks: Optional[dict] = None) -> torch.Tensor:
    """``BiGCN.forward`` (``BiGCN_Twitter.py:125-131``): TD first, BU second, concat
    **BU first** (``:128``), fc, log_softmax.  ``relu_masks``: {prefix: (m1, m2)}, see
    ``direction_forward``."""
    rm = relu_masks or {}
    td = direction_forward(p, "TDrumorGCN", x, td_edge_index, batch, rootindex, training, td_mask,
                           degree_on, stages, rm.get("TDrumorGCN"))
    bu = direction_forward(p, "BUrumorGCN", x, bu_edge_index, batch, rootindex, training, bu_mask,
                           degree_on, stages, rm.get("BUrumorGCN"))
    h = torch.cat((bu, td), 1)
    if stages is not None:
        stages["head_in"] = h.detach().clone()
    h = F.linear(h, p["fc.weight"], p["fc.bias"])
    return F.log_softmax(h, dim=1)


def bigcn_loss(logp: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """``F.nll_loss(out_labels, Batch_data.y)`` (``BiGCN_Twitter.py:184``)."""
    return F.nll_loss(logp, y)


def make_optimizer(p: Dict[str, torch.Tensor], lr: float = 5e-4, weight_decay: float = 1e-4):
    """Adam with three groups (``BiGCN_Twitter.py:146-153``): BU conv1/conv2 at lr/5."""
    bu1 = [p[k] for k in p if k.startswith("BUrumorGCN.conv1.")]
    bu2 = [p[k] for k in p if k.startswith("BUrumorGCN.conv2.")]
    base = [p[k] for k in p if not k.startswith("BUrumorGCN.conv")]
    return torch.optim.Adam([
        {"params": base},
        {"params": bu1, "lr": lr / 5},
        {"params": bu2, "lr": lr / 5},
    ], lr=lr, weight_decay=weight_decay)


def train_step(p: Dict[str, torch.Tensor], opt, batch: dict, training: bool = True,
               td_mask=None, bu_mask=None, degree_on: str = "col") -> float:
    """One step of the ``train_GCN`` batch loop (``BiGCN_Twitter.py:183-189``)."""
    logp = bigcn_forward(p, batch["x"], batch["edge_index"], batch["BU_edge_index"], batch["batch"],
                         batch["rootindex"], training, td_mask, bu_mask, degree_on)
    loss = bigcn_loss(logp, batch["y"])
    opt.zero_grad()
    loss.backward()
    val = loss.item()
    opt.step()
    return val


def params_requiring_grad(p: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    return {k: v.detach().clone().requires_grad_(True) for k, v in p.items()}


def reference_grads(p: Dict[str, torch.Tensor], batch: dict, training: bool = False,
                    td_mask=None, bu_mask=None, degree_on: str = "col",
                    stages: Optional[dict] = None, relu_masks: Optional[dict] = None):
    """Forward + NLL + backward on fresh leaf copies of ``p``; returns (loss, logp, grads)."""
    q = params_requiring_grad(p)
    logp = bigcn_forward(q, batch["x"], batch["edge_index"], batch["BU_edge_index"], batch["batch"],
                         batch["rootindex"], training, td_mask, bu_mask, degree_on, stages, relu_masks)
    loss = bigcn_loss(logp, batch["y"])
    loss.backward()
    return loss.detach(), logp.detach(), {k: v.grad.detach().clone() for k, v in q.items()}


# ----------------------------------------------------------------------------
# DropEdge (Process/dataset.py:68-90), restated for the device draw
# ----------------------------------------------------------------------------
_M64 = (1 << 64) - 1


def drop_key(seed: int, direction: int, e):
    """The 32-bit key of edge position ``e`` (numpy array) of list ``direction``
    (0 = TD, 1 = BU): splitmix64 finaliser with the salt used by bgcn_drop.hip."""
    import numpy as np
    e = np.asarray(e, dtype=np.uint64)
    with np.errstate(over="ignore"):
        base = np.uint64(((int(seed) & _M64) ^ 0xD1B54A32D192ED03) & _M64)
        z = base + np.uint64(0x9E3779B97F4A7C15) * (((e << np.uint64(1)) | np.uint64(direction))
                                                    + np.uint64(1))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(32)).astype(np.uint32)


def kept_count(length: int, droprate: float) -> int:
    """``int(length * (1 - droprate))`` exactly as ``dataset.py:72,84`` computes it
    (only applied when ``droprate > 0``)."""
    return int(length * (1 - droprate)) if droprate > 0 else int(length)


def drop_edges(edge_index, batch, num_graphs: int, droprate: float, seed: int, direction: int,
               masked: bool = False):
    """Per tree (edges grouped by tree in collation order, tree = batch[src]): keep the
    ``kept_count`` edges with the smallest (key, position), in original order - the
    device's uniform random subset, restated bit for bit.  Returns the kept [2, E']
    list, or with ``masked`` the [2, E] list holding, per tree, the kept edges in order
    followed by the dropped ones as self loops (d, d)."""
    import numpy as np
    ei = np.asarray(edge_index, dtype=np.int64)
    b = np.asarray(batch, dtype=np.int64)
    E = ei.shape[1]
    tree = b[ei[0]] if E else np.zeros(0, np.int64)
    assert np.all(np.diff(tree) >= 0), "edges must be grouped by tree"
    bounds = np.searchsorted(tree, np.arange(num_graphs + 1), side="left")
    keep = np.zeros(E, dtype=bool)
    for t in range(num_graphs):
        e0, e1 = int(bounds[t]), int(bounds[t + 1])
        k = kept_count(e1 - e0, droprate)
        pos = np.arange(e0, e1)
        order = np.lexsort((pos, drop_key(seed, direction, pos)))   # key, then position
        keep[pos[order[:k]]] = True
    if masked:   # per tree: kept edges in order, then the dropped ones as loops (d, d)
        out = np.empty_like(ei)
        for t in range(num_graphs):
            e0, e1 = int(bounds[t]), int(bounds[t + 1])
            kt, dr = keep[e0:e1], ~keep[e0:e1]
            seg = ei[:, e0:e1]
            nk = int(kt.sum())
            out[:, e0:e0 + nk] = seg[:, kt]
            out[0, e0 + nk:e1] = seg[1, dr]
            out[1, e0 + nk:e1] = seg[1, dr]
        return out
    return ei[:, keep]


# ----------------------------------------------------------------------------
# Dropout keep words (F.dropout p = 0.5 of BiGCN_Twitter.py:54 as drawn in-kernel):
# restatement of bgcn_common.h keep_word, bit-exact
# ----------------------------------------------------------------------------
def _mix32(x):
    import numpy as np
    x = np.asarray(x, dtype=np.uint32).copy()
    with np.errstate(over="ignore"):
        x ^= x >> np.uint32(16)
        x *= np.uint32(0x7FEB352D)
        x ^= x >> np.uint32(15)
        x *= np.uint32(0x846CA68B)
        x ^= x >> np.uint32(16)
    return x


def keep_words(seed: int, num_nodes: int, num_words: int):
    """[2, N, nw] uint32 keep words of the in-kernel dropout draw (bgcn_keep_words): word w
    of node i in direction d holds the keep bits of concat columns [32 w, 32 w + 32);
    ``mix32(mix32(i ^ seed_lo) ^ ((2 w + d) * 0x9E3779B9 + seed_hi))``."""
    import numpy as np
    seed = int(seed) & _M64
    s0, s1 = np.uint32(seed & 0xFFFFFFFF), np.uint32(seed >> 32)
    base = _mix32(np.arange(num_nodes, dtype=np.uint32) ^ s0)
    out = np.empty((2, num_nodes, num_words), dtype=np.uint32)
    w = np.arange(num_words, dtype=np.uint32)
    with np.errstate(over="ignore"):
        for d in range(2):
            c = ((w << np.uint32(1)) | np.uint32(d)) * np.uint32(0x9E3779B9) + s1
            out[d] = _mix32(base[:, None] ^ c[None, :])
    return out
