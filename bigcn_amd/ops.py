"""Autograd operators over the HIP kernels of libbgcn (the hot path of BiGCN).

* :class:`Graph` / :func:`build_graph` - ``gcn_norm`` + ``add_remaining_self_loops`` +
  CSR (K1), built once per batch and direction, shared by conv1/conv2 forward and
  backward (the reference recomputes it 4x per step, ``cached=False``).
* :func:`gcn_conv` - PyG-2.x ``GCNConv.forward`` (lin -> propagate -> +bias) with a
  HIP backward (K2, K3, K4, K10).
* :func:`scatter_mean` - ``torch_scatter.scatter_mean`` (K8).
* :func:`bigcn_encoder` - the fused TD+BU encoder of ``BiGCN.forward``
  (``model/Twitter/BiGCN_Twitter.py:125-128``), all of K1-K10 on the GPU.

Every function runs on the caller's current HIP stream and never falls back to a
CPU or PyTorch implementation.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _lib
from ._lib import BiGCNArgs, GraphView, check, ptr, stream_handle, workspace

HID = 64


def _dev_check(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise _lib.BGCNError("bigcn_amd ops take device tensors (no CPU path)")


# ----------------------------------------------------------------------------- K1
_GRAPH_I32 = ("t_ptr", "s_ptr", "t_row", "t_col", "s_row", "s_col")
_GRAPH_F32 = ("t_w", "s_w")
_SEG_ALIGN = 64   # elements: every array starts 256-byte aligned inside its buffer


class Graph:
    """Normalised adjacency of one direction in both CSR orientations.

    ``t_*`` rows are targets (forward aggregation, ``out[i] = sum norm * h[src]``),
    ``s_*`` rows are sources (the transposed product of the backward pass).  The arrays
    live in two flat buffers (int32 / fp32, shared by the TD and BU graphs of a pair);
    the per-array tensors are views made on first access - the kernels take pointers."""

    __slots__ = ("num_nodes", "num_edges", "capacity", "status", "_bufs", "_lay", "_views", "_ptrs", "_plan",
                 "_plan_ws", "_tree_checked")

    def _array(self, name: str) -> torch.Tensor:
        v = self._views.get(name)
        if v is None:
            k, off, n = self._lay[name]
            v = self._bufs[k].narrow(0, off, n)
            self._views[name] = v
        return v

    def view(self) -> GraphView:
        v = GraphView()
        q = self._ptrs
        v.t_ptr, v.t_row, v.t_col, v.t_w = q["t_ptr"], q["t_row"], q["t_col"], q["t_w"]
        v.s_ptr, v.s_row, v.s_col, v.s_w = q["s_ptr"], q["s_row"], q["s_col"], q["s_w"]
        v.capacity = self.capacity
        if self._plan is not None:   # the aggregation plans of bgcn_build_graph_pair
            v.plan[0], v.plan[1] = self._plan
        if self._tree_checked:       # built with the batch vector: status carries BGCN_STATUS_CROSS_TREE
            v.tree_status = self.status.data_ptr()
        return v

    def check(self) -> None:
        """Host sync: raise IndexError if edge_index held an index outside [0, N)."""
        s = int(self.status.item())
        if s & 8:
            raise RuntimeError("libbgcn: an internal cross-workgroup hand-off timed out")
        if s & ~_lib.BGCN_STATUS_CROSS_TREE:   # (an edge across trees is legal, only noted)
            raise IndexError("edge_index contains an index out of range [0, num_nodes)")


for _name in _GRAPH_I32 + _GRAPH_F32:
    setattr(Graph, _name, property(lambda self, _n=_name: self._array(_n)))


def _seg(n: int) -> int:
    return (n + _SEG_ALIGN - 1) // _SEG_ALIGN * _SEG_ALIGN


def _alloc_graphs(edges, N: int, dev, status=None):
    """Graphs of E = edges[k] edges over N nodes, all arrays carved from one int32 and
    one fp32 allocation."""
    ni = sum(2 * _seg(N + 1) + 4 * _seg(E + N) for E in edges)
    nf = sum(2 * _seg(E + N) for E in edges)
    bi = torch.empty(ni, dtype=torch.int32, device=dev)
    bf = torch.empty(nf, dtype=torch.float32, device=dev)
    pi, pf = bi.data_ptr(), bf.data_ptr()
    st = torch.zeros(1, dtype=torch.int32, device=dev) if status is None else status
    out, oi, of = [], 0, 0
    for E in edges:
        cap = E + N
        g = Graph()
        g.num_nodes, g.num_edges, g.capacity, g.status = N, E, cap, st
        g._bufs, g._views, g._lay, g._ptrs = (bi, bf), {}, {}, {}
        g._plan = g._plan_ws = None
        g._tree_checked = False
        for name in _GRAPH_I32:
            n = N + 1 if name.endswith("ptr") else cap
            g._lay[name], g._ptrs[name] = (0, oi, n), pi + 4 * oi
            oi += _seg(n)
        for name in _GRAPH_F32:
            g._lay[name], g._ptrs[name] = (1, of, cap), pf + 4 * of
            of += _seg(cap)
        out.append(g)
    return out


def _alloc_graph(E: int, N: int, dev, status=None) -> Graph:
    return _alloc_graphs((E,), N, dev, status)[0]


def _csr_out(g: Graph) -> _lib.CsrOut:
    c = _lib.CsrOut()
    q = g._ptrs
    c.t_ptr, c.t_row, c.t_col, c.t_w = q["t_ptr"], q["t_row"], q["t_col"], q["t_w"]
    c.s_ptr, c.s_row, c.s_col, c.s_w = q["s_ptr"], q["s_row"], q["s_col"], q["s_w"]
    return c


def degree_code(degree_on: str) -> int:
    """C-ABI code of a gcn_norm degree convention: 'col' (PyG >= 1.6: target degree) -> 0,
    'row' (PyG 1.3.2: source degree) -> 1; anything else raises."""
    if degree_on == "col":
        return 0
    if degree_on == "row":
        return 1
    raise ValueError(f"degree_on must be 'col' or 'row', got {degree_on!r}")


def _check_ei(edge_index: torch.Tensor) -> torch.Tensor:
    if edge_index.dim() != 2 or edge_index.size(0) != 2:
        raise ValueError("edge_index must be [2, E]")
    if edge_index.dtype == torch.int64 and edge_index.is_contiguous():
        return edge_index
    return edge_index.to(torch.int64).contiguous()


def build_graph_pair(td_edge_index: torch.Tensor, bu_edge_index: torch.Tensor, num_nodes: int,
                     degree_on: str = "col", validate: bool = False, batch: Optional[torch.Tensor] = None):
    """TD and BU graphs of one batch in one launch sequence (the fused step's K1).  The
    build's workspace (≈3.5 MB at Twitter size, about the graphs' own size) stays with the
    two graphs: it holds their aggregation plans (``bgcn_graph_pair_plans``).

    ``batch`` (the collated batch vector, optional): the build also notes on the device
    whether an edge joins two trees.  Only graphs built with it let the fused encoder take
    its sign-word readout backward (which handles such edges by per-neighbour scales);
    without it the encoder keeps the general readout backward."""
    _dev_check(td_edge_index, bu_edge_index, batch)
    if batch is not None:
        if batch.numel() != int(num_nodes):
            raise ValueError("batch must have one entry per node")
        batch = batch.to(torch.int64).contiguous()
    dcode = degree_code(degree_on)
    td_ei, bu_ei = _check_ei(td_edge_index), _check_ei(bu_edge_index)
    N = int(num_nodes)
    dev = td_ei.device
    td, bu = _alloc_graphs((int(td_ei.size(1)), int(bu_ei.size(1))), N, dev)
    L = _lib.lib()
    ws = workspace(L.bgcn_graph_pair_workspace_size(td.num_edges, bu.num_edges, N), dev)
    a, b = _csr_out(td), _csr_out(bu)
    check(L.bgcn_build_graph_pair(td_ei.data_ptr(), td.num_edges, bu_ei.data_ptr(), bu.num_edges, N,
                                  dcode, ctypes.byref(a), ctypes.byref(b), ptr(batch),
                                  td.status.data_ptr(), ws.data_ptr(), ws.numel(), stream_handle()))
    td._tree_checked = bu._tree_checked = batch is not None
    # the build leaves both graphs' aggregation plans in its workspace: keep it with the
    # graphs so the fused encoder takes the planned aggregation
    pt, pb = (_lib.SpmmPlan * 2)(), (_lib.SpmmPlan * 2)()
    check(L.bgcn_graph_pair_plans(ws.data_ptr(), ws.numel(), td.num_edges, bu.num_edges, N,
                                  ctypes.addressof(pt), ctypes.addressof(pb)))
    td._plan, bu._plan = (pt[0], pt[1]), (pb[0], pb[1])
    td._plan_ws = bu._plan_ws = ws
    if validate:
        td.check()
    return td, bu


def build_graph(edge_index: torch.Tensor, num_nodes: int, edge_weight: Optional[torch.Tensor] = None,
                degree_on: str = "col", validate: bool = False) -> Graph:
    _dev_check(edge_index, edge_weight)
    dcode = degree_code(degree_on)
    ei = _check_ei(edge_index)
    ew = None if edge_weight is None else edge_weight.to(torch.float32).contiguous()
    E, N = int(ei.size(1)), int(num_nodes)
    dev = ei.device
    g = _alloc_graph(E, N, dev)
    L = _lib.lib()
    ws = workspace(L.bgcn_graph_workspace_size(E, N), dev)
    check(L.bgcn_build_graph(ptr(ei), ptr(ew), E, N, dcode,
                             *(g._ptrs[n] for n in ("t_ptr", "t_row", "t_col", "t_w",
                                                    "s_ptr", "s_row", "s_col", "s_w")),
                             ptr(g.status), ptr(ws), ws.numel(), stream_handle()))
    g._plan_ws = ws   # the build's workspace: D^-1/2 (bgcn_graph_dinv) for the edge-weight gradient
    if validate:
        g.check()
    return g


def _graph_dinv(g: Graph) -> int:
    """Device pointer of the D^-1/2 vector a single-graph build left in its workspace."""
    out = ctypes.c_void_p()
    ws = g._plan_ws
    check(_lib.lib().bgcn_graph_dinv(ws.data_ptr(), ws.numel(), g.num_edges, g.num_nodes, ctypes.byref(out)))
    return int(out.value)


def drop_edges(td_edge_index: Optional[torch.Tensor], bu_edge_index: Optional[torch.Tensor],
               batch: torch.Tensor, num_graphs: int, tddroprate: float = 0.0, budroprate: float = 0.0,
               seed: int = 0, masked: bool = False):
    """DropEdge of ``Process/dataset.py:68-90`` on the device, per tree of a collated batch:
    keep a uniform random subset of exactly ``int(E_t * (1 - rate))`` edges in their
    original order (``rate <= 0`` keeps all).  TD and BU are drawn independently from
    ``seed`` (a counter-based draw, not Python's ``random`` stream).

    ``masked=False`` returns the compacted lists (one host sync for the kept counts);
    ``masked=True`` returns ``[2, E]`` lists holding, per tree, the kept edges in order
    and then every dropped edge ``(s, d)`` as the self loop ``(d, d)``, which
    :func:`build_graph` removes (no sync)."""
    ref = td_edge_index if td_edge_index is not None else bu_edge_index
    if ref is None:
        raise ValueError("drop_edges: no edge list given")
    _dev_check(td_edge_index, bu_edge_index, batch)
    td = None if td_edge_index is None else _check_ei(td_edge_index)
    bu = None if bu_edge_index is None else _check_ei(bu_edge_index)
    batch = batch.to(torch.int64).contiguous()
    N, B = int(batch.numel()), int(num_graphs)
    dev = batch.device
    td_out = None if td is None else torch.empty_like(td)
    bu_out = None if bu is None else torch.empty_like(bu)
    counts = torch.zeros(2, dtype=torch.int64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    L = _lib.lib()
    ws = workspace(L.bgcn_drop_edges_workspace_size(B), dev)
    Etd = 0 if td is None else int(td.size(1))
    Ebu = 0 if bu is None else int(bu.size(1))
    check(L.bgcn_drop_edges(ptr(td), Etd, float(tddroprate), ptr(td_out), max(Etd, 1),
                            ptr(bu), Ebu, float(budroprate), ptr(bu_out), max(Ebu, 1), ptr(batch), N, B,
                            int(seed) & (2**64 - 1), int(masked), ptr(counts), ptr(status), ptr(ws),
                            ws.numel(), stream_handle()))
    if masked:
        return td_out, bu_out
    kept = counts.cpu()
    if int(status.item()) & 1:
        raise IndexError("drop_edges: an edge index is out of range or the edges are not "
                         "grouped by tree in batch order")
    if td_out is not None:
        td_out = td_out[:, :int(kept[0])].contiguous()
    if bu_out is not None:
        bu_out = bu_out[:, :int(kept[1])].contiguous()
    return td_out, bu_out


# ----------------------------------------------------------------------------- K3/K4
def spmm(g: Graph, x: torch.Tensor, bias: Optional[torch.Tensor] = None, relu: bool = False,
         transposed: bool = False, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``out = A_hat x (+bias)`` (or ``A_hat^T x``); x [N, F] with F % 4 == 0 (computed in
    fp32: other dtypes are converted)."""
    _dev_check(x, bias)
    if x.dim() != 2 or x.size(0) != g.num_nodes:
        raise ValueError(f"x must be [num_nodes={g.num_nodes}, F]")
    N, F = x.shape
    if x.dtype != torch.float32:
        x = x.float()
    if x.stride(1) != 1:
        x = x.contiguous()
    if bias is not None:
        bias = bias.to(torch.float32).contiguous()
        if bias.numel() != F:
            raise ValueError("bias must have F elements")
    if out is None:
        out = torch.empty(N, F, dtype=torch.float32, device=x.device)
    elif out.dtype != torch.float32 or out.shape != (N, F) or out.stride(1) != 1:
        raise ValueError("out must be a row-major fp32 [N, F] tensor")
    L = _lib.lib()
    ws = workspace(L.bgcn_spmm_workspace_size(g.capacity, F), x.device)
    p = [g._ptrs[("s_" if transposed else "t_") + n] for n in ("ptr", "row", "col", "w")]
    check(L.bgcn_spmm(p[0], p[1], p[2], p[3], N, g.capacity, ptr(x), x.stride(0),
                      ptr(out), out.stride(0), F, ptr(bias), 1 if relu else 0, ptr(ws), ws.numel(),
                      stream_handle()))
    return out


def _pad4(t: torch.Tensor) -> torch.Tensor:
    """Zero-pad the last dim to a multiple of 4 (spmm works on float4 rows)."""
    F = t.size(-1)
    if F % 4 == 0:
        return t.contiguous()
    return torch.nn.functional.pad(t, (0, 4 - F % 4)).contiguous()


def _linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """x [N, K] . w[O, K]^T on MFMA."""
    N, K = x.shape
    O = w.size(0)
    y = torch.empty(N, O, dtype=torch.float32, device=x.device)
    check(_lib.lib().bgcn_gemm_xwt(ptr(x), x.stride(0), ptr(w), 0, w.stride(0), O, ptr(y), O, N, O, K,
                                   stream_handle()))
    return y


class _GCNConvFn(torch.autograd.Function):
    """PyG-2.x GCNConv: out = A_hat (x W^T) + b, A_hat = gcn_norm(edge_index, edge_weight)."""

    @staticmethod
    def forward(ctx, x, weight, bias, g: Graph, edge_index=None, edge_weight=None, degree_on="col"):
        x = x.contiguous().float()
        weight = weight.contiguous()
        z = _pad4(_linear(x, weight))
        O = weight.size(0)
        b = None if bias is None else _pad4(bias.view(1, -1)).view(-1)
        out = spmm(g, z, b)[:, :O]
        ctx.g = g
        ctx.degree_on = degree_on
        ew_grad = edge_weight is not None and ctx.needs_input_grad[5]
        # the edge-weight gradient needs h = x W^T (padded) and the edge list
        ctx.save_for_backward(x, weight, z if ew_grad else None, edge_index if ew_grad else None)
        ctx.has_bias = bias is not None
        return out.contiguous()

    @staticmethod
    def backward(ctx, dout):
        x, weight, z, ei = ctx.saved_tensors
        g: Graph = ctx.g
        L = _lib.lib()
        N, K = x.shape
        O = weight.size(0)
        d = _pad4(dout.float())
        dzp = spmm(g, d, transposed=True)                       # A_hat^T dout (padded width)
        dz = dzp[:, :O].contiguous()
        dx = dw = db = dew = None
        if len(ctx.needs_input_grad) > 5 and ctx.needs_input_grad[5] and z is not None:
            # gcn_norm's backward (EBGCN.py:84,178 learn edge_weight): row dots of
            # (dout, A_hat h) and (h, A_hat^T dout), then one dot per edge
            agg = spmm(g, z)                                     # A_hat h, no bias
            E = int(ei.size(1))
            dew = torch.empty(E, dtype=torch.float32, device=x.device)
            ws = workspace(L.bgcn_edge_weight_grad_workspace_size(N), x.device)
            F4 = int(z.size(1))
            check(L.bgcn_edge_weight_grad(ptr(ei), E, N, degree_code(ctx.degree_on), _graph_dinv(g), ptr(z),
                                          ptr(agg), ptr(d), ptr(dzp), F4, F4, ptr(dew), ptr(ws), ws.numel(),
                                          stream_handle()))
        if ctx.needs_input_grad[0]:
            dx = torch.empty(N, K, dtype=torch.float32, device=x.device)
            check(L.bgcn_gemm_xw(ptr(dz), dz.stride(0), ptr(weight), weight.stride(0), ptr(dx), K,
                                 N, K, O, stream_handle()))
        if ctx.needs_input_grad[1]:
            dw = torch.empty(O, K, dtype=torch.float32, device=x.device)
            ws = workspace(L.bgcn_gemm_tn_workspace_size(O, K, N), x.device)
            check(L.bgcn_gemm_tn(ptr(dz), dz.stride(0), ptr(x), x.stride(0), ptr(dw), 0, K, O, O, K,
                                 N, ptr(ws), ws.numel(), stream_handle()))
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = torch.empty(O, dtype=torch.float32, device=x.device)
            dd = dout.float().contiguous()
            ws = workspace(L.bgcn_colsum_workspace_size(N, O), x.device)
            check(L.bgcn_colsum(ptr(dd), dd.stride(0), N, O, ptr(db), ptr(ws), ws.numel(),
                                stream_handle()))
        return (dx, dw, db, None, None, dew, None)[:len(ctx.needs_input_grad)]


def gcn_conv(x: torch.Tensor, edge_index_or_graph, weight: torch.Tensor,
             bias: Optional[torch.Tensor] = None, edge_weight: Optional[torch.Tensor] = None,
             degree_on: str = "col") -> torch.Tensor:
    _dev_check(x, weight, bias, edge_weight)
    g = edge_index_or_graph
    if edge_weight is not None and edge_weight.requires_grad and torch.is_grad_enabled():
        # EBGCN (EBGCN.py:101-102 -> :84,178) learns its edge weights: gcn_norm's backward
        if isinstance(g, Graph):
            raise ValueError("gcn_conv: a learned edge_weight needs edge_index (the graph is built from it)")
        ei = _check_ei(g)
        if edge_weight.dim() != 1 or edge_weight.numel() != ei.size(1):
            raise ValueError("edge_weight must be [E]")
        g = build_graph(ei, x.size(0), edge_weight.detach(), degree_on)
        return _GCNConvFn.apply(x, weight, bias, g, ei, edge_weight, degree_on)
    if not isinstance(g, Graph):
        g = build_graph(g, x.size(0), edge_weight, degree_on)
    return _GCNConvFn.apply(x, weight, bias, g)


# ----------------------------------------------------------------------------- K8
class _ScatterMeanFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, src, index, B):
        src = src.contiguous().float()
        n, C = src.shape
        out = torch.empty(B, C, dtype=torch.float32, device=src.device)
        cnt = torch.empty(B, dtype=torch.float32, device=src.device)
        status = torch.zeros(1, dtype=torch.int32, device=src.device)
        L = _lib.lib()
        ws = workspace(L.bgcn_scatter_mean_workspace_size(B), src.device)
        check(L.bgcn_scatter_mean_fwd(ptr(src), src.stride(0), ptr(index), n, C, B, ptr(out), C,
                                      ptr(cnt), ptr(status), ptr(ws), ws.numel(), stream_handle()))
        ctx.save_for_backward(index, cnt)
        ctx.shape = (n, C, B)
        return out

    @staticmethod
    def backward(ctx, dout):
        index, cnt = ctx.saved_tensors
        n, C, B = ctx.shape
        dout = dout.contiguous().float()
        dsrc = torch.empty(n, C, dtype=torch.float32, device=dout.device)
        check(_lib.lib().bgcn_scatter_mean_bwd(ptr(dout), dout.stride(0), ptr(index), ptr(cnt), n, C, B,
                                               ptr(dsrc), C, stream_handle()))
        return dsrc, None, None


def scatter_mean(src: torch.Tensor, index: torch.Tensor, dim: int = 0, out=None,
                 dim_size: Optional[int] = None) -> torch.Tensor:
    """``torch_scatter.scatter_mean(src, index, dim=0)`` on the GPU.  Like torch_scatter,
    ``dim_size=None`` means ``index.max() + 1`` (a host sync, as in the reference)."""
    if dim not in (0, -src.dim()):
        raise NotImplementedError("scatter_mean: only dim=0 is on the BiGCN path")
    _dev_check(src, index)
    index = index.to(torch.int64).contiguous()
    if dim_size is None:
        dim_size = int(index.max().item()) + 1 if index.numel() else 0
    if dim_size == 0:
        return src.new_zeros((0,) + tuple(src.shape[1:]))
    shp = src.shape
    res = _ScatterMeanFn.apply(src.reshape(shp[0], -1), index, int(dim_size))
    res = res.view((int(dim_size),) + tuple(shp[1:]))
    if out is not None:
        out.copy_(res)
        return out
    return res


# ----------------------------------------------------------------------------- fused encoder
_PARAM_ORDER = ("td_w1", "td_b1", "td_w2", "td_b2", "bu_w1", "bu_b1", "bu_w2", "bu_b2")


_FEAT_MODES = {"auto": _lib.BGCN_FEAT_AUTO, "sparse": _lib.BGCN_FEAT_AUTO, "dense": _lib.BGCN_FEAT_DENSE}


def feat_path(feat_mode: str, data) -> int:
    """C-ABI feature path for a batch: "auto" becomes BGCN_FEAT_SPARSE (no dense fallback
    launched) when the batch's host-side hints say its rows fit the sparse path - every row
    within the ELL cap, or the entries past it within the spill pool (``collate`` /
    ``synth_batch`` set them, bound to x's identity and version); "sparse" forces it (in
    the fused step a batch that does not fit -> check_status raises)."""
    if feat_mode == "sparse":
        return _lib.BGCN_FEAT_SPARSE
    if feat_mode == "auto" and int(data.x.size(1)) <= 5120:
        hint = data.x_nnz_hint() if hasattr(data, "x_nnz_hint") else None
        if hint is not None and int(hint) <= _lib.BGCN_SPARSE_CAP:
            return _lib.BGCN_FEAT_SPARSE
        spill = data.x_spill_hint() if hasattr(data, "x_spill_hint") else None
        if spill is not None and int(spill) <= int(data.x.size(0)) * _lib.BGCN_SPARSE_SPILL_PER_ROW:
            return _lib.BGCN_FEAT_SPARSE
    return _FEAT_MODES[feat_mode]


def _feat_code(feat_mode) -> int:
    return feat_mode if isinstance(feat_mode, int) else _FEAT_MODES[feat_mode]


def check_encoder_shapes(x: torch.Tensor, batch: torch.Tensor, rootindex: torch.Tensor, params) -> None:
    """Host-side shape contract of the fused encoder (the kernels trust it)."""
    if x.dim() != 2:
        raise ValueError("x must be [N, F]")
    N, F = x.shape
    want = [(HID, F), (HID,), (HID, HID + F), (HID,)] * 2
    for p, shp in zip(params, want):
        if tuple(p.shape) != shp:
            raise ValueError(f"parameter of shape {tuple(p.shape)}, expected {shp} for in_feats={F}")
    if batch.numel() != N:
        raise ValueError("batch must have one entry per node")
    if rootindex.dim() != 1:
        raise ValueError("rootindex must be 1-D")


def features(x: torch.Tensor) -> torch.Tensor:
    """Node features as the fused path reads them: bf16 stays bf16 (the bf16
    configuration: bag-of-words counts are exact), anything else becomes fp32;
    contiguous rows."""
    if x.dtype != torch.bfloat16 and x.dtype != torch.float32:
        x = x.float()
    return x.contiguous()


def x_dtype_code(x: torch.Tensor) -> int:
    return _lib.BGCN_DTYPE_BF16 if x.dtype == torch.bfloat16 else _lib.BGCN_DTYPE_F32


_GRAD_ORDER = tuple(n.replace("_w", "_dw").replace("_b", "_db") for n in _PARAM_ORDER)


def _fill_args(a: BiGCNArgs, x, batch, rootindex, td, bu, B, training, seed, keep, feat_mode, xs, params):
    N, F = x.shape
    a.x, a.ldx, a.num_nodes, a.num_graphs, a.in_feats, a.hid = x.data_ptr(), x.stride(0), N, B, F, HID
    a.x_dtype = x_dtype_code(x)
    a.batch, a.rootindex = batch.data_ptr(), rootindex.data_ptr()
    a.td, a.bu = td.view(), bu.view()
    a.td_w1, a.td_b1, a.td_w2, a.td_b2, a.bu_w1, a.bu_b1, a.bu_w2, a.bu_b2 = (p.data_ptr() for p in params)
    a.training, a.seed = int(bool(training)), int(seed) & (2**64 - 1)
    a.keep_words = ptr(keep)
    a.feat_mode = feat_mode
    if xs is not None:
        a.x_flags, a.x_nnz, a.x_cols, a.x_vals = (t.data_ptr() for t in xs)


def _encoder_forward(ctx, x, batch, rootindex, td: Graph, bu: Graph, B, training, seed, keep_words,
                     feat_mode, params, stream, prep=None):
    """The encoder's native forward; returns (head [B, 256], tensors for backward) and
    keeps the rest of the forward -> backward state on ``ctx`` (``_encoder_backward``).
    ``prep`` (a ``PreparedBatch`` of this batch, ``td`` / ``bu`` then None): the graphs,
    tree pointers, items and ELL / CSC of X come from it (bgcn_bigcn_args.prepared)."""
    x = features(x)
    N, F = x.shape
    dev = x.device
    L = _lib.lib()
    if prep is not None:
        return _encoder_forward_prepared(ctx, x, batch, rootindex, B, training, seed, keep_words, feat_mode,
                                         params, stream, prep)
    xs = None
    if feat_mode != _lib.BGCN_FEAT_DENSE:
        cap = _lib.BGCN_SPARSE_CAP
        xs = (torch.empty(8, dtype=torch.int32, device=dev), torch.empty(N, dtype=torch.int32, device=dev),
              torch.empty(N * cap, dtype=torch.int32, device=dev),
              torch.empty(N * cap, dtype=torch.float32, device=dev))
    a = BiGCNArgs()
    _fill_args(a, x, batch, rootindex, td, bu, B, training, seed, keep_words, feat_mode, xs, params)
    tree_ptr = torch.empty(B + 1, dtype=torch.int32, device=dev)
    h1 = torch.empty(N, 2 * HID, dtype=torch.float32, device=dev)
    h2 = torch.empty(N, 2 * HID, dtype=torch.float32, device=dev)
    head = torch.empty(B, 4 * HID, dtype=torch.float32, device=dev)
    a.tree_ptr, a.h1, a.h2, a.head_in = tree_ptr.data_ptr(), h1.data_ptr(), h2.data_ptr(), head.data_ptr()
    a.save_for_backward = 1 if any(ctx.needs_input_grad) else 0
    ws = workspace(L.bgcn_bigcn_workspace_size(N, B, F, HID), dev)
    check(L.bgcn_bigcn_forward(ctypes.byref(a), ws.data_ptr(), ws.numel(), stream))
    ctx.ws = ws if a.save_for_backward else None   # forward -> backward state (bgcn.h)
    ctx.args = a                                   # the backward reuses the filled struct
    ctx.graphs = (td, bu)
    ctx.meta = (B, N, params[0].device)
    ctx.has_keep = keep_words is not None
    empty = x.new_empty(0)
    # saved for autograd's version checks and lifetime (the struct holds their pointers)
    saved = (x, batch, rootindex, keep_words if keep_words is not None else empty, tree_ptr, h1, h2,
             *(xs if xs is not None else (empty,) * 4), *params)
    return head, saved


_ENC_SAVED = 11   # tensors of _encoder_forward's `saved` before the parameters


def _encoder_forward_prepared(ctx, x, batch, rootindex, B, training, seed, keep_words, feat_mode, params,
                              stream, prep):
    N, F = x.shape
    dev = x.device
    prep.check_matches(x, batch, rootindex, B, feat_mode)
    L = _lib.lib()
    a = BiGCNArgs()
    a.x, a.ldx, a.num_nodes, a.num_graphs, a.in_feats, a.hid = x.data_ptr(), x.stride(0), N, B, F, HID
    a.x_dtype = x_dtype_code(x)
    a.batch, a.rootindex = batch.data_ptr(), rootindex.data_ptr()
    a.td_w1, a.td_b1, a.td_w2, a.td_b2, a.bu_w1, a.bu_b1, a.bu_w2, a.bu_b2 = (p.data_ptr() for p in params)
    a.training, a.seed = int(bool(training)), int(seed) & (2**64 - 1)
    a.keep_words = ptr(keep_words)
    a.feat_mode = feat_mode
    a.prepared, a.prepared_bytes = prep.buf.data_ptr(), prep.buf.numel()
    a.td_num_edges, a.bu_num_edges = prep.td_num_edges, prep.bu_num_edges
    h1 = torch.empty(N, 2 * HID, dtype=torch.float32, device=dev)
    h2 = torch.empty(N, 2 * HID, dtype=torch.float32, device=dev)
    head = torch.empty(B, 4 * HID, dtype=torch.float32, device=dev)
    a.h1, a.h2, a.head_in = h1.data_ptr(), h2.data_ptr(), head.data_ptr()
    a.save_for_backward = 1 if any(ctx.needs_input_grad) else 0
    prep.wait()                                    # its preparation ordered before this forward
    ws = workspace(L.bgcn_bigcn_workspace_size(N, B, F, HID), dev)
    check(L.bgcn_bigcn_forward(ctypes.byref(a), ws.data_ptr(), ws.numel(), stream))
    ctx.ws = ws if a.save_for_backward else None
    ctx.args = a
    ctx.graphs = (prep,)                           # the prepared buffer lives until the backward
    ctx.meta = (B, N, params[0].device)
    ctx.has_keep = keep_words is not None
    empty = x.new_empty(0)
    saved = (x, batch, rootindex, keep_words if keep_words is not None else empty, empty, h1, h2,
             empty, empty, empty, empty, *params)
    return head, saved


class PreparedBatch:
    """A batch's weight-independent state built ahead of its forward (``prepare_batch``:
    K1 gcn_norm + CSR of both directions with their aggregation plans, tree pointers and
    work items, the ELL / spill pool / CSC of X - bgcn_prepare_batch) in a caller-side
    buffer, plus the event that ends its preparation.  The drop-in model's forward takes it
    from ``data._bgcn_prep`` (``prepare_ahead`` attaches it) and then runs no K1 and no pass
    over X of its own (bgcn_bigcn_args.prepared)."""

    def __init__(self, buf, N, B, F, td_edges, bu_edges, degree_on, dense, key, keep, event):
        self.buf, self.num_nodes, self.num_graphs, self.in_feats = buf, N, B, F
        self.td_num_edges, self.bu_num_edges = td_edges, bu_edges
        self.degree_on, self.dense, self.key, self._keep, self.event = degree_on, dense, key, keep, event
        self._waited = False
        # (slot, generation) when the buffer is one of a pipeline's reused slots
        # (prepare_ahead): the slot's counter moves on when a later batch is prepared into
        # it, and this preparation then no longer matches
        self._slot = None

    def current(self) -> bool:
        """Whether the buffer still holds this preparation (a reused slot may have taken a
        later batch since)."""
        return self._slot is None or self._slot[0][0] == self._slot[1]

    def matches(self, data, degree_on: str, feat_mode: int) -> bool:
        """Whether this preparation is of ``data`` as it is now (same tensors, unmodified,
        its buffer not reused) for that degree convention and feature path."""
        return (self.current() and self.degree_on == degree_on
                and self.dense == (feat_mode == _lib.BGCN_FEAT_DENSE) and self.key == _prep_key(data))

    def check_matches(self, x, batch, rootindex, B, feat_mode) -> None:
        if (x.size(0), B, x.size(1)) != (self.num_nodes, self.num_graphs, self.in_feats) or \
                self.dense != (feat_mode == _lib.BGCN_FEAT_DENSE):
            raise ValueError("prepared batch does not match the forward's inputs")

    def wait(self) -> None:
        """The current stream waits for the preparation (once) and is recorded as a user of
        the buffer (it may have been allocated on the preparing stream)."""
        if not self._waited:
            s = torch.cuda.current_stream(self.buf.device)
            if self.event is not None:
                s.wait_event(self.event)
            self.buf.record_stream(s)
        self._waited = True


def _prep_key(data):
    x = data.x
    return (x.data_ptr(), x._version, tuple(x.shape), data.edge_index.data_ptr(), data.edge_index._version,
            int(data.edge_index.size(1)), data.BU_edge_index.data_ptr(), data.BU_edge_index._version,
            int(data.BU_edge_index.size(1)), data.batch.data_ptr(), data.batch._version,
            data.rootindex.data_ptr(), data.rootindex._version)


def prepare_batch(data, degree_on: str = "col", feat_mode: str = "auto", buf: Optional[torch.Tensor] = None,
                  stream: Optional[torch.cuda.Stream] = None) -> PreparedBatch:
    """bgcn_prepare_batch of a collated device batch (its edge lists as they are: the
    reference's DropEdge happened in the dataset) on ``stream`` (default: the current
    one), into ``buf`` when it is large enough.  The returned object's event marks the end
    of the preparation; the batch's tensors must be ready on ``stream`` when it runs."""
    from ._lib import BatchDesc
    x = features(data.x)
    td_ei, bu_ei = _check_ei(data.edge_index), _check_ei(data.BU_edge_index)
    batch = data.batch if data.batch.dtype == torch.int64 and data.batch.is_contiguous() else \
        data.batch.to(torch.int64).contiguous()
    root = data.rootindex if data.rootindex.dtype == torch.int64 and data.rootindex.is_contiguous() else \
        data.rootindex.to(torch.int64).contiguous()
    _dev_check(x, td_ei, bu_ei, batch, root)
    N, F = x.shape
    B = int(root.numel())
    code = _feat_code(feat_path(feat_mode, data) if isinstance(feat_mode, str) else feat_mode)
    d = BatchDesc()
    d.x, d.ldx, d.num_nodes, d.num_graphs = ptr(x), x.stride(0), N, B
    d.x_dtype = x_dtype_code(x)
    d.batch, d.rootindex = ptr(batch), ptr(root)
    d.td_edge_index, d.td_num_edges = ptr(td_ei), td_ei.size(1)
    d.bu_edge_index, d.bu_num_edges = ptr(bu_ei), bu_ei.size(1)
    L = _lib.lib()
    n = L.bgcn_prepare_workspace_size(N, B, F, d.td_num_edges, d.bu_num_edges)
    if buf is None or buf.numel() < n:
        buf = workspace(n, x.device)
    s = stream if stream is not None else torch.cuda.current_stream(x.device)
    check(L.bgcn_prepare_batch(ctypes.byref(d), F, degree_code(degree_on), code, buf.data_ptr(), buf.numel(),
                               s.cuda_stream))
    ev = torch.cuda.Event()
    ev.record(s)
    return PreparedBatch(buf, N, B, F, int(d.td_num_edges), int(d.bu_num_edges), degree_on,
                         code == _lib.BGCN_FEAT_DENSE, _prep_key(data), (x, td_ei, bu_ei, batch, root), ev)


def _encoder_backward(ctx, saved, dhead, stream):
    """Gradients of the 8 encoder parameters (reference order) from dhead [B, 256]."""
    params = saved[_ENC_SAVED:_ENC_SAVED + 8]
    L = _lib.lib()
    a = ctx.args
    a.dhead_in = dhead.data_ptr()
    grads = [torch.empty_like(p) for p in params]
    for name, gt in zip(_GRAD_ORDER, grads):
        setattr(a, name, gt.data_ptr())
    ws = ctx.ws
    ctx.ws = None
    if ws is None:
        raise RuntimeError("bigcn_encoder: backward called twice or without a saved forward")
    for g in ctx.graphs:
        if isinstance(g, PreparedBatch) and not g.current():
            raise RuntimeError("bigcn_encoder: the forward's prepared batch buffer was reused by a later "
                               "batch (prepare_ahead) before this backward")
    check(L.bgcn_bigcn_backward(ctypes.byref(a), ws.data_ptr(), ws.numel(), stream))
    return grads


class _BiGCNEncoderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, batch, rootindex, td: Graph, bu: Graph, B, training, seed, keep_words,
                feat_mode, prep, *params):
        head, saved = _encoder_forward(ctx, x, batch, rootindex, td, bu, B, training, seed, keep_words,
                                       feat_mode, params, stream_handle(), prep)
        ctx.save_for_backward(*saved)
        return head

    @staticmethod
    def backward(ctx, dhead):
        saved = ctx.saved_tensors
        dhead = dhead.contiguous().float()
        return (None,) * 11 + tuple(_encoder_backward(ctx, saved, dhead, stream_handle()))


class _BiGCNNetFn(torch.autograd.Function):
    """encoder -> fc -> log_softmax (``BiGCN.forward``, BiGCN_Twitter.py:126-130) as one
    autograd node: the encoder's native forward / backward plus the K9 head
    (``bgcn_head_forward`` / ``bgcn_head_backward``) - no library GEMM, log_softmax or
    their backward kernels, and one node for the autograd engine to run."""

    @staticmethod
    def forward(ctx, x, batch, rootindex, td: Graph, bu: Graph, B, training, seed, keep_words,
                feat_mode, prep, fc_w, fc_b, *params):
        s = stream_handle()
        head, saved = _encoder_forward(ctx, x, batch, rootindex, td, bu, B, training, seed, keep_words,
                                       feat_mode, params, s, prep)
        C = fc_w.size(0)
        logp = torch.empty(B, C, dtype=torch.float32, device=head.device)
        check(_lib.lib().bgcn_head_forward(head.data_ptr(), fc_w.data_ptr(), fc_b.data_ptr(), B, C,
                                           logp.data_ptr(), s))
        ctx.save_for_backward(*saved, head, logp, fc_w, fc_b)
        return logp

    @staticmethod
    def backward(ctx, dlogp):
        saved = ctx.saved_tensors
        head, logp, fc_w, fc_b = saved[-4:]
        dlogp = dlogp.contiguous().float()
        B, C = logp.shape
        s = stream_handle()
        dhead = torch.empty_like(head)
        dfc_w, dfc_b = torch.empty_like(fc_w), torch.empty_like(fc_b)
        check(_lib.lib().bgcn_head_backward(head.data_ptr(), logp.data_ptr(), dlogp.data_ptr(), fc_w.data_ptr(),
                                            B, C, dhead.data_ptr(), dfc_w.data_ptr(), dfc_b.data_ptr(), s))
        grads = _encoder_backward(ctx, saved, dhead, s)
        return (None,) * 11 + (dfc_w, dfc_b) + tuple(grads)


def _encoder_inputs(x, batch, rootindex, params, keep_words):
    _dev_check(x, batch, rootindex, keep_words, *params)
    for p in params:
        if p.dtype != torch.float32 or not p.is_contiguous():
            raise ValueError("parameters must be contiguous fp32")
    check_encoder_shapes(x, batch, rootindex, params)
    if batch.dtype != torch.int64 or not batch.is_contiguous():
        batch = batch.to(torch.int64).contiguous()
    if rootindex.dtype != torch.int64 or not rootindex.is_contiguous():
        rootindex = rootindex.to(torch.int64).contiguous()
    return batch, rootindex, (keep_words.contiguous() if keep_words is not None else None)


def bigcn_encoder(x: torch.Tensor, batch: torch.Tensor, rootindex: torch.Tensor, td: Graph, bu: Graph,
                  num_graphs: int, params, training: bool = False, seed: int = 0,
                  keep_words: Optional[torch.Tensor] = None, feat_mode: str = "auto",
                  prep: Optional["PreparedBatch"] = None) -> torch.Tensor:
    """cat(BU_x, TD_x) [B, 256] of ``BiGCN.forward`` (``BiGCN_Twitter.py:126-128``).

    ``params`` = (td_w1, td_b1, td_w2, td_b2, bu_w1, bu_b1, bu_w2, bu_b2) in the
    reference layout (``convN.lin.weight [out, in]``, ``convN.bias``).  ``keep_words``
    optionally injects the dropout draw as packed bits [2, N, ceil((64+F)/32)] int32.
    ``feat_mode``: "auto" (sparse feature path, dense MFMA fallback decided on the
    device), "dense" (always the dense MFMA kernels) or a C-ABI code (``feat_path``:
    BGCN_FEAT_SPARSE when the batch's hints say its rows fit)."""
    batch, rootindex, keep_words = _encoder_inputs(x, batch, rootindex, params, keep_words)
    return _BiGCNEncoderFn.apply(x, batch, rootindex, td, bu, int(num_graphs), bool(training), int(seed),
                                 keep_words, _feat_code(feat_mode), prep, *params)


def head_fits(fc: torch.nn.Module) -> bool:
    """Whether ``fc`` is a head the K9 kernels take in place of ``fc(...)``: exactly a
    ``torch.nn.Linear(256, C <= 16)`` (not a subclass with its own forward) with a bias,
    no forward hooks (their side effects would be skipped), contiguous fp32 weights on
    16-byte boundaries (``bgcn_head_forward``'s alignment contract).  Anything else runs
    through ``fc`` itself and torch's log_softmax."""
    w, b = getattr(fc, "weight", None), getattr(fc, "bias", None)
    return (type(fc) is torch.nn.Linear and w is not None and b is not None and w.dim() == 2
            and not fc._forward_hooks and not fc._forward_pre_hooks
            and not torch.nn.modules.module._global_forward_hooks
            and not torch.nn.modules.module._global_forward_pre_hooks
            and w.size(1) == 4 * HID and 0 < w.size(0) <= 16 and w.dtype == torch.float32
            and b.dtype == torch.float32 and w.is_contiguous() and b.is_contiguous()
            and w.data_ptr() % 16 == 0 and b.data_ptr() % 4 == 0)


def bigcn_net(x: torch.Tensor, batch: torch.Tensor, rootindex: torch.Tensor, td: Graph, bu: Graph,
              num_graphs: int, params, fc_w: torch.Tensor, fc_b: torch.Tensor, training: bool = False,
              seed: int = 0, keep_words: Optional[torch.Tensor] = None, feat_mode: str = "auto",
              prep: Optional["PreparedBatch"] = None) -> torch.Tensor:
    """``log_softmax(fc(bigcn_encoder(...)), dim=1)`` [B, C] (``BiGCN_Twitter.py:126-130``)
    as one autograd node: the encoder plus the K9 head kernels.  ``fc_w`` [C, 256] and
    ``fc_b`` [C] are the ``fc`` Linear's parameters (C <= 16)."""
    batch, rootindex, keep_words = _encoder_inputs(x, batch, rootindex, params, keep_words)
    _dev_check(fc_w, fc_b)
    if (fc_w.dim() != 2 or fc_w.size(1) != 4 * HID or not 0 < fc_w.size(0) <= 16 or fc_b.shape != (fc_w.size(0),)
            or fc_w.dtype != torch.float32 or fc_b.dtype != torch.float32
            or not fc_w.is_contiguous() or not fc_b.is_contiguous()):
        raise ValueError("fc must be a contiguous fp32 Linear(256, C <= 16) with a bias")
    return _BiGCNNetFn.apply(x, batch, rootindex, td, bu, int(num_graphs), bool(training), int(seed), keep_words,
                             _feat_code(feat_mode), prep, fc_w, fc_b, *params)


def keep_words(seed: int, num_nodes: int, in_feats: int, device) -> torch.Tensor:
    """Materialise the in-kernel dropout keep bits [2, N, nw] (int32 view of uint32)."""
    nw = (HID + in_feats + 31) // 32
    w = torch.empty(2, num_nodes, nw, dtype=torch.int32, device=device)
    check(_lib.lib().bgcn_keep_words(int(seed) & (2**64 - 1), num_nodes, nw, ptr(w), stream_handle()))
    return w


def unpack_keep(words: torch.Tensor, width: int) -> torch.Tensor:
    """[..., nw] packed keep words -> [..., width] bool (bit j of word w = column 32w+j)."""
    w = words.to(torch.int64) & 0xFFFFFFFF
    bits = torch.arange(32, device=w.device, dtype=torch.int64)
    m = ((w.unsqueeze(-1) >> bits) & 1).bool()
    return m.reshape(*words.shape[:-1], -1)[..., :width]


def pack_keep(mask: torch.Tensor) -> torch.Tensor:
    """[..., width] bool -> [..., ceil(width/32)] int32 words."""
    width = mask.size(-1)
    nw = (width + 31) // 32
    pad = nw * 32 - width
    m = torch.nn.functional.pad(mask.to(torch.int64), (0, pad)).reshape(*mask.shape[:-1], nw, 32)
    w = (m << torch.arange(32, dtype=torch.int64, device=mask.device)).sum(-1)
    w = torch.where(w >= 2**31, w - 2**32, w)
    return w.to(torch.int32)


def set_kernel_timing(enable, classes=None) -> None:
    """Enable (all classes, or the iterable ``classes``) / disable the kernel-timing hook."""
    mask = 0
    if enable:
        mask = 0xFF if classes is None else sum(1 << int(c) for c in classes)
    check(_lib.lib().bgcn_set_kernel_timing(mask))


def kernel_timing(kernel_class: int):
    """(total_ms, launches) of a kernel class since set_kernel_timing(True) (syncs)."""
    ms = ctypes.c_float(0.0)
    n = ctypes.c_int64(0)
    check(_lib.lib().bgcn_kernel_timing(kernel_class, ctypes.byref(ms), ctypes.byref(n)))
    return float(ms.value), int(n.value)


def kernel_span(kernel_class: int):
    """(total_ms, launches) of a stamped kernel class's device-side spans since
    set_kernel_timing(True) (the kernel's own first-block-start to last-block-end; syncs)."""
    ms = ctypes.c_float(0.0)
    n = ctypes.c_int64(0)
    check(_lib.lib().bgcn_kernel_span(kernel_class, ctypes.byref(ms), ctypes.byref(n)))
    return float(ms.value), int(n.value)
