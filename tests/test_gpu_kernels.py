"""GPU parity tests of the individual HIP kernels (K1-K4, K8, K10) through the C ABI.

Each kernel is compared against the CPU oracle / a float64 torch restatement on the
same seeded inputs.  Tolerance (fp32 path vs fp64 reference): |a - b| <= 1e-4 * (|b| + s)
with s the reference's scale, i.e. the north-star "within 1e-4 fp32"; integer/index
outputs are compared exactly.
"""
import math

import numpy as np
import pytest
import torch

from oracle import bigcn_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-4


def close(a, b, tol=TOL, what=""):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    assert a.shape == b.shape, (what, a.shape, b.shape)
    scale = float(b.abs().max()) if b.numel() else 1.0
    err = float((a - b).abs().max()) if b.numel() else 0.0
    assert err <= tol * max(scale, 1e-30) + 1e-30, f"{what}: max err {err:.3e} vs scale {scale:.3e}"


def rand_forest(rng, sizes, star=False):
    rows, cols, off = [], [], 0
    for n in sizes:
        for k in range(1, n):
            p = 0 if (star or k == 1 or rng.random() < 0.5) else int(rng.integers(1, k))
            rows.append(off + p)
            cols.append(off + k)
        off += n
    return torch.tensor([rows, cols], dtype=torch.int64), off


def dense_adj(ptr, row, col, w, N):
    """Dense matrix A[row, col] = w from a CSR (row-major by `row`)."""
    nnz = int(ptr[N])
    A = torch.zeros(N, N, dtype=torch.float64)
    A.index_put_((row[:nnz].long(), col[:nnz].long()), w[:nnz].double(), accumulate=True)
    return A


@pytest.mark.parametrize("degree_on", ["col", "row"])
@pytest.mark.parametrize("star", [False, True])
def test_build_graph_matches_gcn_norm(degree_on, star):
    from bigcn_amd.ops import build_graph
    rng = np.random.default_rng(1)
    ei, N = rand_forest(rng, [1, 2, 7, 40, 300], star=star)
    g = build_graph(ei.to(DEV), N, degree_on=degree_on, validate=True)
    e, w = O.gcn_norm(ei, None, N, degree_on, dtype=torch.float64)
    ref = torch.zeros(N, N, dtype=torch.float64)
    ref.index_put_((e[1], e[0]), w, accumulate=True)      # target-major: A[dst, src]
    t = [x.cpu() for x in (g.t_ptr, g.t_row, g.t_col, g.t_w)]
    s = [x.cpu() for x in (g.s_ptr, g.s_row, g.s_col, g.s_w)]
    close(dense_adj(*t, N), ref, 1e-6, "t-csr")
    close(dense_adj(*s, N), ref.t(), 1e-6, "s-csr")
    # row structure: self loop last, real entries keep edge order
    tp = t[0]
    assert int(tp[N]) == ei.size(1) + N
    for i in range(0, N, 37):
        a, b = int(tp[i]), int(tp[i + 1])
        assert int(t[2][b - 1]) == i and bool((t[1][a:b] == i).all())


@pytest.mark.parametrize("shuffle", [False, True])
def test_build_graph_pair_matches_single(shuffle):
    """Paired TD/BU build == two single builds, bit for bit; grouped (tree order) and
    general (shuffled edge order) placement both restore edge order in every row."""
    from bigcn_amd.ops import build_graph, build_graph_pair
    rng = np.random.default_rng(7)
    ei, N = rand_forest(rng, [3, 50, 1, 600, 9], star=False)
    order = np.lexsort((ei[1].numpy(), ei[0].numpy()))           # reference order (parent, child)
    td = ei[:, torch.as_tensor(order)]
    if shuffle:
        td = td[:, torch.as_tensor(rng.permutation(td.size(1)))]
    bu = td.flip(0)
    a, b = build_graph_pair(td.to(DEV), bu.to(DEV), N, validate=True)
    for g, e in ((a, td), (b, bu)):
        s = build_graph(e.to(DEV), N)
        for k in ("t_ptr", "t_row", "t_col", "t_w", "s_ptr", "s_row", "s_col", "s_w"):
            n = int(s.t_ptr[N])
            assert torch.equal(getattr(g, k)[:n + 1] if "ptr" in k else getattr(g, k)[:n],
                               getattr(s, k)[:n + 1] if "ptr" in k else getattr(s, k)[:n]), k
        # rows keep edge order: the sources of target row i appear as in `e`
        tp, tc = s.t_ptr.cpu(), s.t_col.cpu()
        for i in range(0, N, 53):
            want = e[0][e[1] == i].tolist() + [i]
            assert tc[int(tp[i]):int(tp[i + 1])].tolist() == want


def test_build_graph_drops_input_self_loops_and_flags_bad_index():
    from bigcn_amd.ops import build_graph
    ei = torch.tensor([[0, 1, 1, 2], [1, 1, 2, 0]])
    g = build_graph(ei.to(DEV), 3)
    e, w = O.gcn_norm(ei, None, 3, "col", dtype=torch.float64)
    ref = torch.zeros(3, 3, dtype=torch.float64)
    ref.index_put_((e[1], e[0]), w, accumulate=True)
    close(dense_adj(*[x.cpu() for x in (g.t_ptr, g.t_row, g.t_col, g.t_w)], 3), ref, 1e-6)
    bad = torch.tensor([[0, 5], [1, 0]])
    with pytest.raises(IndexError):
        build_graph(bad.to(DEV), 3, validate=True)


@pytest.mark.parametrize("case", ["inside_src_run", "inside_dst_run", "between_runs", "tail"])
def test_build_graph_self_loops_inside_runs(case):
    """Input self loops placed inside a node's run of edges (which would shift run-based
    ranks), between runs, and at a tree's tail (the masked DropEdge layout)."""
    from bigcn_amd.ops import build_graph
    ei = {"inside_src_run": [[0, 0, 0, 1, 1], [1, 0, 2, 3, 4]],
          "inside_dst_run": [[1, 2, 2, 3, 0], [2, 2, 2, 2, 1]],
          "between_runs": [[0, 0, 3, 1, 1], [1, 2, 3, 3, 4]],
          "tail": [[0, 0, 1, 2, 4], [1, 2, 3, 2, 4]]}[case]
    ei = torch.tensor(ei)
    for degree_on in ("col", "row"):
        g = build_graph(ei.to(DEV), 5, degree_on=degree_on)
        e, w = O.gcn_norm(ei, None, 5, degree_on, dtype=torch.float64)
        ref = torch.zeros(5, 5, dtype=torch.float64)
        ref.index_put_((e[1], e[0]), w, accumulate=True)
        close(dense_adj(*[x.cpu() for x in (g.t_ptr, g.t_row, g.t_col, g.t_w)], 5), ref, 1e-6)
        # the transposed orientation holds the same entries
        refT = ref.t().contiguous()
        close(dense_adj(*[x.cpu() for x in (g.s_ptr, g.s_row, g.s_col, g.s_w)], 5), refT, 1e-6)
        # and every row keeps edge order, its self loop last (the reference's summation order)
        kept = [(int(a), int(b)) for a, b in ei.t() if a != b]
        for ptr_, col_, key, other in ((g.t_ptr.cpu(), g.t_col.cpu(), 1, 0), (g.s_ptr.cpu(), g.s_col.cpu(), 0, 1)):
            for i in range(5):
                want = [ed[other] for ed in kept if ed[key] == i] + [i]
                assert col_[int(ptr_[i]):int(ptr_[i + 1])].tolist() == want, (case, i)


def test_build_graph_edge_weight():
    from bigcn_amd.ops import build_graph
    rng = np.random.default_rng(3)
    ei, N = rand_forest(rng, [9, 20])
    ew = torch.rand(ei.size(1), dtype=torch.float64) + 0.1
    g = build_graph(ei.to(DEV), N, ew.float().to(DEV))
    e, w = O.gcn_norm(ei, ew, N, "col", dtype=torch.float64)
    ref = torch.zeros(N, N, dtype=torch.float64)
    ref.index_put_((e[1], e[0]), w, accumulate=True)
    close(dense_adj(*[x.cpu() for x in (g.t_ptr, g.t_row, g.t_col, g.t_w)], N), ref, 1e-6)


@pytest.mark.parametrize("F", [64, 128, 12, 5000])
@pytest.mark.parametrize("star", [False, True])
def test_spmm_forward_and_transpose(F, star):
    from bigcn_amd.ops import build_graph, spmm
    rng = np.random.default_rng(F)
    sizes = [2, 3, 700, 5, 64] if not star else [3000, 2, 33]
    ei, N = rand_forest(rng, sizes, star=star)
    g = build_graph(ei.to(DEV), N)
    e, w = O.gcn_norm(ei, None, N, "col", dtype=torch.float64)
    A = torch.zeros(N, N, dtype=torch.float64)
    A.index_put_((e[1], e[0]), w, accumulate=True)
    x = torch.randn(N, F, dtype=torch.float64)
    bias = torch.randn(F, dtype=torch.float64)
    out = spmm(g, x.float().to(DEV), bias.float().to(DEV))
    close(out, A @ x + bias, what="A x + b")
    outr = spmm(g, x.float().to(DEV), bias.float().to(DEV), relu=True)
    close(outr, torch.relu(A @ x + bias), what="relu")
    outt = spmm(g, x.float().to(DEV), transposed=True)
    close(outt, A.t() @ x, what="A^T x")


@pytest.mark.parametrize("F", [12, 300, 5000, 6144])
def test_spmm_wide_row_lengths_around_chunk_size(F):
    """Wide kernel chunking: rows of 14..18 and 31..34 entries (around the 16-entry
    chunk, where boundaries are moved to row starts or rows are split) at every offset."""
    from bigcn_amd.ops import build_graph, spmm
    rows, cols, off = [], [], 0
    for deg in [15, 16, 17, 1, 31, 32, 33, 2, 14, 18, 34, 0, 16, 16, 1, 17]:
        for c in range(deg):        # a star: parent `off`, children off+1..off+deg
            rows.append(off)
            cols.append(off + 1 + c)
        off += deg + 1
    N = off
    ei = torch.tensor([rows, cols], dtype=torch.int64)
    g = build_graph(ei.to(DEV), N)
    e, w = O.gcn_norm(ei, None, N, "col", dtype=torch.float64)
    A = torch.zeros(N, N, dtype=torch.float64)
    A.index_put_((e[1], e[0]), w, accumulate=True)
    x = torch.randn(N, F, dtype=torch.float64)
    close(spmm(g, x.float().to(DEV)), A @ x, what="A x")
    close(spmm(g, x.float().to(DEV), transposed=True), A.t() @ x, what="A^T x")


def test_spmm_wide_many_chunks_per_block():
    """Wide kernel with > 512 chunks per block (chunk boundaries computed in several
    windows, next-chunk entries prefetched across window edges): 1.2M nodes of random
    trees and stars, F = 12, against an index_add restatement in fp64."""
    from bigcn_amd.ops import build_graph, spmm
    rng = np.random.default_rng(11)
    sizes = rng.integers(2, 400, size=6000)
    sizes[::50] = 3000                      # star roots split over many chunks
    n = int(sizes.sum())
    par = []
    off = 0
    for s in sizes:                         # vectorised rand_forest: parent 0 or uniform earlier
        k = np.arange(1, s)
        p = np.where(rng.random(s - 1) < 0.5, 0, (rng.random(s - 1) * np.maximum(k - 1, 1)).astype(np.int64) + 1)
        p = np.where(k == 1, 0, np.minimum(p, k - 1))
        if s == 3000:
            p[:] = 0
        par.append(np.stack([off + p, off + k]))
        off += s
    ei = torch.from_numpy(np.concatenate(par, 1))
    g = build_graph(ei.to(DEV), n)
    e, w = O.gcn_norm(ei, None, n, "col", dtype=torch.float64)
    x = torch.randn(n, 12, dtype=torch.float64)
    for transposed in (False, True):
        src, dst = (e[1], e[0]) if transposed else (e[0], e[1])
        ref = torch.zeros(n, 12, dtype=torch.float64).index_add_(0, dst, w[:, None] * x[src])
        close(spmm(g, x.float().to(DEV), transposed=transposed), ref, what=f"A x (T={transposed})")


def test_spmm_any_width_and_rejects_bad_width():
    """The wide aggregation has no width limit (256-float slices); F must stay a
    multiple of 4 (float4 rows), else the C ABI refuses the call."""
    from bigcn_amd._lib import BGCNError
    from bigcn_amd.ops import build_graph, spmm
    ei = torch.tensor([[0, 0, 1], [1, 2, 3]])
    g = build_graph(ei.to(DEV), 4)
    e, w = O.gcn_norm(ei, None, 4, "col", dtype=torch.float64)
    A = torch.zeros(4, 4, dtype=torch.float64)
    A.index_put_((e[1], e[0]), w, accumulate=True)
    x = torch.randn(4, 9000, dtype=torch.float64)
    close(spmm(g, x.float().to(DEV)), A @ x, what="A x at F=9000")
    with pytest.raises(BGCNError):
        spmm(g, torch.zeros(4, 6146, device=DEV))


def test_spmm_deterministic():
    from bigcn_amd.ops import build_graph, spmm
    rng = np.random.default_rng(5)
    ei, N = rand_forest(rng, [2000, 100, 5], star=True)
    g = build_graph(ei.to(DEV), N)
    x = torch.randn(N, 64, device=DEV)
    a = spmm(g, x, transposed=True)
    b = spmm(g, x, transposed=True)
    assert torch.equal(a, b)


@pytest.mark.parametrize("M,Nc,K", [(1000, 128, 5000), (8300, 128, 5000), (77, 64, 5064), (130, 20, 37), (5, 128, 8)])
def test_gemm_xwt(M, Nc, K):
    from bigcn_amd import _lib
    from bigcn_amd._lib import check, ptr, stream_handle
    torch.manual_seed(M)
    X = torch.randn(M, K, dtype=torch.float64)
    W = torch.randn(Nc, K, dtype=torch.float64)
    Xd, Wd = X.float().to(DEV), W.float().to(DEV)
    Y = torch.empty(M, Nc, device=DEV)
    split = Nc // 2
    check(_lib.lib().bgcn_gemm_xwt(ptr(Xd), K, ptr(Wd), ptr(Wd[split:]), K, split, ptr(Y), Nc, M, Nc, K,
                                   stream_handle()))
    close(Y, X @ W.t(), 1e-5, "X W^T")


def _segment_tail(rows, cols):
    """A [rows, cols] fp32 view ending exactly at the end of its own allocation (a fresh
    2 MiB-multiple block of the caching allocator): any read past its last element leaves
    the allocation."""
    n = rows * cols
    seg = 2 << 20
    total = (n * 4 + seg - 1) // seg * seg // 4
    torch.cuda.empty_cache()
    buf = torch.empty(total, device=DEV)
    return buf[total - n:].view(rows, cols)


def test_gemm_xwt_operands_at_allocation_end():
    """The six-product conv1 (k_gemm_xwt_x6p, >= 8192 rows) prefetches k-tiles past the last
    one; with X and W ending exactly at their allocations' ends those loads must read zeros
    through the buffer range check (the tile offset rides in the VGPR offset), not past the
    allocation."""
    from bigcn_amd import _lib
    from bigcn_amd._lib import check, ptr, stream_handle
    M, Nc, K = 8200, 128, 5000
    torch.manual_seed(7)
    X = torch.randn(M, K, dtype=torch.float64)
    W = torch.randn(Nc, K, dtype=torch.float64)
    Xd = _segment_tail(M, K)
    Xd.copy_(X.float())
    Wd = _segment_tail(Nc, K)
    Wd.copy_(W.float())
    Y = torch.empty(M, Nc, device=DEV)
    split = Nc // 2
    check(_lib.lib().bgcn_gemm_xwt(ptr(Xd), K, ptr(Wd), ptr(Wd[split:]), K, split, ptr(Y), Nc, M, Nc, K,
                                   stream_handle()))
    close(Y, X @ W.t(), 1e-5, "X W^T at the allocation end")


@pytest.mark.parametrize("M,Nc,K", [(500, 5000, 64), (33, 13, 7), (64, 128, 128)])
def test_gemm_xw(M, Nc, K):
    from bigcn_amd import _lib
    from bigcn_amd._lib import check, ptr, stream_handle
    torch.manual_seed(K)
    X = torch.randn(M, K, dtype=torch.float64)
    W = torch.randn(K, Nc, dtype=torch.float64)
    Xd, Wd = X.float().to(DEV), W.float().to(DEV)
    Y = torch.empty(M, Nc, device=DEV)
    check(_lib.lib().bgcn_gemm_xw(ptr(Xd), K, ptr(Wd), Nc, ptr(Y), Nc, M, Nc, K, stream_handle()))
    close(Y, X @ W, 1e-5, "X W")


@pytest.mark.parametrize("Mc,Nc,K", [(128, 5000, 3000), (64, 5064, 257), (20, 30, 1000), (128, 64, 5)])
def test_gemm_tn(Mc, Nc, K):
    from bigcn_amd import _lib
    from bigcn_amd._lib import check, ptr, stream_handle, workspace
    torch.manual_seed(Mc + Nc)
    G = torch.randn(K, Mc, dtype=torch.float64)
    X = torch.randn(K, Nc, dtype=torch.float64)
    Gd, Xd = G.float().to(DEV), X.float().to(DEV)
    split = Mc // 2
    C0 = torch.empty(split, Nc, device=DEV)
    C1 = torch.empty(Mc - split, Nc, device=DEV)
    L = _lib.lib()
    ws = workspace(L.bgcn_gemm_tn_workspace_size(Mc, Nc, K), DEV)
    check(L.bgcn_gemm_tn(ptr(Gd), Mc, ptr(Xd), Nc, ptr(C0), ptr(C1), Nc, split, Mc, Nc, K, ptr(ws),
                         ws.numel(), stream_handle()))
    ref = G.t() @ X
    close(torch.cat([C0, C1]), ref, 1e-5, "G^T X")


def test_colsum():
    from bigcn_amd import _lib
    from bigcn_amd._lib import check, ptr, stream_handle, workspace
    A = torch.randn(3001, 70, dtype=torch.float64)
    Ad = A.float().to(DEV)
    out = torch.empty(70, device=DEV)
    L = _lib.lib()
    ws = workspace(L.bgcn_colsum_workspace_size(3001, 70), DEV)
    check(L.bgcn_colsum(ptr(Ad), 70, 3001, 70, ptr(out), ptr(ws), ws.numel(), stream_handle()))
    close(out, A.sum(0), 1e-5)


@pytest.mark.parametrize("sorted_index", [True, False])
def test_scatter_mean(sorted_index):
    from bigcn_amd import scatter_mean
    torch.manual_seed(0)
    n, C, B = 5000, 128, 40
    idx = torch.randint(0, B, (n,))
    idx[idx == 7] = 8                      # an empty segment
    if sorted_index:
        idx = idx.sort().values
    src = torch.randn(n, C, dtype=torch.float64, requires_grad=True)
    ref = O.scatter_mean(src, idx, dim_size=B)
    ref.backward(torch.ones_like(ref) * torch.arange(C, dtype=torch.float64))
    s = src.detach().float().to(DEV).requires_grad_(True)
    out = scatter_mean(s, idx.to(DEV), dim=0, dim_size=B)
    close(out, ref, what="fwd")
    out.backward(torch.ones_like(out) * torch.arange(C, device=DEV, dtype=torch.float32))
    close(s.grad, src.grad, what="bwd")


def test_gcnconv_module_fwd_bwd():
    from bigcn_amd import GCNConv
    rng = np.random.default_rng(11)
    ei, N = rand_forest(rng, [50, 3, 200])
    torch.manual_seed(0)
    conv = GCNConv(333, 64).to(DEV)
    with torch.no_grad():
        conv.bias.uniform_(-0.1, 0.1)
    assert set(conv.state_dict()) == {"lin.weight", "bias"}
    x = torch.rand(N, 333, dtype=torch.float64, requires_grad=True)
    w = conv.lin.weight.detach().double().cpu().requires_grad_(True)
    b = conv.bias.detach().double().cpu().requires_grad_(True)
    ref = O.gcn_conv(x, ei, w, b)
    gout = torch.randn_like(ref)
    ref.backward(gout)
    xd = x.detach().float().to(DEV).requires_grad_(True)
    out = conv(xd, ei.to(DEV))
    out.backward(gout.float().to(DEV))
    close(out, ref, what="out")
    close(xd.grad, x.grad, what="dx")
    close(conv.lin.weight.grad, w.grad, what="dW")
    close(conv.bias.grad, b.grad, what="db")


@pytest.mark.parametrize("degree_on", ["col", "row"])
def test_gcnconv_edge_weight_fwd_bwd(degree_on):
    """GCNConv(x, edge_index, edge_weight) as EBGCN calls it (EBGCN.py:84,178): the
    per-edge weight enters gcn_norm's degree and every message; grads w.r.t. x, W, b."""
    from bigcn_amd import GCNConv
    rng = np.random.default_rng(12)
    ei, N = rand_forest(rng, [40, 2, 130], star=True)
    ew = torch.rand(ei.size(1), dtype=torch.float64) * 2.0 + 0.05
    torch.manual_seed(1)
    conv = GCNConv(96, 64, degree_on=degree_on).to(DEV)
    with torch.no_grad():
        conv.bias.uniform_(-0.1, 0.1)
    x = torch.randn(N, 96, dtype=torch.float64, requires_grad=True)
    w = conv.lin.weight.detach().double().cpu().requires_grad_(True)
    b = conv.bias.detach().double().cpu().requires_grad_(True)
    ref = O.gcn_conv(x, ei, w, b, edge_weight=ew, degree_on=degree_on)
    gout = torch.randn_like(ref)
    ref.backward(gout)
    xd = x.detach().float().to(DEV).requires_grad_(True)
    out = conv(xd, ei.to(DEV), ew.float().to(DEV))
    out.backward(gout.float().to(DEV))
    close(out, ref, what="out")
    close(xd.grad, x.grad, what="dx")
    close(conv.lin.weight.grad, w.grad, what="dW")
    close(conv.bias.grad, b.grad, what="db")


def _dump_errors(name, pairs, floors=None):
    """Per tensor the max-scaled error and the worst elementwise ratio |a - b| / (|b| +
    floor max|b|) (the test's own floor: 1e-3 unless `floors` names another) against the fp64
    reference, under gpurun_out/parity/ (kept per round under profiles/)."""
    import json
    import os
    out = {}
    for k, (a, b) in pairs.items():
        a = torch.as_tensor(a).detach().double().cpu()
        b = torch.as_tensor(b).detach().double().cpu()
        m = float(b.abs().max())
        err = (a - b).abs()
        fl = (floors or {}).get(k, 1e-3)
        out[k] = {"max_scaled": float(err.max()) / max(m, 1e-300), "floor": fl,
                  "elementwise": float((err / (b.abs() + fl * m).clamp_min(1e-300)).max())}
    d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "parity")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, name + ".json"), "w") as f:
        json.dump({"tol": 1e-4, "errors": out}, f, indent=1)


def close_elem(a, b, what="", rtol=1e-4, floor=1e-3):
    """Elementwise: |a - b| <= rtol * (|b| + floor * max|b|) (fp32 kernels vs fp64 oracle)."""
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    assert a.shape == b.shape, what
    bound = rtol * (b.abs() + floor * float(b.abs().max()))
    bad = (a - b).abs() > bound
    assert not bool(bad.any()), f"{what}: {int(bad.sum())} of {b.numel()} off, worst {float(((a - b).abs() / bound).max()):.2f}x"


@pytest.mark.parametrize("degree_on", ["col", "row"])
def test_gcnconv_learned_edge_weight(degree_on):
    """EBGCN's call form with a LEARNED edge weight: edge_pred = sigmoid(fc(sim)) (EBGCN.py:
    101-102) passed as GCNConv(x, edge_index, edge_weight=edge_pred) (:84,178).  The gradient
    flows through gcn_norm (the per-edge norm and every node's degree) into the weight and on
    into fc - all against O.gcn_conv autograd (fp64), elementwise 1e-4, on a star-heavy
    forest with an input self loop (its weight becomes the node's loop weight)."""
    from bigcn_amd import GCNConv
    rng = np.random.default_rng(13)
    ei, N = rand_forest(rng, [40, 2, 130, 7], star=True)
    ei = torch.cat([ei, torch.tensor([[5], [5]])], 1)                  # an input self loop
    E = ei.size(1)
    torch.manual_seed(2)
    conv = GCNConv(96, 64, degree_on=degree_on).to(DEV)
    with torch.no_grad():
        conv.bias.uniform_(-0.1, 0.1)
    fc = torch.nn.Linear(8, 1).double()
    sim = torch.randn(E, 8, dtype=torch.float64)
    x = torch.randn(N, 96, dtype=torch.float64, requires_grad=True)
    w = conv.lin.weight.detach().double().cpu().requires_grad_(True)
    b = conv.bias.detach().double().cpu().requires_grad_(True)
    ew = torch.sigmoid(fc(sim)).view(-1)
    ew.retain_grad()
    ref = O.gcn_conv(x, ei, w, b, edge_weight=ew, degree_on=degree_on)
    gout = torch.randn_like(ref)
    ref.backward(gout)
    fcd = torch.nn.Linear(8, 1).to(DEV)
    with torch.no_grad():
        fcd.weight.copy_(fc.weight.float())
        fcd.bias.copy_(fc.bias.float())
    xd = x.detach().float().to(DEV).requires_grad_(True)
    ewd = torch.sigmoid(fcd(sim.float().to(DEV))).view(-1)
    ewd.retain_grad()
    out = conv(xd, ei.to(DEV), ewd)
    out.backward(gout.float().to(DEV))
    close(out, ref, what="out")
    _dump_errors(f"edge_weight_{degree_on}", {
        "out": (out, ref), "d edge_weight": (ewd.grad, ew.grad), "dx": (xd.grad, x.grad),
        "dW": (conv.lin.weight.grad, w.grad), "db": (conv.bias.grad, b.grad),
        "d fc.weight": (fcd.weight.grad, fc.weight.grad)}, floors={"d edge_weight": 1e-2})
    # dL/dw_e = g_e dis[s] dis[d] + dL/ddeg[key]: the two terms nearly cancel on some edges,
    # so the elementwise floor is 1e-2 of the largest gradient (still 1e-6 of it absolute)
    close_elem(ewd.grad, ew.grad, what="d edge_weight", floor=1e-2)
    close_elem(xd.grad, x.grad, what="dx")
    close_elem(conv.lin.weight.grad, w.grad, what="dW")
    close_elem(conv.bias.grad, b.grad, what="db")
    close_elem(fcd.weight.grad, fc.weight.grad, what="d fc.weight (through the edge weights)")
    # a prebuilt graph has its weights baked in: a learned weight needs the edge list
    from bigcn_amd.ops import build_graph, gcn_conv
    g = build_graph(ei.to(DEV), N, ewd.detach())
    with pytest.raises(ValueError):
        gcn_conv(xd, g, conv.lin.weight, conv.bias, ewd)
