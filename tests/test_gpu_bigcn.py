"""GPU parity of the fused BiGCN encoder + model against the oracle and golden fixtures.

Tolerance: fp32 HIP path vs fp64 oracle, |a - b| <= 1e-4 * max|b| per tensor
(log-probs, loss, every parameter gradient).  Dropout is compared with the SAME keep
mask: either injected (golden fixtures) or the in-kernel mask materialised with
``bgcn_keep_words`` and fed to the oracle.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import golden_batch, golden_params, load_golden
from oracle import bigcn_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-4

GOLDEN = ["bigcn_eval_mixed.npz", "bigcn_train_mixed.npz", "bigcn_train_dropedge.npz",
          "bigcn_eval_stars_rowdeg.npz", "bigcn_train_rootmid.npz", "bigcn_eval_single.npz",
          "bigcn_train_alldropped.npz"]

ENC_KEYS = ["TDrumorGCN.conv1.lin.weight", "TDrumorGCN.conv1.bias", "TDrumorGCN.conv2.lin.weight",
            "TDrumorGCN.conv2.bias", "BUrumorGCN.conv1.lin.weight", "BUrumorGCN.conv1.bias",
            "BUrumorGCN.conv2.lin.weight", "BUrumorGCN.conv2.bias"]


def close(a, b, tol=TOL, what=""):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    assert a.shape == b.shape, (what, a.shape, b.shape)
    scale = float(b.abs().max()) if b.numel() else 1.0
    err = float((a - b).abs().max()) if b.numel() else 0.0
    assert err <= tol * max(scale, 1e-12), f"{what}: max err {err:.3e} vs scale {scale:.3e}"


def gpu_step(b, p, training, keep_words=None, degree_on="col", seed=0, mode="auto"):
    """Fused encoder + torch head on the GPU; returns (logp, loss, grads, head)."""
    from bigcn_amd.ops import bigcn_encoder, build_graph
    q = {k: v.float().to(DEV).contiguous().requires_grad_(True) for k, v in p.items()}
    N = b.x.size(0)
    td = build_graph(b.edge_index, N, degree_on=degree_on, validate=True)
    bu = build_graph(b.BU_edge_index, N, degree_on=degree_on, validate=True)
    head = bigcn_encoder(b.x, b.batch, b.rootindex, td, bu, b.num_graphs, [q[k] for k in ENC_KEYS],
                         training=training, seed=seed, keep_words=keep_words, feat_mode=mode)
    logp = F.log_softmax(F.linear(head, q["fc.weight"], q["fc.bias"]), dim=1)
    loss = F.nll_loss(logp, b.y)
    loss.backward()
    return logp, loss, {k: v.grad for k, v in q.items()}, head


@pytest.mark.parametrize("mode", ["auto", "dense"])
@pytest.mark.parametrize("name", GOLDEN)
def test_fused_matches_golden(name, mode):
    from bigcn_amd.ops import pack_keep
    g = load_golden(name)
    b = golden_batch(g, DEV)
    p = golden_params(g)
    training = bool(g["training"])
    kw = None
    if training:
        kw = torch.stack([pack_keep(torch.as_tensor(g["td_keep"])), pack_keep(torch.as_tensor(g["bu_keep"]))]).to(DEV)
    logp, loss, grads, head = gpu_step(b, p, training, kw, str(g["degree_on"]), mode=mode)
    close(head, g["stage:head_in"], what="head_in")
    close(logp, g["logp"], what="logp")
    close(loss, g["loss"], what="loss")
    for k in p:
        close(grads[k], g["grad:" + k], what=k)


@pytest.mark.parametrize("name", GOLDEN)
def test_dense_dw2_root_tiles_on_small_trees(name, monkeypatch):
    """The dense path's dW2 root columns as tree-run k-tiles (``k_dw2_root``) forced onto
    the golden batches (``BGCN_DW2_ROOT=2``; the library keeps ``k_dw2_f32`` below 32 nodes
    per tree): runs of one node (single-node trees), stars, a root in mid-batch, injected
    keep words whose last column tile reaches past the node's words (F = 96: the clamped
    word), against the fixture at the same tolerance."""
    monkeypatch.setenv("BGCN_DW2_ROOT", "2")
    test_fused_matches_golden(name, "dense")


def _synth(seed, B, mean, F=5000, droprates=(0.2, 0.2), root_random=False):
    from bigcn_amd.data import synth_batch, synth_tree_sizes
    rng = np.random.default_rng(seed)
    sizes = synth_tree_sizes(rng, B, mean)
    return synth_batch(rng, sizes, F, 4, *droprates, device=DEV, root_random=root_random)


def _oracle(b, p, training, td_mask=None, bu_mask=None, degree_on="col", relu_masks=None):
    batch = {"x": b.x.double().cpu(), "edge_index": b.edge_index.cpu(), "BU_edge_index": b.BU_edge_index.cpu(),
             "batch": b.batch.cpu(), "rootindex": b.rootindex.cpu(), "y": b.y.cpu()}
    pd = {k: v.double() for k, v in p.items()}
    st = {}
    loss, logp, grads = O.reference_grads(pd, batch, training, td_mask, bu_mask, degree_on, st, relu_masks)
    return logp, loss, grads, st


@pytest.mark.parametrize("mode", ["auto", "dense"])
@pytest.mark.parametrize("training", [False, True])
def test_fused_midsize_5000_features(training, mode):
    """B = 12 trees (~120 nodes each), F = 5000: the real feature width, in-kernel dropout
    mask materialised for the oracle."""
    from bigcn_amd.ops import keep_words, unpack_keep
    b = _synth(21, 12, 120, root_random=True)
    p = O.make_params(5000, 64, 64, 4, seed=5)
    N = b.x.size(0)
    seed = 1234567
    masks = (None, None)
    if training:
        kw = keep_words(seed, N, 5000, DEV)
        m = unpack_keep(kw, 64 + 5000).cpu()
        masks = (m[0], m[1])
        frac = float(m.float().mean())
        assert 0.49 < frac < 0.51, frac
        assert not torch.equal(m[0], m[1])
    logp, loss, grads, head = gpu_step(b, p, training, None, seed=seed, mode=mode)
    rlogp, rloss, rgrads, st = _oracle(b, p, training, *masks)
    close(head, st["head_in"], what="head_in")
    close(logp, rlogp, what="logp")
    for k in p:
        close(grads[k], rgrads[k], what=k)


@pytest.mark.parametrize("mode", ["auto", "dense"])
def test_fused_is_deterministic_full_size(mode):
    """Full Twitter15-shaped batch (B = 128, mean 256 nodes, F = 5000): two runs of the
    training step give bitwise-identical outputs and gradients (atomic-free kernels)."""
    b = _synth(22, 128, 256)
    p = O.make_params(5000, 64, 64, 4, seed=6)
    r1 = gpu_step(b, p, True, None, seed=99, mode=mode)
    r2 = gpu_step(b, p, True, None, seed=99, mode=mode)
    assert torch.equal(r1[0], r2[0])
    for k in r1[2]:
        assert torch.equal(r1[2][k], r2[2][k]), k
    r3 = gpu_step(b, p, True, None, seed=100, mode=mode)   # another draw changes the result
    assert not torch.equal(r1[0], r3[0])
    assert torch.isfinite(r1[1])


@pytest.mark.parametrize("mode", ["auto", "dense"])
def test_aux_stream_branches_match_inline(mode):
    """On a non-default stream the fused step forks independent branches (the CSC of X,
    the dW2 chain) onto the library's auxiliary stream; on the legacy null stream they
    run inline.  Both schedules give bitwise-identical results, also when the caller's
    stream is busy with unrelated work queued ahead of the step."""
    b = _synth(23, 64, 256)
    p = O.make_params(5000, 64, 64, 4, seed=7)
    r0 = gpu_step(b, p, True, None, seed=11, mode=mode)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        big = torch.randn(4096, 4096, device=DEV)
        for _ in range(4):
            big = big @ big * 1e-3                     # keeps the stream busy ahead of the step
        r1 = gpu_step(b, p, True, None, seed=11, mode=mode)
    torch.cuda.synchronize()
    assert torch.equal(r0[0], r1[0])
    for k in r0[2]:
        assert torch.equal(r0[2][k], r1[2][k]), k


def test_sparse_and_dense_paths_agree_full_size():
    """The sparse feature path and the dense MFMA path compute the same step (fp32
    rounding only) on a full Twitter15-shaped batch."""
    b = _synth(25, 128, 256)
    p = O.make_params(5000, 64, 64, 4, seed=8)
    rs = gpu_step(b, p, True, None, seed=5, mode="auto")
    rd = gpu_step(b, p, True, None, seed=5, mode="dense")
    close(rs[3], rd[3], what="head")
    for k in rs[2]:
        close(rs[2][k], rd[2][k], what=k)


@pytest.mark.parametrize("mean,root", [(8, "1"), (8, "2"), (200, "1"), (200, "0")])
def test_dense_bf16_dw2_forms_agree_with_sparse_path(mean, root, monkeypatch):
    """bf16 X on the dense path against the sparse path on the same bf16 batch: small trees
    (mean 8: ``k_dw2_bf16`` with the H1 columns' blocks in its launch by default, the
    tree-run tiles of ``k_dw2_root<bf16>`` forced by BGCN_DW2_ROOT=2) and Twitter-sized ones
    (``k_dw2_root`` by default, ``k_dw2_bf16`` with BGCN_DW2_ROOT=0)."""
    from bigcn_amd.data import synth_batch, synth_tree_sizes
    monkeypatch.setenv("BGCN_DW2_ROOT", root)
    rng = np.random.default_rng(31 + mean)
    sizes = synth_tree_sizes(rng, 64 if mean == 200 else 400, mean)
    b = synth_batch(rng, sizes, 5000, 4, 0.2, 0.2, device=DEV, dtype=torch.bfloat16)
    p = O.make_params(5000, 64, 64, 4, seed=9)
    rs = gpu_step(b, p, True, None, seed=7, mode="auto")
    rd = gpu_step(b, p, True, None, seed=7, mode="dense")
    close(rs[3], rd[3], what="head")
    for k in rs[2]:
        close(rs[2][k], rd[2][k], what=k)


@pytest.mark.parametrize("dense_rows", [1, 200])
def test_sparse_overflow_falls_back_to_dense(dense_rows):
    """Dense rows (512 non-zeros): one fits the spill pool (the sparse path adds its spilled
    terms), 200 exceed it and switch the batch to the dense path on the device; results
    match the oracle either way."""
    from bigcn_amd.ops import keep_words, unpack_keep
    b = _synth(26, 6, 60, F=512)
    g = torch.Generator().manual_seed(3)
    rows = torch.randperm(b.x.size(0), generator=g)[:dense_rows]
    b.x[rows.to(DEV)] = torch.rand(dense_rows, 512, generator=g).to(DEV)
    p = O.make_params(512, 64, 64, 4, seed=9)
    N = b.x.size(0)
    m = unpack_keep(keep_words(7, N, 512, DEV), 64 + 512).cpu()
    logp, loss, grads, head = gpu_step(b, p, True, None, seed=7, mode="auto")
    rlogp, _, rgrads, st = _oracle(b, p, True, m[0], m[1])
    close(logp, rlogp, what="logp")
    for k in p:
        close(grads[k], rgrads[k], what=k)


def test_model_module_matches_oracle_and_state_dict():
    from bigcn_amd import BiGCN, Net, make_optimizer
    torch.manual_seed(0)
    m = BiGCN(5000, 64, 64, DEV).to(DEV)
    ref_keys = {"TDrumorGCN.conv1.lin.weight", "TDrumorGCN.conv1.bias", "TDrumorGCN.conv2.lin.weight",
                "TDrumorGCN.conv2.bias", "BUrumorGCN.conv1.lin.weight", "BUrumorGCN.conv1.bias",
                "BUrumorGCN.conv2.lin.weight", "BUrumorGCN.conv2.bias", "fc.weight", "fc.bias"}
    assert set(m.state_dict()) == ref_keys
    assert m.state_dict()["TDrumorGCN.conv2.lin.weight"].shape == (64, 5064)
    assert Net(5000, 64, 64).fc.out_features == 2
    b = _synth(23, 6, 80)
    m.eval()
    logp = m(b)
    p = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    rlogp, _, _, _ = _oracle(b, p, False)
    close(logp, rlogp, what="eval logp")
    # one training step with the reference optimiser groups
    m.train()
    opt = make_optimizer(m)
    loss = F.nll_loss(m(b), b.y)
    opt.zero_grad()
    loss.backward()
    opt.step()
    assert all(torch.isfinite(v).all() for v in m.state_dict().values())


def test_direction_modules_generic_path():
    """TDrumorGCN / BUrumorGCN called on their own (drop-in GCNConv + scatter_mean)."""
    from bigcn_amd import BiGCN
    torch.manual_seed(1)
    m = BiGCN(5000, 64, 64).to(DEV).eval()
    b = _synth(24, 5, 60, root_random=True)
    p = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    _, _, _, st = _oracle(b, p, False)
    close(m.TDrumorGCN(b), st["TDrumorGCN.out"], what="TD")
    close(m.BUrumorGCN(b), st["BUrumorGCN.out"], what="BU")
    head = m.encode(b)
    close(head, st["head_in"], what="fused head")


@pytest.mark.parametrize("B,C", [(1, 4), (3, 2), (128, 4), (130, 16), (300, 2)])
def test_head_kernels_match_torch(B, C):
    """K9 (bgcn_head_forward / _backward) against torch's Linear + log_softmax and autograd,
    in fp64, for an arbitrary upstream gradient dlogp; elementwise bar
    |a - b| <= 1e-5 * (|b| + rms(b))."""
    from bigcn_amd import _lib
    from bigcn_amd._lib import check, stream_handle
    g = torch.Generator().manual_seed(B * 31 + C)
    head = torch.randn(B, 256, generator=g).abs()           # relu'd readout values
    W = torch.randn(C, 256, generator=g) * 0.06
    bias = torch.randn(C, generator=g) * 0.1
    dlogp = torch.randn(B, C, generator=g)
    hd, Wd, bd = (t.double().requires_grad_(True) for t in (head, W, bias))
    ref = F.log_softmax(F.linear(hd, Wd, bd), dim=1)
    ref.backward(dlogp.double())
    L = _lib.lib()
    h, w, bb, dl = (t.to(DEV).contiguous() for t in (head, W, bias, dlogp))
    logp = torch.empty(B, C, device=DEV)
    dhead, dW, db = torch.empty(B, 256, device=DEV), torch.empty(C, 256, device=DEV), torch.empty(C, device=DEV)
    s = stream_handle()
    check(L.bgcn_head_forward(h.data_ptr(), w.data_ptr(), bb.data_ptr(), B, C, logp.data_ptr(), s))
    check(L.bgcn_head_backward(h.data_ptr(), logp.data_ptr(), dl.data_ptr(), w.data_ptr(), B, C,
                               dhead.data_ptr(), dW.data_ptr(), db.data_ptr(), s))
    for a, b, what in ((logp, ref, "logp"), (dhead, hd.grad, "dhead"), (dW, Wd.grad, "dW"), (db, bd.grad, "db")):
        a, b = a.double().cpu(), b.detach().cpu()
        rms = float(b.pow(2).mean().sqrt())
        bad = (a - b).abs() > 1e-5 * (b.abs() + rms)
        assert not bad.any(), f"{what}: {int(bad.sum())} elements off, max err {float((a - b).abs().max()):.3e}"


def test_head_rejects_bad_shapes():
    from bigcn_amd import _lib
    from bigcn_amd._lib import stream_handle
    L = _lib.lib()
    h = torch.empty(4, 256, device=DEV)
    w = torch.empty(17, 256, device=DEV)
    out = torch.empty(4, 17, device=DEV)
    assert L.bgcn_head_forward(h.data_ptr(), w.data_ptr(), w.data_ptr(), 4, 17, out.data_ptr(), stream_handle()) != 0
    assert L.bgcn_head_forward(h.data_ptr(), w.data_ptr(), 0, 4, 4, out.data_ptr(), stream_handle()) != 0


@pytest.mark.parametrize("cls", ["BiGCN", "Net"])
def test_model_fused_head_matches_torch_head(cls):
    """BiGCN.forward with the K9 head in the encoder's node (fused_head, the default) against
    the same model with torch's fc + log_softmax: same dropout seed, logp and every
    parameter gradient (fc included) after F.nll_loss(...).backward()."""
    import bigcn_amd
    torch.manual_seed(3)
    m = getattr(bigcn_amd, cls)(5000, 64, 64, DEV).to(DEV).train()
    b = _synth(41, 9, 70)
    if cls == "Net":
        b.y = b.y % 2
    out = {}
    for fused in (True, False):
        m.fused_head = fused
        m.zero_grad(set_to_none=True)
        logp = m(b, seed=1234)
        F.nll_loss(logp, b.y).backward()
        out[fused] = (logp.detach().clone(), {k: p.grad.detach().clone() for k, p in m.named_parameters()})
    close(out[True][0], out[False][0], tol=1e-5, what="logp")
    for k in out[False][1]:
        close(out[True][1][k], out[False][1][k], tol=1e-5, what=k)


def test_model_sparse_hint_matches_gated_auto():
    """BiGCN.forward on a batch whose hints say its rows fit (BGCN_FEAT_SPARSE: the dense
    fallback kernels are not launched) computes the same step, bit for bit, as with the
    hints dropped (auto: the fallback launched and gated off on the device)."""
    from bigcn_amd import BiGCN, _lib
    from bigcn_amd.ops import feat_path
    torch.manual_seed(5)
    m = BiGCN(5000, 64, 64, DEV).to(DEV).train()
    b = _synth(43, 7, 90)
    assert feat_path("auto", b) == _lib.BGCN_FEAT_SPARSE
    out = []
    for hinted in (True, False):
        if not hinted:
            b._x_nnz_of = None
            assert feat_path("auto", b) == _lib.BGCN_FEAT_AUTO
        m.zero_grad(set_to_none=True)
        logp = m(b, seed=99)
        F.nll_loss(logp, b.y).backward()
        out.append((logp.detach().clone(), [p.grad.detach().clone() for p in m.parameters()]))
    assert torch.equal(out[0][0], out[1][0])
    for a, c in zip(out[0][1], out[1][1]):
        assert torch.equal(a, c)


@pytest.mark.parametrize("plan", ["1", "0"])
def test_model_train_step_matches_oracle(plan, monkeypatch):
    """The drop-in model step (BiGCN.forward -> F.nll_loss -> backward) at F = 5000 in
    training mode against the oracle with the in-kernel dropout draw materialised.  The
    model's graphs come from bgcn_build_graph_pair with their aggregation plans
    (bgcn_graph_pair_plans): plan "1" runs the planned aggregation and the sign-word readout
    backward, "0" (BGCN_SPMM_PLAN=0) the merge-path chunks + fix-up and k_readout_bwd."""
    from bigcn_amd import BiGCN
    from bigcn_amd.ops import keep_words, unpack_keep
    monkeypatch.setenv("BGCN_SPMM_PLAN", plan)
    b = _synth(25, 12, 120, root_random=True)
    p = O.make_params(5000, 64, 64, 4, seed=7)
    m = BiGCN(5000, 64, 64, DEV).to(DEV)
    m.load_state_dict({k: v.float() for k, v in p.items()})
    m.train()
    seed = 424242
    logp = m(b, seed=seed)
    loss = F.nll_loss(logp, b.y)
    loss.backward()
    km = unpack_keep(keep_words(seed, b.x.size(0), 5000, DEV), 64 + 5000).cpu()
    rlogp, rloss, rgrads, _ = _oracle(b, p, True, km[0], km[1])
    close(logp, rlogp, what="logp")
    close(loss, rloss, what="loss")
    grads = dict((k, q.grad) for k, q in m.named_parameters())
    for k in p:
        close(grads[k], rgrads[k], what=k)


@pytest.mark.parametrize("fused_step", [False, True])
def test_edge_across_trees(fused_step):
    """An edge joining two trees (never made by PyG collation, but legal for GCNConv +
    scatter_mean): K1 built with the batch vector flags BGCN_STATUS_CROSS_TREE and the
    sign-word readout backward then scales every gathered row by its own tree - gradients
    match the oracle and the general readout backward (graphs built without the check)."""
    from bigcn_amd import _lib
    from bigcn_amd.ops import bigcn_encoder, build_graph_pair
    b = _synth(77, 6, 20, droprates=(0.0, 0.0))
    N = b.x.size(0)
    u, v = int(b.ptr[0]) + 1, int(b.ptr[2]) + 2          # tree 0 -> tree 2
    extra = torch.tensor([[u], [v]], device=DEV)
    b.edge_index = torch.cat([b.edge_index, extra], 1)
    b.BU_edge_index = torch.cat([b.BU_edge_index, extra.flip(0)], 1)
    p = O.make_params(5000, 64, 64, 4, seed=31)
    _, rloss, rgrads, _ = _oracle(b, p, False)
    if fused_step:
        from bigcn_amd import FusedTrainStep
        from test_gpu_train import _model
        m = _model(p)
        m.eval()
        st = FusedTrainStep(m)
        loss = st.forward_backward(b, seed=0)
        torch.cuda.synchronize()
        st.check_status()
        close(loss, rloss, what="loss")
        for k, prm in zip(ENC_KEYS + ["fc.weight", "fc.bias"], st.step_params):
            close(st.grads()[prm], rgrads[k], what=k)
        return
    got = {}
    for checked in (True, False):
        td, bu = build_graph_pair(b.edge_index, b.BU_edge_index, N, batch=b.batch if checked else None)
        q = {k: v.float().to(DEV).contiguous().requires_grad_(True) for k, v in p.items()}
        head = bigcn_encoder(b.x, b.batch, b.rootindex, td, bu, b.num_graphs, [q[k] for k in ENC_KEYS])
        loss = F.nll_loss(F.log_softmax(F.linear(head, q["fc.weight"], q["fc.bias"]), 1), b.y)
        loss.backward()
        torch.cuda.synchronize()
        assert (int(td.status.item()) & _lib.BGCN_STATUS_CROSS_TREE) == (_lib.BGCN_STATUS_CROSS_TREE if checked else 0)
        td.check()
        close(loss, rloss, what="loss")
        for k in ENC_KEYS:
            close(q[k].grad, rgrads[k], what=k)
        got[checked] = [q[k].grad.clone() for k in ENC_KEYS]
    for a, c in zip(got[True], got[False]):   # per-neighbour scales = the general readout backward
        assert torch.allclose(a, c, rtol=1e-5, atol=1e-7 * float(c.abs().max()))
