"""GPU parity of the one-call training step (bgcn_train_step via FusedTrainStep).

Oracle: ``oracle/bigcn_oracle.py`` (CPU fp64 restatement of BiGCN_Twitter.py:183-189)
with the in-kernel dropout draw materialised by ``keep_words``; tolerance 1e-4 of
each tensor's max magnitude (fp32 kernels vs fp64 oracle)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import bigcn_oracle as O
from test_gpu_bigcn import DEV, _oracle, _synth, close

pytestmark = pytest.mark.gpu

KEYS = ["TDrumorGCN.conv1.lin.weight", "TDrumorGCN.conv1.bias", "TDrumorGCN.conv2.lin.weight",
        "TDrumorGCN.conv2.bias", "BUrumorGCN.conv1.lin.weight", "BUrumorGCN.conv1.bias",
        "BUrumorGCN.conv2.lin.weight", "BUrumorGCN.conv2.bias", "fc.weight", "fc.bias"]


def _unhinted(b):
    """Drop the batch's host-side nnz hint: "auto" then runs the device-gated fallback
    path instead of BGCN_FEAT_SPARSE."""
    b._x_nnz_of = None
    return b


def _model(p, mode="auto", classes=4):
    from bigcn_amd import BiGCN, Net
    m = (BiGCN if classes == 4 else Net)(p["TDrumorGCN.conv1.lin.weight"].shape[1], 64, 64).to(DEV)
    m.load_state_dict({k: v.float() for k, v in p.items()})
    m.feat_mode = mode
    return m


@pytest.mark.parametrize("mode", ["auto", "auto-hinted", "sparse", "dense"])
@pytest.mark.parametrize("training", [False, True])
def test_train_step_matches_oracle(training, mode):
    """auto: sparse path + device-gated dense fallback; auto-hinted: the batch's host nnz
    hint selects BGCN_FEAT_SPARSE (no fallback launched); sparse: forced; dense."""
    from bigcn_amd import FusedTrainStep
    from bigcn_amd.ops import keep_words, unpack_keep
    b = _synth(31, 16, 150, root_random=True)
    if mode == "auto":
        _unhinted(b)
    mode = "auto" if mode == "auto-hinted" else mode
    p = O.make_params(5000, 64, 64, 4, seed=12)
    m = _model(p, mode)
    m.train(training)
    step = FusedTrainStep(m)
    N = b.x.size(0)
    seed = 424242
    logp = torch.empty(b.num_graphs, 4, device=DEV)
    loss = step.forward_backward(b, seed=seed, logp=logp)
    masks = (None, None)
    if training:
        mk = unpack_keep(keep_words(seed, N, 5000, DEV), 64 + 5000).cpu()
        masks = (mk[0], mk[1])
    rlogp, rloss, rgrads, _ = _oracle(b, p, training, *masks)
    close(logp, rlogp, what="logp")
    close(loss, rloss, what="loss")
    g = step.grads()
    for k, prm in zip(KEYS, step.step_params):
        close(g[prm], rgrads[k], what=k)
    step.check_status()


@pytest.mark.parametrize("mode", ["auto", "dense"])
def test_train_step_matches_autograd_path(mode):
    """The one-call step and the per-op autograd path compute the same step."""
    from bigcn_amd import FusedTrainStep
    b = _synth(32, 64, 256)
    p = O.make_params(5000, 64, 64, 4, seed=13)
    m = _model(p, mode)
    m.train()
    step = FusedTrainStep(m)
    loss = step.forward_backward(b, seed=77)
    fused = {k: v.clone() for k, v in step.grads().items()}
    m.zero_grad()
    ref = F.nll_loss(m(b, seed=77), b.y)
    ref.backward()
    close(loss, ref, what="loss")
    for prm, gv in fused.items():
        close(gv, prm.grad, what=str(tuple(prm.shape)))


def test_train_step_adam_matches_torch_adam():
    """Three full steps: the fused Adam (reference groups, grad_scale path) applied to the
    step's gradients equals torch.optim.Adam (fp32, same groups) fed the same gradients."""
    from bigcn_amd import FusedTrainStep, make_optimizer
    b = _synth(33, 8, 100)
    p = O.make_params(5000, 64, 64, 4, seed=14)
    m = _model(p)
    m.train()
    step = FusedTrainStep(m)
    shadow = _model(p)
    topt = make_optimizer(shadow)
    for it in range(3):
        step.forward_backward(b, seed=1000 + it)
        for sp, prm in zip(shadow.parameters(), m.parameters()):
            sp.grad = step.grads()[prm].clone()
        topt.step()
        step.opt.step(grads=step.bucket.views(), grad_scale=1.0)
    for (k, v), (k2, v2) in zip(m.state_dict().items(), shadow.state_dict().items()):
        assert k == k2
        close(v, v2, tol=1e-6, what=k)


def test_train_step_weibo_head_and_determinism():
    """Net (2 classes): two identical calls are bitwise equal; the step matches the oracle."""
    from bigcn_amd import FusedTrainStep
    b = _synth(34, 32, 200)
    b.y = b.y % 2
    p = O.make_params(5000, 64, 64, 2, seed=15)
    m = _model(p, classes=2)
    m.train()
    step = FusedTrainStep(m)
    l1 = step.forward_backward(b, seed=5)
    g1 = [v.clone() for v in step.grads().values()]
    l2 = step.forward_backward(b, seed=5)
    g2 = list(step.grads().values())
    assert torch.equal(l1, l2)
    for a, c in zip(g1, g2):
        assert torch.equal(a, c)
    m.eval()
    loss = step.forward_backward(b)
    _, rloss, rgrads, _ = _oracle(b, p, False)
    close(loss, rloss, what="loss")
    for k, prm in zip(KEYS, step.step_params):
        close(step.grads()[prm], rgrads[k], what=k)


def test_train_step_reports_bad_inputs():
    from bigcn_amd import FusedTrainStep
    b = _synth(35, 4, 30)
    p = O.make_params(5000, 64, 64, 4, seed=16)
    step = FusedTrainStep(_model(p))
    b.y = b.y.clone()
    b.y[0] = 7
    step.forward_backward(b, seed=1)
    with pytest.raises(IndexError, match="label"):
        step.check_status()
    b = _synth(35, 4, 30)
    b.edge_index = b.edge_index.clone()
    b.edge_index[1, 0] = b.x.size(0) + 5
    step.forward_backward(b, seed=1)
    with pytest.raises(IndexError, match="edge_index"):
        step.check_status()


@pytest.mark.parametrize("mode", ["auto", "sparse", "dense"])
def test_next_batch_prefetch_matches_plain_steps(mode):
    """Preparing the next batch inside a step (side lane) gives bitwise the same losses and
    gradients as preparing every batch inside its own step; a prefetched buffer is only
    used when the next call trains on that very batch."""
    from bigcn_amd import FusedTrainStep
    batches = [_synth(40 + k, 24, 150) for k in range(3)]
    p = O.make_params(5000, 64, 64, 4, seed=17)
    ref, got = [], []
    m1 = _model(p, mode)
    s1 = FusedTrainStep(m1)
    for k, b in enumerate(batches):
        loss = s1.forward_backward(b, seed=k)
        ref.append((loss.clone(), [v.clone() for v in s1.grads().values()]))
    m2 = _model(p, mode)
    s2 = FusedTrainStep(m2)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):                       # non-default stream: real side lane
        for k, b in enumerate(batches):
            nxt = batches[k + 1] if k + 1 < len(batches) else None
            loss = s2.forward_backward(b, seed=k, next_data=nxt)
            got.append((loss.clone(), [v.clone() for v in s2.grads().values()]))
        # a prefetched batch that is not the next one trained on is ignored
        s2.forward_backward(batches[0], seed=9, next_data=batches[1])
        loss = s2.forward_backward(batches[2], seed=2)
        got_last = [v.clone() for v in s2.grads().values()]
    torch.cuda.synchronize()
    for (l1, g1), (l2, g2) in zip(ref, got):
        assert torch.equal(l1, l2)
        for a, c in zip(g1, g2):
            assert torch.equal(a, c)
    for a, c in zip(ref[2][1], got_last):
        assert torch.equal(a, c)
    s2.check_status()


@pytest.mark.parametrize("mode", ["auto", "sparse", "dense"])
def test_weight_images_kept_by_adam_match_derived(mode):
    """Five full steps (step + fused Adam).  With the weight images (W1^T, W2^T, the bf16
    splits of W2[:, :64]) written by the Adam's tile epilogue, the steps after the first
    launch no prologue; losses, gradients and parameters are bitwise those of steps that
    re-derive the images from the weights every time.  A load_state_dict between steps
    (version counters) makes the next step re-derive them; zeroing the kept images shows
    that a current step really reads them."""
    from bigcn_amd import FusedTrainStep
    batches = [_synth(60 + k, 24, 150) for k in range(3)]
    p = O.make_params(5000, 64, 64, 4, seed=18)
    p2 = O.make_params(5000, 64, 64, 4, seed=19)
    runs = []
    for keep in (True, False):
        m = _model(p, mode)
        m.train()
        step = FusedTrainStep(m)
        out, current = [], []
        for it in range(5):
            if it == 3:
                m.load_state_dict({k: v.float() for k, v in p2.items()})
            if not keep:
                step.invalidate_images()
            current.append(step._images_key is not None and step._images_key == step._image_key())
            loss = step(batches[it % 3], seed=100 + it)
            out.append((loss.clone(), [v.clone() for v in step.grads().values()]))
        out.append([v.clone() for v in m.state_dict().values()])
        runs.append((out, current))
    (a, ca), (b, cb) = runs
    assert ca == [False, True, True, False, True]
    assert cb == [False] * 5
    for (l1, g1), (l2, g2) in zip(a[:5], b[:5]):
        assert torch.equal(l1, l2)
        for x, y in zip(g1, g2):
            assert torch.equal(x, y)
    for x, y in zip(a[5], b[5]):
        assert torch.equal(x, y)
    if mode != "dense":   # negative control: a current step reads the kept images
        m = _model(p, mode)
        m.train()
        step = FusedTrainStep(m)
        step(batches[0], seed=100)
        ref = step.forward_backward(batches[1], seed=101).clone()
        step._images.zero_()
        assert not torch.equal(step.forward_backward(batches[1], seed=101), ref)


@pytest.mark.parametrize("mode", ["auto", "dense"])
@pytest.mark.parametrize("training", [False, True])
def test_pheme_768_dense_features(training, mode):
    """PHEME version 2 (BiGCN_Twitter.py:139-140,177-182): x = the [CLS] BERT embedding,
    768 dense signed features per node.  In auto mode every row overflows the sparse
    (ELL) capacity, so the device flag routes the whole step to the dense kernels; the
    relu on the root-extended x (:51) is no longer a no-op."""
    from bigcn_amd import FusedTrainStep
    from bigcn_amd.ops import keep_words, unpack_keep
    b = _synth(33, 16, 90, F=768, root_random=True)
    g = torch.Generator().manual_seed(33)
    b.x = torch.randn(b.x.shape, generator=g).to(DEV)
    p = O.make_params(768, 64, 64, 4, seed=13)
    m = _model(p, mode)
    m.train(training)
    step = FusedTrainStep(m)
    N = b.x.size(0)
    seed = 99
    logp = torch.empty(b.num_graphs, 4, device=DEV)
    loss = step.forward_backward(b, seed=seed, logp=logp)
    masks = (None, None)
    if training:
        mk = unpack_keep(keep_words(seed, N, 768, DEV), 64 + 768).cpu()
        masks = (mk[0], mk[1])
    rlogp, rloss, rgrads, _ = _oracle(b, p, training, *masks)
    close(logp, rlogp, what="logp")
    close(loss, rloss, what="loss")
    gr = step.grads()
    for k, prm in zip(KEYS, step.step_params):
        close(gr[prm], rgrads[k], what=k)
    step.check_status()
    # the module path (per-op autograd encoder) on the same batch
    m.zero_grad()
    out = m(b, seed=seed) if training else m(b)
    close(out, rlogp, what="module logp")


@pytest.mark.parametrize("training", [False, True])
def test_sparse_signed_features(training):
    """Sparse rows with negative values (the auto/ELL path): relu(x_root) must be taken
    per stored value, and negative stored values must not count as dropped columns."""
    from bigcn_amd import FusedTrainStep
    from bigcn_amd.ops import keep_words, unpack_keep
    b = _synth(34, 12, 70, F=2000, root_random=True)
    sign = torch.where(torch.rand(b.x.shape, device=DEV) < 0.5, -1.0, 1.0)
    b.x = b.x * sign
    p = O.make_params(2000, 64, 64, 4, seed=14)
    m = _model(p, "auto")
    m.train(training)
    step = FusedTrainStep(m)
    N = b.x.size(0)
    seed = 7
    logp = torch.empty(b.num_graphs, 4, device=DEV)
    loss = step.forward_backward(b, seed=seed, logp=logp)
    masks = (None, None)
    if training:
        mk = unpack_keep(keep_words(seed, N, 2000, DEV), 64 + 2000).cpu()
        masks = (mk[0], mk[1])
    rlogp, rloss, rgrads, _ = _oracle(b, p, training, *masks)
    close(logp, rlogp, what="logp")
    close(loss, rloss, what="loss")
    gr = step.grads()
    for k, prm in zip(KEYS, step.step_params):
        close(gr[prm], rgrads[k], what=k)


@pytest.mark.parametrize("mode", ["auto", "dense"])
def test_weibo_bf16_features_match_fp32(mode):
    """The Weibo configuration (BASELINE configs[2]: 2-class Net, bf16): node features
    stored as bf16 (bag-of-words counts are exact in bf16), every product accumulated in
    fp32.  Sparse path: the step is bitwise the fp32 step on the same values.  Dense path:
    conv1 and dW1 run on the bf16 MFMA (X exact, the fp32 operand split three ways), so
    the step equals the fp32 step to fp32 rounding (1e-5 of each tensor's max); both match
    the oracle."""
    from bigcn_amd import FusedTrainStep
    from bigcn_amd.ops import keep_words, unpack_keep
    b = _synth(35, 16, 110, root_random=True)
    b.y = b.y % 2                                         # Weibo: 2 classes
    xb = b.x.to(torch.bfloat16)
    assert torch.equal(xb.float(), b.x)                  # counts: exact
    p = O.make_params(5000, 64, 64, 2, seed=16)
    seed = 2024
    outs = []
    for x in (b.x, xb):
        b.x = x
        m = _model(p, mode, classes=2)
        m.train(True)
        step = FusedTrainStep(m)
        logp = torch.empty(b.num_graphs, 2, device=DEV)
        loss = step.forward_backward(b, seed=seed, logp=logp)
        step.check_status()
        outs.append((loss.clone(), logp.clone(), [g.clone() for g in step.grads().values()]))
    (l0, p0, g0), (l1, p1, g1) = outs
    if mode == "auto":
        assert torch.equal(l0, l1) and torch.equal(p0, p1)
        for a, c in zip(g0, g1):
            assert torch.equal(a, c)
    else:
        close(l1, l0, tol=1e-5, what="loss bf16 vs fp32")
        close(p1, p0, tol=1e-5, what="logp bf16 vs fp32")
        for k, a, c in zip(KEYS, g1, g0):
            close(a, c, tol=1e-5, what=f"{k} bf16 vs fp32")
    b.x = xb.float()
    N = b.x.size(0)
    mk = unpack_keep(keep_words(seed, N, 5000, DEV), 64 + 5000).cpu()
    rlogp, rloss, rgrads, _ = _oracle(b, p, True, mk[0], mk[1])
    close(p1, rlogp, what="logp")
    close(l1, rloss, what="loss")
    for k, g in zip(KEYS, g1):
        close(g, rgrads[k], what=k)


@pytest.mark.parametrize("F", [5000, 4996, 4100])
def test_bf16_compaction_any_width_matches_fp32(F):
    """The compaction reads X in 16-byte pieces per lane (eight bf16 or four fp32
    elements): widths whose bf16 row does not end on a 16-byte boundary, non-zeros in the
    last columns and negative zeros (not counted), inside the step and in the next-batch
    preparation, give bitwise the fp32 result."""
    from bigcn_amd import FusedTrainStep
    batches = []
    for k in range(2):
        b = _unhinted(_synth(60 + k, 12, 90, F=F))
        x = b.x.clone()
        x[::3, F - 1] = 3.0
        x[1::4, F - 4] = 1.0
        x[::5, F - 9] = -0.0
        b.x = x
        batches.append(b)
    p = O.make_params(F, 64, 64, 4, seed=18)
    outs = []
    for dt in (torch.float32, torch.bfloat16):
        xs = [b.x for b in batches]
        for b in batches:
            b.x = b.x.to(dt)
        step = FusedTrainStep(_model(p, "auto"))
        res = []
        for k, b in enumerate(batches):
            nxt = batches[k + 1] if k + 1 < len(batches) else None
            loss = step.forward_backward(b, seed=k, next_data=nxt)
            res.append((loss.clone(), [g.clone() for g in step.grads().values()]))
        step.check_status()
        outs.append(res)
        for b, x in zip(batches, xs):
            b.x = x
    for (l0, g0), (l1, g1) in zip(*outs):
        assert torch.equal(l0, l1)
        for a, c in zip(g0, g1):
            assert torch.equal(a, c)


def test_bf16_features_module_path():
    """BiGCN.forward (the per-op autograd encoder) takes bf16 features as well."""
    b = _synth(36, 8, 60)
    p = O.make_params(5000, 64, 64, 4, seed=17)
    m = _model(p)
    m.eval()
    out32 = m(b)
    b.x = b.x.to(torch.bfloat16)
    out16 = m(b)
    assert torch.equal(out32, out16)


def test_sparse_hint_matches_gated_fallback_path():
    """BGCN_FEAT_SPARSE (chosen by the hint) and AUTO (gate on the device) launch
    different kernel sets but compute the same step, bit for bit."""
    from bigcn_amd import FusedTrainStep
    b = _synth(45, 32, 200)
    p = O.make_params(5000, 64, 64, 4, seed=19)
    res = []
    for hinted in (True, False):
        if not hinted:
            _unhinted(b)
        step = FusedTrainStep(_model(p))
        loss = step.forward_backward(b, seed=5)
        res.append((loss.clone(), [v.clone() for v in step.grads().values()]))
        step.check_status()
    assert torch.equal(res[0][0], res[1][0])
    for a, c in zip(res[0][1], res[1][1]):
        assert torch.equal(a, c)


def test_sparse_mode_flags_overfull_rows():
    """feat_mode "sparse" with every row dense (768 non-zeros: far beyond the 32-entry ELL and
    the spill pool): status bit 2, check_status raises; a replaced x invalidates the batch's
    hint (auto then falls back correctly)."""
    from bigcn_amd import FusedTrainStep
    b = _synth(46, 8, 60, F=768)
    g = torch.Generator().manual_seed(46)
    b.x = torch.randn(b.x.shape, generator=g).to(DEV)   # dense rows: every row overflows
    assert b.x_nnz_hint() is None                       # hint bound to the old x
    p = O.make_params(768, 64, 64, 4, seed=21)
    step = FusedTrainStep(_model(p, "sparse"))
    step.forward_backward(b, seed=1)
    with pytest.raises(ValueError):
        step.check_status()
    step = FusedTrainStep(_model(p, "auto"))
    step.forward_backward(b, seed=1)
    step.check_status()


@pytest.mark.parametrize("plan", ["0", "1"])
def test_planned_and_merge_path_aggregation_match_oracle(plan, monkeypatch):
    """Both aggregation forms of the fused step - K1's plans (complete rows per chunk,
    long rows per block, no fixup) and merge-path chunks + fixup (chosen above 2^17
    entries) - against the oracle, on trees with star roots of hundreds of children."""
    from bigcn_amd import FusedTrainStep
    from bigcn_amd.data import synth_batch
    from bigcn_amd.ops import keep_words, unpack_keep
    monkeypatch.setenv("BGCN_SPMM_PLAN", plan)
    rng = np.random.default_rng(47)
    b = synth_batch(rng, [700, 3, 40, 17, 18, 2, 300], 512, 4, 0.2, 0.2, device=DEV)
    p = O.make_params(512, 64, 64, 4, seed=23)
    m = _model(p)
    m.train()
    step = FusedTrainStep(m)
    seed = 31
    logp = torch.empty(b.num_graphs, 4, device=DEV)
    loss = step.forward_backward(b, seed=seed, logp=logp)
    mk = unpack_keep(keep_words(seed, b.x.size(0), 512, DEV), 64 + 512).cpu()
    rlogp, rloss, rgrads, _ = _oracle(b, p, True, mk[0], mk[1])
    close(logp, rlogp, what="logp")
    close(loss, rloss, what="loss")
    g = step.grads()
    for k, prm in zip(KEYS, step.step_params):
        close(g[prm], rgrads[k], what=k)
    step.check_status()


def test_dw1_column_split_matches(monkeypatch):
    """dW1 over the CSC of X by XCD-aware output slices (the default, "0"), with one wave
    per column and with four waves per column: the same gradients up to summation order,
    and every other gradient (the dW2 root columns included) bit for bit."""
    from bigcn_amd import FusedTrainStep
    b = _synth(48, 64, 200)
    p = O.make_params(5000, 64, 64, 4, seed=29)
    res = {}
    for split in ("0", "1", "4"):
        monkeypatch.setenv("BGCN_DW1_SPLIT", split)
        step = FusedTrainStep(_model(p))
        step.forward_backward(b, seed=3)
        g = step.grads()
        res[split] = {k: g[prm].clone() for k, prm in zip(KEYS, step.step_params)}
    for k in KEYS:
        if k.endswith("conv1.lin.weight"):
            close(res["4"][k], res["1"][k], what=k)
            close(res["0"][k], res["1"][k], what=k)
        else:
            assert torch.equal(res["1"][k], res["4"][k]), k
            assert torch.equal(res["1"][k], res["0"][k]), k


@pytest.mark.parametrize("mode", ["auto", "sparse"])
def test_readout_sign_path_matches_readout_bwd(monkeypatch, mode):
    """The readout backward folded into dZ2's aggregation (the readout's H2 sign words and
    per-item positive counts, db2 and the head's weight gradients in the middle launch)
    against the separate k_readout_bwd launch + aggregation of the dH2 tensor
    (BGCN_READOUT_SIGN=0): loss and logp bit for bit (same forward), every gradient within
    1e-5 of its max (each row's neighbour sum is scaled by its tree's dhead / size once
    instead of per neighbour).  Trees of up to ~1500 nodes span several items."""
    from bigcn_amd import FusedTrainStep
    b = _synth(49, 48, 300)
    if mode == "auto":
        _unhinted(b)   # the device-gated dense fallback launched (and gated off)
    p = O.make_params(5000, 64, 64, 4, seed=33)
    res = {}
    for sign in ("1", "0"):
        monkeypatch.setenv("BGCN_READOUT_SIGN", sign)
        m = _model(p, mode)
        m.train()
        step = FusedTrainStep(m)
        logp = torch.empty(b.num_graphs, 4, device=DEV)
        loss = step.forward_backward(b, seed=8, logp=logp)
        step.check_status()
        g = step.grads()
        res[sign] = (loss.clone(), logp.clone(), {k: g[prm].clone() for k, prm in zip(KEYS, step.step_params)})
    assert torch.equal(res["1"][0], res["0"][0])
    assert torch.equal(res["1"][1], res["0"][1])
    for k in KEYS:
        close(res["1"][2][k], res["0"][2][k], tol=1e-5, what=k)


def test_train_step_more_than_four_classes():
    """C = 7: the readout holds every class's head operands (k_readout_items<16>); loss,
    logp and every gradient match the oracle."""
    from bigcn_amd import BiGCN, FusedTrainStep
    b = _synth(50, 24, 300)
    b.y = (b.y * 7 + torch.arange(b.y.numel(), device=DEV)) % 7
    p = O.make_params(5000, 64, 64, 7, seed=34)
    m = BiGCN(5000, 64, 64).to(DEV)
    m.fc = torch.nn.Linear(4 * 64, 7).to(DEV)
    m.load_state_dict({k: v.float() for k, v in p.items()})
    m.eval()
    step = FusedTrainStep(m)
    logp = torch.empty(b.num_graphs, 7, device=DEV)
    loss = step.forward_backward(b, logp=logp)
    rlogp, rloss, rgrads, _ = _oracle(b, p, False)
    close(logp, rlogp, what="logp")
    close(loss, rloss, what="loss")
    g = step.grads()
    for k, prm in zip(KEYS, step.step_params):
        close(g[prm], rgrads[k], what=k)
    step.check_status()


def test_wrong_hint_skips_update():
    """The host nnz hint (collate / synth_batch) is bound to x's identity and version
    counter, so an in-place edit drops it.  A hint that is wrong anyway (set by hand after
    an edit that overfills the sparse path) is caught on the device: the step flags status
    bit 2, the fused Adam skips the update (parameters and moments unchanged, no host sync)
    and check_status() raises.  (One long row fits the spill pool; every row at 100 words -
    68 spilled per row against 32 per row of pool - does not.)"""
    from bigcn_amd import FusedTrainStep
    b = _synth(47, 8, 60)
    assert b.x_nnz_hint() is not None
    b.x[:, :100] = 1.0                                  # beyond ELL + spill pool, in place
    assert b.x_nnz_hint() is None and b.x_spill_hint() is None
    b.set_x_nnz_max(5, 0)                               # a wrong hint
    p = O.make_params(5000, 64, 64, 4, seed=22)
    m = _model(p)
    m.train()
    step = FusedTrainStep(m)
    before = {k: v.clone() for k, v in m.state_dict().items()}
    step(b, seed=3)
    torch.cuda.synchronize()
    assert float(step.bucket.flag) != 0.0
    for k, v in m.state_dict().items():
        assert torch.equal(v, before[k]), k
    for mom in step.opt.state.values():
        assert not mom[0].any() and not mom[1].any()
    with pytest.raises(ValueError, match="non-zeros"):
        step.check_status()
    # a valid batch afterwards trains again (flag rewritten by the step)
    b2 = _synth(48, 8, 60)
    step(b2, seed=4)
    torch.cuda.synchronize()
    step.check_status()
    assert float(step.bucket.flag) == 0.0
    assert any(not torch.equal(v, before[k]) for k, v in m.state_dict().items())


def test_fused_adam_follows_lr_changes():
    """FusedAdam reads param_groups[i]['lr'] every step (an LR scheduler works as with
    torch.optim.Adam): three steps with a StepLR-like halving match torch Adam."""
    from bigcn_amd import FusedTrainStep, make_optimizer
    b = _synth(49, 8, 100)
    p = O.make_params(5000, 64, 64, 4, seed=23)
    m = _model(p)
    m.train()
    step = FusedTrainStep(m)
    shadow = _model(p)
    topt = make_optimizer(shadow)
    for it in range(3):
        step.forward_backward(b, seed=2000 + it)
        for sp, prm in zip(shadow.parameters(), m.parameters()):
            sp.grad = step.grads()[prm].clone()
        topt.step()
        step.opt.step(grads=step.bucket.views(), grad_scale=1.0)
        for g, tg in zip(step.opt.param_groups, topt.param_groups):
            g["lr"] *= 0.5
            tg["lr"] *= 0.5
    for (k, v), (k2, v2) in zip(m.state_dict().items(), shadow.state_dict().items()):
        close(v, v2, tol=1e-6, what=k)


def test_row_degree_model_trains_and_evaluates_consistently():
    """degree_on is model-wide: FusedTrainStep and model(data) use the same (PyG 1.3.2
    source-degree) normalisation, and both match the oracle's row convention."""
    from bigcn_amd import FusedTrainStep
    b = _synth(50, 16, 120, root_random=True)
    p = O.make_params(5000, 64, 64, 4, seed=24)
    m = _model(p)
    m.degree_on = "row"
    m.eval()
    step = FusedTrainStep(m)
    loss = step.forward_backward(b)
    _, rloss, rgrads, _ = _oracle(b, p, False, degree_on="row")
    close(loss, rloss, what="loss")
    for k, prm in zip(KEYS, step.step_params):
        close(step.grads()[prm], rgrads[k], what=k)
    m.zero_grad()
    ref = F.nll_loss(m(b), b.y)
    close(ref, rloss, what="model(data) loss")
    ref.backward()
    for k, prm in zip(KEYS, step.step_params):
        close(prm.grad, rgrads[k], what="autograd " + k)
    with pytest.raises(ValueError):
        FusedTrainStep(m, degree_on="col")


@pytest.mark.parametrize("split", ["0", "1", "4"])
def test_deferred_dw1_matches_one_call(split, monkeypatch):
    """defer_dw1 (the data-parallel overlap: everything but the conv1 weight gradients,
    then bgcn_train_step_dw1) writes the same bits as the one-call step, with the next
    batch's preparation running beside both, under every dW1 form of the tail."""
    from bigcn_amd import FusedTrainStep
    monkeypatch.setenv("BGCN_DW1_SPLIT", split)
    b0, b1 = _synth(61, 32, 200), _synth(62, 32, 200)
    p = O.make_params(5000, 64, 64, 4, seed=41)
    res = []
    for defer in (False, True):
        step = FusedTrainStep(_model(p), tddroprate=0.2, budroprate=0.2, drop_seed=5)
        step.model.train()
        step.forward_backward(b0, seed=3, next_data=b1, defer_dw1=defer)
        if defer:
            step.finish_dw1()
            with pytest.raises(RuntimeError):
                step.finish_dw1()
        loss = step.forward_backward(b1, seed=4, defer_dw1=defer)
        if defer:
            step.finish_dw1()
        torch.cuda.synchronize()
        step.check_status()
        res.append((loss.clone(), [step.grads()[prm].clone() for prm in step.step_params]))
    assert torch.equal(res[0][0], res[1][0])
    for k, a, c in zip(KEYS, res[0][1], res[1][1]):
        assert torch.equal(a, c), k


@pytest.mark.parametrize("mode,classes,split", [("auto", 4, "0"), ("sparse", 2, "0"), ("dense", 4, "0"),
                                                ("auto", 4, "1")])
def test_optimizer_inside_step_matches_separate_launch(mode, classes, split, monkeypatch):
    """The single-process step with the Adam update inside its last launch
    (bgcn_step_args.adam) leaves bitwise the parameters, moments, weight images and losses
    of the step followed by its own bgcn_adam_step, over six steps with the next batch
    prepared beside each; an invalid step (bad label, step 3) is skipped and counted in
    both.  dense / BGCN_DW1_SPLIT=1: the library falls back to the separate launch."""
    from bigcn_amd import FusedTrainStep
    monkeypatch.setenv("BGCN_DW1_SPLIT", split)
    batches = [_synth(70 + k, 24, 150) for k in range(3)]
    for b in batches:
        b.y = b.y % classes
    bad = _synth(73, 24, 150)
    bad.y = bad.y.clone() % classes
    bad.y[2] = 9
    p = O.make_params(5000, 64, 64, classes, seed=43)
    runs = []
    for fuse in (True, False):
        m = _model(p, mode, classes)
        m.train()
        step = FusedTrainStep(m, tddroprate=0.2, budroprate=0.2, drop_seed=11, fuse_optimizer=fuse)
        seq = [batches[0], batches[1], bad, batches[2], batches[0], batches[1]]
        losses = []
        for it, b in enumerate(seq):
            nxt = seq[it + 1] if it + 1 < len(seq) else None
            losses.append(step(b, seed=300 + it, next_data=nxt).clone())
        torch.cuda.synchronize()
        runs.append((losses, [v.clone() for v in m.state_dict().values()],
                     [t.clone() for mv in step.opt.state.values() for t in mv],
                     step._images.clone(), int(step.skipped), step.opt.step_count))
    a, b = runs
    for x, y in zip(a[0], b[0]):
        assert torch.equal(x, y)
    for k, (x, y) in enumerate(zip(a[1], b[1])):
        assert torch.equal(x, y), k
    for x, y in zip(a[2], b[2]):
        assert torch.equal(x, y)
    assert torch.equal(a[3], b[3])
    assert a[4] == b[4] == 1
    assert a[5] == b[5] == 6

