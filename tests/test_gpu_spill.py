"""Rows of more non-zeros than the 32-entry ELL list: the spill pool.

The reference caps no row (``Process/getTwittergraph.py:16-24``: a post's "idx:count"
pairs all become non-zeros of x).  A row over ``BGCN_SPARSE_CAP`` keeps its first 32
entries in the ELL list and spills the rest to a per-batch pool; conv1, conv2's root
extension (a long ROOT row), dW1 over the CSC of X and the dW2 root columns add the spilled
terms.  Only a batch whose spill exceeds the pool (N * BGCN_SPARSE_SPILL_PER_ROW entries)
falls back to the dense MFMA kernels.

Oracle: ``oracle/bigcn_oracle.py`` (fp64, dense x: it never sees the ELL / spill split);
the in-kernel dropout draw materialised by ``keep_words``.  Tolerances: max-scaled
``|a-b| <= 1e-4 max|b|`` and elementwise ``|a-b| <= 1e-4 (|b| + rms(b))`` per tensor.
"""
import numpy as np
import pytest
import torch

from oracle import bigcn_oracle as O
from test_gpu_bigcn import DEV, _oracle, close, gpu_step
from test_gpu_fullsize import close_elem
from test_gpu_train import KEYS, _model, _unhinted

pytestmark = pytest.mark.gpu


def _long_batch(seed, B=16, mean=150, F=5000, long_rows=(0.03, 33, 300, 5), droprates=(0.2, 0.2)):
    from bigcn_amd.data import synth_batch, synth_tree_sizes
    rng = np.random.default_rng(seed)
    sizes = synth_tree_sizes(rng, B, mean)
    b = synth_batch(rng, sizes, F, 4, *droprates, device=DEV, root_random=True, long_rows=long_rows)
    return b


def _boundary_rows(b, F=5000):
    """Rows of exactly 32, 33, 64 and 65 non-zeros (the ELL edge and one pool round), one of
    them a tree root; the host hints are refreshed."""
    g = torch.Generator().manual_seed(5)
    N = b.x.size(0)
    root = int(b.rootindex[1])
    picks = [root, 3, N // 2, N - 2]
    for r, n in zip(picks, (33, 32, 64, 65)):
        cols = torch.randperm(F, generator=g)[:n]
        row = torch.zeros(F, dtype=b.x.dtype)
        row[cols] = torch.randint(1, 4, (n,), generator=g).to(b.x.dtype)
        b.x[r] = row.to(DEV)
    nnz = (b.x != 0).sum(1)
    b.set_x_nnz_max(int(nnz.max()), int((nnz - 32).clamp_min(0).sum()))
    return b


def _check(got, ref, what):
    close(got, ref, what=what)
    close_elem(got, ref, what=what)


@pytest.mark.parametrize("split", ["0", "1", "4"])
@pytest.mark.parametrize("mode", ["hinted", "auto"])
def test_long_rows_train_step_matches_oracle(mode, split, monkeypatch):
    """The one-call step on a batch with 3 % long rows (33-300 words; five tree roots among
    them) and the ELL-boundary rows: loss, log-probs and all ten gradients vs the oracle,
    under every dW1 form of the tail (XCD slices, one / four waves per column).  hinted: the
    host spill hint selects BGCN_FEAT_SPARSE; auto: the device-gated form."""
    from bigcn_amd import FusedTrainStep
    from bigcn_amd.ops import keep_words, unpack_keep
    monkeypatch.setenv("BGCN_DW1_SPLIT", split)
    b = _boundary_rows(_long_batch(41))
    nnz = (b.x != 0).sum(1)
    assert int(nnz.max()) > 200 and int((nnz[b.rootindex] > 32).sum()) >= 5
    if mode == "auto":
        _unhinted(b)
    p = O.make_params(5000, 64, 64, 4, seed=21)
    m = _model(p, "auto")
    m.train()
    step = FusedTrainStep(m)
    seed = 31337
    logp = torch.empty(b.num_graphs, 4, device=DEV)
    loss = step.forward_backward(b, seed=seed, logp=logp)
    torch.cuda.synchronize()
    step.check_status()
    N = b.x.size(0)
    mk = unpack_keep(keep_words(seed, N, 5000, DEV), 64 + 5000).cpu()
    h1, h2 = (t.cpu() for t in step.saved_activations())
    masks = {d: (h1[:, 64 * k:64 * (k + 1)] > 0, h2[:, 64 * k:64 * (k + 1)] > 0)
             for k, d in enumerate(("TDrumorGCN", "BUrumorGCN"))}
    rlogp, rloss, rgrads, _ = _oracle(b, p, True, mk[0], mk[1], relu_masks=masks)
    _check(logp, rlogp, "logp")
    close(loss, rloss, what="loss")
    g = step.grads()
    for k, prm in zip(KEYS, step.step_params):
        _check(g[prm], rgrads[k], k)


@pytest.mark.parametrize("training", [False, True])
def test_long_rows_encoder_matches_oracle(training):
    """The per-op encoder (bgcn_bigcn_forward / _backward: compaction fused with conv1, the
    CSC built on the side lane) with long rows and long roots."""
    from bigcn_amd.ops import keep_words, unpack_keep
    b = _boundary_rows(_long_batch(42, B=12, mean=120))
    p = O.make_params(5000, 64, 64, 4, seed=22)
    N = b.x.size(0)
    seed = 99
    masks = (None, None)
    if training:
        mk = unpack_keep(keep_words(seed, N, 5000, DEV), 64 + 5000).cpu()
        masks = (mk[0], mk[1])
    logp, loss, grads, head = gpu_step(b, p, training, None, seed=seed, mode="auto")
    rlogp, rloss, rgrads, st = _oracle(b, p, training, *masks)
    close(head, st["head_in"], what="head_in")
    close(logp, rlogp, what="logp")
    for k in p:
        close(grads[k], rgrads[k], what=k)


def test_long_rows_sparse_equals_dense_path():
    """With long rows the sparse path (ELL + spill) and the dense MFMA path compute the same
    step: a Twitter15-sized batch with 1 % of the rows holding 40-300 words."""
    b = _long_batch(43, B=128, mean=256, long_rows=(0.01, 40, 300, 3))
    p = O.make_params(5000, 64, 64, 4, seed=23)
    rs = gpu_step(b, p, True, None, seed=5, mode="auto")
    rd = gpu_step(b, p, True, None, seed=5, mode="dense")
    close(rs[3], rd[3], what="head")
    for k in rs[2]:
        close(rs[2][k], rd[2][k], what=k)


def test_spill_pool_overflow(monkeypatch):
    """A batch whose entries past the ELL exceed the pool (every row dense, F = 512: 480
    spilled per row against 32 per row of capacity): "auto" falls back to the dense kernels
    on the device and still matches the oracle; a forced "sparse" step is invalid - status
    bit 2, check_status raises, the update is skipped."""
    from bigcn_amd import FusedTrainStep
    from bigcn_amd.ops import keep_words, unpack_keep
    from test_gpu_bigcn import _synth
    b = _synth(44, 6, 60, F=512)
    g = torch.Generator().manual_seed(4)
    b.x = torch.rand(b.x.shape, generator=g).to(DEV)
    p = O.make_params(512, 64, 64, 4, seed=24)
    m = _model(p, "auto")
    m.train()
    step = FusedTrainStep(m)
    loss = step.forward_backward(b, seed=8)
    torch.cuda.synchronize()
    step.check_status()
    N = b.x.size(0)
    mk = unpack_keep(keep_words(8, N, 512, DEV), 64 + 512).cpu()
    _, rloss, rgrads, _ = _oracle(b, p, True, mk[0], mk[1])
    close(loss, rloss, what="loss")
    for k, prm in zip(KEYS, step.step_params):
        close(step.grads()[prm], rgrads[k], what=k)
    m2 = _model(p, "sparse")
    m2.train()
    step2 = FusedTrainStep(m2)
    before = {k: v.clone() for k, v in m2.state_dict().items()}
    step2(b, seed=8)
    torch.cuda.synchronize()
    with pytest.raises(ValueError):
        step2.check_status()
    for k, v in m2.state_dict().items():
        assert torch.equal(v, before[k]), k
