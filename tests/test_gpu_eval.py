"""GPU parity of the fused evaluation step (FusedTrainStep.evaluate -> bgcn_eval_step): the
reference's test loop body (model/Twitter/BiGCN_Twitter.py:207-222: model.eval(); val_out =
model(Batch_data); val_loss = F.nll_loss(val_out, y); _, val_pred = val_out.max(dim=1);
correct = val_pred.eq(y).sum()) on the device with no host sync.

Tolerance: the fp32 HIP path vs the fp64 oracle, |a - b| <= 1e-4 * max|b| per tensor (log-
probabilities, loss); predictions and the correct count exactly (the argmax of the oracle's
log-probabilities, where no two classes are within the tolerance of each other)."""
import numpy as np
import pytest
import torch

from conftest import golden_batch, golden_params, load_golden
from oracle import bigcn_oracle as O

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL = 1e-4
EVAL_GOLDEN = ["bigcn_eval_mixed.npz", "bigcn_eval_stars_rowdeg.npz", "bigcn_eval_single.npz"]


def close(a, b, tol=TOL, what=""):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    assert a.shape == b.shape, (what, a.shape, b.shape)
    scale = float(b.abs().max()) if b.numel() else 1.0
    err = float((a - b).abs().max()) if b.numel() else 0.0
    assert err <= tol * max(scale, 1e-12), f"{what}: max err {err:.3e} vs scale {scale:.3e}"


def _model(p, F, classes=4, degree_on="col", feat_mode="auto"):
    from bigcn_amd import BiGCN, Net
    m = (BiGCN if classes == 4 else Net)(F, 64, 64).to(DEV)
    m.load_state_dict({k: torch.as_tensor(v).float() for k, v in p.items()})
    m.degree_on = degree_on
    m.feat_mode = feat_mode
    return m


def _check_argmax(pred, correct, rlogp, y):
    """pred must be the oracle's argmax wherever the oracle's top two classes are further
    apart than the log-probabilities' tolerance; where they are within it (a near-tie) any
    class within the tolerance of the maximum is right.  correct counts pred == y."""
    rl = torch.as_tensor(rlogp).double().cpu()
    pred = pred.cpu()
    tol = 2 * TOL * float(rl.abs().max())
    top = rl.max(1).values
    chosen = rl.gather(1, pred.view(-1, 1)).view(-1)
    assert bool(((top - chosen) <= tol).all()), (pred, rl.argmax(1))
    near = (rl >= (top - tol).view(-1, 1)).sum(1) > 1
    want = rl.argmax(1)
    assert torch.equal(pred[~near], want[~near]), (pred, want)
    assert int(correct) == int((pred == y.cpu()).sum())


@pytest.mark.parametrize("mode", ["auto", "dense"])
@pytest.mark.parametrize("name", EVAL_GOLDEN)
def test_eval_step_matches_golden(name, mode):
    from bigcn_amd import FusedTrainStep
    g = load_golden(name)
    assert not bool(g["training"])
    b = golden_batch(g, DEV)
    p = golden_params(g)
    m = _model(p, int(g["in_feats"]), degree_on=str(g["degree_on"]), feat_mode=mode)
    m.train()      # evaluate() runs eval semantics whatever the module's mode
    st = FusedTrainStep(m, tddroprate=0.2, budroprate=0.2, drop_seed=1)
    logp = torch.empty(b.num_graphs, 4, device=DEV)
    loss, correct, pred = st.evaluate(b, logp=logp, pred=True)
    torch.cuda.synchronize()
    st.check_status()
    close(logp, g["logp"], what="logp")
    close(loss, g["loss"], what="loss")
    _check_argmax(pred, correct, g["logp"], b.y)


def _oracle_eval(b, p, degree_on="col"):
    batch = {"x": b.x.double().cpu(), "edge_index": b.edge_index.cpu(), "BU_edge_index": b.BU_edge_index.cpu(),
             "batch": b.batch.cpu(), "rootindex": b.rootindex.cpu(), "y": b.y.cpu()}
    pd = {k: v.double() for k, v in p.items()}
    loss, logp, _ = O.reference_grads(pd, batch, False, None, None, degree_on)
    return loss, logp


@pytest.mark.parametrize("workload", ["twitter15", "weibo_bf16"])
def test_eval_step_full_size_vs_oracle(workload):
    """A full-size evaluation batch (BASELINE workloads: 128 trees, 5000-dim features; the
    Weibo shape with bf16 x and the 2-class head) vs the fp64 oracle in eval mode, with the
    next batch prefetched on the side lane; a second evaluation of the same batch is
    bitwise identical."""
    import bench
    from bigcn_amd import FusedTrainStep
    wl = bench.WORKLOADS[workload]
    pool = bench.make_pool(wl, 0, 2, DEV, (0.0, 0.0))
    classes = wl["classes"]
    p = O.make_params(wl["feats"], 64, 64, classes, seed=31)
    m = _model(p, wl["feats"], classes)
    m.eval()
    st = FusedTrainStep(m)
    loss, correct, pred = st.evaluate(pool[0], next_data=pool[1], pred=True)
    loss1, correct1, pred1 = st.evaluate(pool[1], pred=True)
    loss0, correct0 = st.evaluate(pool[0])
    torch.cuda.synchronize()
    st.check_status()
    assert st.run_report()["status"] == 0
    for b, (ls, cr, pr) in zip(pool, [(loss, correct, pred), (loss1, correct1, pred1)]):
        rloss, rlogp = _oracle_eval(b, p)
        close(ls, rloss, what=f"{workload} loss")
        _check_argmax(pr, cr, rlogp, b.y)
    assert torch.equal(loss, loss0) and torch.equal(correct, correct0)


def test_eval_step_matches_per_op_model_and_training_loss():
    """The evaluation step's log-probabilities equal the drop-in modules' model(data) in
    eval mode (the same kernels, 1e-5), and with dropout off its loss equals the training
    step's forward loss on the same batch bit for bit (the same head and loss order)."""
    import torch.nn.functional as F
    from bigcn_amd import FusedTrainStep
    from bigcn_amd.data import synth_batch, synth_tree_sizes
    rng = np.random.default_rng(41)
    b = synth_batch(rng, synth_tree_sizes(rng, 32, 120), 5000, 4, 0.0, 0.0, device=DEV)
    p = O.make_params(5000, 64, 64, 4, seed=32)
    m = _model(p, 5000)
    m.eval()
    st = FusedTrainStep(m)
    logp = torch.empty(32, 4, device=DEV)
    loss, _ = st.evaluate(b, logp=logp)
    with torch.no_grad():
        ref = m(b)
    close(logp, ref, 1e-5, "logp vs model(data)")
    close(loss, F.nll_loss(ref, b.y), 1e-5, "loss vs F.nll_loss(model(data))")
    tl = st.forward_backward(b)        # eval mode: the training step without dropout
    torch.cuda.synchronize()
    assert torch.equal(tl, loss)
