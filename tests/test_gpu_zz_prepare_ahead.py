"""GPU parity of the drop-in loop over batches prepared one step ahead (feed.prepare_ahead,
ABI 11 bgcn_bigcn_args.prepared).  In a file of its own, run last: the suite's other files
do not depend on it."""
import torch

import pytest

pytestmark = pytest.mark.gpu


def test_prepare_ahead_matches_inline_preparation():
    """The reference loop body (model(data) -> nll_loss -> zero_grad -> backward -> step)
    over batches prepared one step ahead on a side stream (feed.prepare_ahead: the forward
    takes the prepared graphs / ELL / CSC, no K1 or pass over X of its own) gives the losses,
    gradients and parameters of the same loop preparing inline, to 1e-6 of their scale; a
    batch modified after its preparation is prepared inline again."""
    import torch.nn.functional as F
    from oracle import bigcn_oracle as O
    from test_gpu_bigcn import _synth, close
    from test_gpu_train import _model
    from bigcn_amd.feed import prepare_ahead
    from bigcn_amd.optim import bigcn_adam
    batches = [_synth(90 + k, 24, 150) for k in range(3)]
    p = O.make_params(5000, 64, 64, 4, seed=47)
    runs = []
    for ahead in (False, True):
        m = _model(p)
        m.train()
        opt = bigcn_adam(m)
        seq = [batches[k % 3] for k in range(5)]
        for b in batches:
            b.__dict__.pop("_bgcn_graphs", None)
            b.__dict__.pop("_bgcn_prep", None)
        out, used = [], []
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for k, b in enumerate(prepare_ahead(seq, m) if ahead else seq):
                b.__dict__.pop("_bgcn_graphs", None)
                logp = m(b, seed=500 + k)
                used.append("_bgcn_graphs" not in b.__dict__)
                loss = F.nll_loss(logp, b.y)
                opt.zero_grad()
                loss.backward()
                out.append((loss.detach().clone(), [q.grad.clone() for q in m.parameters()]))
                opt.step()
        torch.cuda.synchronize()
        runs.append((out, [v.clone() for v in m.state_dict().values()], used))
    (a, pa, ua), (b, pb, ub) = runs
    assert not any(ua) and all(ub)
    for (l1, g1), (l2, g2) in zip(a, b):
        close(l1, l2, tol=1e-6, what="loss")
        for x, y in zip(g1, g2):
            close(x, y, tol=1e-6, what="grad")
    for x, y in zip(pa, pb):
        close(x, y, tol=1e-6, what="param")
    # a preparation no longer of its batch is not used
    b0 = batches[0]
    for b in batches:
        b.__dict__.pop("_bgcn_graphs", None)
    it = iter(prepare_ahead([b0], _model(p)))
    bb = next(it)
    bb.x.add_(0.0)             # bumps x's version: the preparation is stale
    m = _model(p)
    m(bb, seed=1)
    assert "_bgcn_graphs" in bb.__dict__


def test_prepare_ahead_reused_slot_is_not_taken():
    """A batch run again after its prepared buffer was reused by a later batch (two slots,
    three batches: batch 0's slot takes batch 2) is prepared inline, and its output is the
    inline output (advisor finding: the stale buffer held another batch's graphs)."""
    from oracle import bigcn_oracle as O
    from test_gpu_bigcn import _synth, close
    from test_gpu_train import _model
    from bigcn_amd.feed import prepare_ahead
    batches = [_synth(120 + k, 16 + 8 * k, 150) for k in range(3)]
    p = O.make_params(5000, 64, 64, 4, seed=48)
    m = _model(p)
    m.eval()
    for b in batches:
        b.__dict__.pop("_bgcn_graphs", None)
        b.__dict__.pop("_bgcn_prep", None)
    seen = [m(b) for b in prepare_ahead(batches, m)]
    b0 = batches[0]
    assert not b0._bgcn_prep.current() and batches[2]._bgcn_prep.current()
    assert "_bgcn_graphs" not in b0.__dict__
    again = m(b0)                              # slot 0 now holds batch 2's preparation
    assert "_bgcn_graphs" in b0.__dict__       # ... so batch 0 was prepared inline
    torch.cuda.synchronize()
    close(again, seen[0], tol=1e-6, what="logp of a batch run again")
