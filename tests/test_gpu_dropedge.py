"""GPU parity of DropEdge on the device (bgcn_drop_edges; Process/dataset.py:68-90).

The device draw is a counter-based function of (seed, list, edge position); the oracle
(oracle/bigcn_oracle.py drop_edges) restates it, so kept lists are compared bit for
bit.  Against the reference's own Python-random draw the comparison is by property:
exact per-tree counts int(E_t * (1 - rate)), original order, uniform inclusion."""
import numpy as np
import pytest
import torch

from oracle import bigcn_oracle as O
from test_gpu_bigcn import DEV, _oracle, _synth, close
from test_oracle import _forest_edges

pytestmark = pytest.mark.gpu


def _dev(a):
    return torch.as_tensor(np.ascontiguousarray(a)).to(DEV)


@pytest.mark.parametrize("rate", [0.0, 0.2, 0.5, 0.93])
def test_drop_edges_match_oracle(rate):
    from bigcn_amd.ops import drop_edges
    rng = np.random.default_rng(40)
    sizes = [1, 2, 3, 5, 300, 1, 17, 2, 8193, 64, 1, 2]   # single-node trees, 1-edge trees, 8192 edges
    ei, batch = _forest_edges(rng, sizes)
    bu = ei[::-1].copy()
    B = len(sizes)
    seed = 0xABCDEF12345
    td_o, bu_o = drop_edges(_dev(ei), _dev(bu), _dev(batch), B, rate, rate * 0.5, seed)
    assert np.array_equal(td_o.cpu().numpy(), O.drop_edges(ei, batch, B, rate, seed, 0))
    assert np.array_equal(bu_o.cpu().numpy(), O.drop_edges(bu, batch, B, rate * 0.5, seed, 1))
    td_m, bu_m = drop_edges(_dev(ei), _dev(bu), _dev(batch), B, rate, rate * 0.5, seed, masked=True)
    assert np.array_equal(td_m.cpu().numpy(), O.drop_edges(ei, batch, B, rate, seed, 0, masked=True))
    assert np.array_equal(bu_m.cpu().numpy(), O.drop_edges(bu, batch, B, rate * 0.5, seed, 1, masked=True))


def test_drop_edges_single_list_and_empty():
    from bigcn_amd.ops import drop_edges
    rng = np.random.default_rng(41)
    sizes = [4, 9, 1]
    ei, batch = _forest_edges(rng, sizes)
    td_o, bu_o = drop_edges(_dev(ei), None, _dev(batch), 3, 0.2, 0.0, 5)
    assert bu_o is None
    assert np.array_equal(td_o.cpu().numpy(), O.drop_edges(ei, batch, 3, 0.2, 5, 0))
    bu = ei[::-1].copy()
    td_o, bu_o = drop_edges(None, _dev(bu), _dev(batch), 3, 0.0, 0.5, 5)
    assert td_o is None
    assert np.array_equal(bu_o.cpu().numpy(), O.drop_edges(bu, batch, 3, 0.5, 5, 1))
    empty = torch.zeros(2, 0, dtype=torch.int64, device=DEV)
    td_o, _ = drop_edges(empty, None, _dev(np.zeros(3, np.int64)), 1, 0.2)
    assert td_o.shape == (2, 0)


def test_drop_edges_uniform_inclusion():
    """3000 ten-edge trees at rate 0.2: every position kept with probability 0.8, and
    exactly 8 per tree (the reference's random.sample count)."""
    from bigcn_amd.ops import drop_edges
    rng = np.random.default_rng(42)
    sizes = [11] * 3000
    ei, batch = _forest_edges(rng, sizes)
    td, _ = drop_edges(_dev(ei), None, _dev(batch), len(sizes), 0.2, seed=31337)
    td = td.cpu().numpy()
    assert np.all(np.bincount(batch[td[0]], minlength=len(sizes)) == 8)
    posmap = np.full(len(batch), -1)
    posmap[ei[1]] = np.arange(ei.shape[1])            # every child has one parent edge
    kept = np.zeros(ei.shape[1], bool)
    kept[posmap[td[1]]] = True
    freq = kept.reshape(len(sizes), 10).mean(axis=0)
    assert np.all(np.abs(freq - 0.8) < 0.03), freq
    td_m, _ = drop_edges(_dev(ei), None, _dev(batch), len(sizes), 0.2, seed=31337, masked=True)
    loops = (td_m[0] == td_m[1]).view(len(sizes), 10).cpu()
    assert torch.all(loops[:, :8] == 0) and torch.all(loops[:, 8:] == 1)   # kept first, then loops


def test_drop_edges_rejects_ungrouped_edges():
    from bigcn_amd.ops import drop_edges
    rng = np.random.default_rng(43)
    ei, batch = _forest_edges(rng, [6, 7])
    swapped = np.concatenate([ei[:, 5:], ei[:, :5]], axis=1)   # tree 1's edges first
    with pytest.raises(IndexError):
        drop_edges(_dev(swapped), None, _dev(batch), 2, 0.2, seed=1)


@pytest.mark.parametrize("prefetch", [False, True])
def test_train_step_device_dropedge_matches_oracle(prefetch):
    """FusedTrainStep(tddroprate=0.2, budroprate=0.2) on undropped batches equals the
    oracle step on the lists the drop oracle keeps for the step's drop seed."""
    from bigcn_amd import FusedTrainStep
    from test_gpu_train import KEYS, _model
    b1 = _synth(44, 16, 120, droprates=(0.0, 0.0))
    b2 = _synth(45, 16, 120, droprates=(0.0, 0.0))
    p = O.make_params(5000, 64, 64, 4, seed=15)
    m = _model(p)
    m.train(True)
    step = FusedTrainStep(m, tddroprate=0.2, budroprate=0.2, drop_seed=1000)
    seeds = []
    for b, nxt in ((b1, b2 if prefetch else None), (b2, None)):
        loss = step.forward_backward(b, seed=77, next_data=nxt)
        seeds.append(step.last_drop_seed)
        B = b.num_graphs
        batch = b.batch.cpu().numpy()
        td = O.drop_edges(b.edge_index.cpu().numpy(), batch, B, 0.2, step.last_drop_seed, 0)
        bu = O.drop_edges(b.BU_edge_index.cpu().numpy(), batch, B, 0.2, step.last_drop_seed, 1)
        assert td.shape[1] < b.edge_index.size(1)
        from bigcn_amd.ops import keep_words, unpack_keep
        mk = unpack_keep(keep_words(77, b.x.size(0), 5000, DEV), 64 + 5000).cpu()
        ref_b = type("B", (), {})()
        ref_b.x, ref_b.batch, ref_b.rootindex, ref_b.y = b.x, b.batch, b.rootindex, b.y
        ref_b.edge_index, ref_b.BU_edge_index = torch.as_tensor(td), torch.as_tensor(bu)
        _, rloss, rgrads, _ = _oracle(ref_b, p, True, mk[0], mk[1])
        close(loss, rloss, what="loss")
        g = step.grads()
        for k, prm in zip(KEYS, step.step_params):
            close(g[prm], rgrads[k], what=k)
        step.check_status()
    assert seeds == [1000, 1001]


@pytest.mark.parametrize("seed", [0, 987654321, 2**63 + 12345])
def test_keep_words_match_restatement(seed):
    """The in-kernel dropout draw (bgcn_keep_words = what every fused kernel computes from
    (seed, direction, node, word)) equals O.keep_words bit for bit."""
    from bigcn_amd.ops import keep_words
    N, F = 3001, 5000
    got = keep_words(seed, N, F, torch.device("cuda:0")).cpu().numpy().view(np.uint32)
    want = O.keep_words(seed, N, (64 + F + 31) // 32)
    assert got.shape == want.shape
    assert np.array_equal(got, want)
