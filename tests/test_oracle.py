"""CPU tests of the oracle (oracle/bigcn_oracle.py) - closed forms + golden fixtures.

The reference holds no golden vectors for GCNConv / scatter_mean (torch_geometric and
torch_scatter are not vendored and not installed): these hand-derived closed forms are
what pins the restatement (see the oracle header: "parity unpinned" against PyG itself).
"""
import math

import numpy as np
import pytest
import torch

from conftest import golden_batch, golden_params, load_golden
from oracle import bigcn_oracle as O


def test_gcn_norm_two_nodes_target_degree():
    ei = torch.tensor([[0], [1]])
    e, w = O.gcn_norm(ei, None, 2, "col")
    # edge (0->1) first, then loops (0,0), (1,1): deg = [1, 2]
    assert e.tolist() == [[0, 0, 1], [1, 0, 1]]
    assert torch.allclose(w, torch.tensor([1 / math.sqrt(2), 1.0, 0.5]))


def test_gcn_norm_two_nodes_source_degree():
    ei = torch.tensor([[0], [1]])
    _, w = O.gcn_norm(ei, None, 2, "row")
    assert torch.allclose(w, torch.tensor([1 / math.sqrt(2), 0.5, 1.0]))


def test_gcn_norm_replaces_existing_self_loops():
    ei = torch.tensor([[0, 1, 1], [1, 1, 0]])
    e, w = O.gcn_norm(ei, None, 2, "col")
    assert e.tolist() == [[0, 1, 0, 1], [1, 0, 0, 1]]  # (1,1) removed, loops appended
    assert torch.allclose(w, torch.full((4,), 0.5))


def test_gcn_conv_closed_form():
    x = torch.tensor([[1.0], [2.0]])
    w = torch.tensor([[3.0]])
    b = torch.tensor([0.5])
    out = O.gcn_conv(x, torch.tensor([[0], [1]]), w, b)
    assert torch.allclose(out, torch.tensor([[3.5], [3 / math.sqrt(2) + 3.0 + 0.5]]))


def test_scatter_mean_closed_form():
    src = torch.tensor([[1.0], [2.0], [3.0]])
    out = O.scatter_mean(src, torch.tensor([0, 0, 2]))
    assert out.tolist() == [[1.5], [0.0], [3.0]]


def test_root_extend_is_global_gather():
    src = torch.arange(12.0).view(6, 2)
    batch = torch.tensor([0, 0, 0, 1, 1, 1])
    rootindex = torch.tensor([1, 5])
    out = O.root_extend(src, batch, rootindex)
    assert torch.equal(out, src[rootindex[batch]])


def test_x2_is_detached_copy():
    """``x2 = copy.copy(h1)`` (BiGCN_Twitter.py:44) creates a new leaf: no gradient reaches
    conv1 through the root-extended x2."""
    torch.manual_seed(0)
    N, F = 6, 8
    x = torch.rand(N, F)
    ei = torch.tensor([[0, 0, 1, 3], [1, 2, 4, 5]])
    batch = torch.tensor([0, 0, 0, 1, 1, 1])
    rootindex = torch.tensor([0, 3])
    p = O.make_params(F, 64, 64, 4, seed=1)
    q = O.params_requiring_grad(p)
    out = O.direction_forward(q, "TDrumorGCN", x, ei, batch, rootindex)
    out[:, 64:].sum().backward()            # only the x2 half
    assert q["TDrumorGCN.conv1.lin.weight"].grad is None or \
        float(q["TDrumorGCN.conv1.lin.weight"].grad.abs().sum()) == 0.0


def test_dropout_mask_injection_scales_by_two():
    torch.manual_seed(0)
    N, F = 5, 8
    x = torch.rand(N, F)
    ei = torch.tensor([[0, 0, 1], [1, 2, 3]])
    batch = torch.tensor([0, 0, 0, 0, 1])
    rootindex = torch.tensor([0, 4])
    p = O.make_params(F, 64, 64, 4, seed=2)
    st_eval, st_train = {}, {}
    O.direction_forward(p, "TDrumorGCN", x, ei, batch, rootindex, False, stages=st_eval)
    keep = torch.ones(N, 64 + F, dtype=torch.bool)
    O.direction_forward(p, "TDrumorGCN", x, ei, batch, rootindex, True, keep, stages=st_train)
    assert torch.allclose(st_train["TDrumorGCN.a2"], 2 * st_eval["TDrumorGCN.a2"])


def test_head_concat_is_bu_first():
    torch.manual_seed(0)
    N, F = 4, 8
    x = torch.rand(N, F)
    ei = torch.tensor([[0, 0], [1, 2]])
    bei = torch.tensor([[1, 2], [0, 0]])
    batch = torch.zeros(N, dtype=torch.long)
    rootindex = torch.tensor([0])
    p = O.make_params(F, 64, 64, 4, seed=3)
    st = {}
    O.bigcn_forward(p, x, ei, bei, batch, rootindex, stages=st)
    assert torch.equal(st["head_in"][:, :128], st["BUrumorGCN.out"])
    assert torch.equal(st["head_in"][:, 128:], st["TDrumorGCN.out"])


@pytest.mark.parametrize("name", ["bigcn_eval_mixed.npz", "bigcn_train_mixed.npz", "bigcn_train_dropedge.npz",
                                  "bigcn_eval_stars_rowdeg.npz", "bigcn_train_rootmid.npz",
                                  "bigcn_eval_single.npz", "bigcn_train_alldropped.npz"])
def test_oracle_fp32_matches_golden(name):
    """The fp32 oracle (the CPU baseline) reproduces the fp64 golden values."""
    g = load_golden(name)
    b = golden_batch(g)
    p = golden_params(g)
    training = bool(g["training"])
    tdm = torch.as_tensor(g["td_keep"]) if training else None
    bum = torch.as_tensor(g["bu_keep"]) if training else None
    batch = {"x": b.x, "edge_index": b.edge_index, "BU_edge_index": b.BU_edge_index,
             "batch": b.batch, "rootindex": b.rootindex, "y": b.y}
    loss, logp, grads = O.reference_grads(p, batch, training, tdm, bum, str(g["degree_on"]))
    np.testing.assert_allclose(logp.numpy(), g["logp"], rtol=1e-4, atol=1e-5)
    for k, v in grads.items():
        np.testing.assert_allclose(v.numpy(), g["grad:" + k], rtol=1e-4, atol=1e-6, err_msg=k)


def test_train_step_runs_adam_groups():
    g = load_golden("bigcn_train_mixed.npz")
    b = golden_batch(g)
    p = {k: v.clone().requires_grad_(True) for k, v in golden_params(g).items()}
    opt = O.make_optimizer(p)
    assert [grp["lr"] for grp in opt.param_groups] == [5e-4, 1e-4, 1e-4]
    batch = {"x": b.x, "edge_index": b.edge_index, "BU_edge_index": b.BU_edge_index,
             "batch": b.batch, "rootindex": b.rootindex, "y": b.y}
    before = p["fc.weight"].detach().clone()
    loss = O.train_step(p, opt, batch, training=False)
    assert math.isfinite(loss)
    assert not torch.equal(before, p["fc.weight"].detach())
