"""CPU tests of the host-side input path (bigcn_amd/data.py).

The RvNN text -> npz conversion is pinned by ``tests/golden/format_trees.npz``, which
``oracle/gen_golden.py`` produced by running the reference's own
``Process/getTwittergraph.py`` (``constructMat`` + ``getfeature``) on the RvNN lines
stored in the fixture."""
import os
import random

import numpy as np
import pytest
import torch

from bigcn_amd import data as D

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "format_trees.npz")


def _fixture():
    with np.load(GOLDEN, allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


def test_rvnn_to_graph_matches_reference_fixture():
    g = _fixture()
    trees = D.parse_rvnn([str(s) for s in g["lines"]])
    for t, eid in enumerate(g["eids"]):
        x, edge, rootfeat, rootindex = D.tree_to_graph(trees[str(eid)])
        n = int(g[f"t{t}_n"])
        assert x.shape == (n, D.VOCAB)
        want = np.zeros((n, D.VOCAB))
        want[g[f"t{t}_x_rows"], g[f"t{t}_x_cols"]] = g[f"t{t}_x_vals"]
        np.testing.assert_array_equal(x, want)
        np.testing.assert_array_equal(edge, g[f"t{t}_edgeindex"])
        assert rootindex == int(g[f"t{t}_rootindex"])
        wroot = np.zeros((1, D.VOCAB))
        wroot[0, g[f"t{t}_rootfeat_cols"]] = g[f"t{t}_rootfeat_vals"]
        np.testing.assert_array_equal(rootfeat, wroot)


def test_edges_sorted_by_parent_then_child():
    rng = np.random.default_rng(0)
    par = D.synth_parents(rng, 40)
    lines = D.tree_to_rvnn_lines("e", par, D.synth_bow(rng, 40, vocab=50), root_pos=7)
    x, edge, _, root = D.tree_to_graph(D.parse_rvnn(lines)["e"], vocab=50)
    keys = edge[0] * 1000 + edge[1]
    assert np.all(np.diff(keys) > 0)
    assert root == 7 and edge.shape == (2, 39)


def test_dropedge_matches_reference_semantics():
    """dataset.py:64-90: TD keeps int(E*(1-r)) sorted positions; BU is the flip of the
    UNdropped TD edges, dropped independently."""
    E = 23
    d = {"x": np.zeros((E + 1, 5)), "root": np.zeros((1, 5)), "rootindex": np.array(0), "y": np.array(2),
         "edgeindex": np.stack([np.zeros(E, np.int64), np.arange(1, E + 1)])}
    s = D.make_sample(d, 0.2, 0.3, random.Random(5))
    assert s.edge_index.shape == (2, int(E * 0.8))
    assert s.BU_edge_index.shape == (2, int(E * 0.7))
    assert torch.all(s.BU_edge_index[1] == 0)                       # flipped: child -> parent
    assert torch.all(s.edge_index[1][1:] > s.edge_index[1][:-1])    # sorted positions
    full = D.make_sample(d)
    assert torch.equal(full.BU_edge_index, full.edge_index.flip(0))


def test_collate_offsets_every_index_key():
    rng = np.random.default_rng(1)
    samples = []
    for n in (3, 5, 1, 4):
        par = D.synth_parents(rng, n)
        tree = D.parse_rvnn(D.tree_to_rvnn_lines("t", par, D.synth_bow(rng, n, vocab=20),
                                                 root_pos=n - 1))["t"]
        samples.append(D.make_sample(D.graph_npz_dict(tree, 1, vocab=20)))
    b = D.collate(samples)
    assert b.num_graphs == 4 and b.x.shape == (13, 20)
    assert b.ptr.tolist() == [0, 3, 8, 9, 13]
    assert b.batch.tolist() == [0] * 3 + [1] * 5 + [2] + [3] * 4
    # rootindex is a GLOBAL node id (the key contains "index")
    assert b.rootindex.tolist() == [2, 3 + 4, 8 + 0, 9 + 3]
    for k in ("edge_index", "BU_edge_index"):
        ei = getattr(b, k)
        assert torch.all(b.batch[ei[0]] == b.batch[ei[1]])          # no edge crosses trees


def test_synth_batch_layout():
    rng = np.random.default_rng(3)
    sizes = D.synth_tree_sizes(rng, 16, 40)
    b = D.synth_batch(rng, sizes, vocab=300, tddroprate=0.2, budroprate=0.2)
    N = int(sizes.sum())
    assert b.x.shape == (N, 300) and b.batch.shape == (N,)
    assert torch.all(b.batch[:-1] <= b.batch[1:])
    assert b.rootindex.tolist() == b.ptr[:-1].tolist()              # root = node 0 of each tree
    nnz = (b.x != 0).sum(1)
    assert int(nnz.min()) >= 1 and int(nnz.max()) <= 32
    td = b.edge_index
    assert torch.all(b.batch[td[0]] == b.batch[td[1]])
    E_full = int((sizes - 1).sum())
    assert td.size(1) == sum(int((n - 1) * 0.8) for n in sizes) < E_full


def test_npz_round_trip_through_dataset(tmp_path):
    rng = np.random.default_rng(4)
    par = D.synth_parents(rng, 9)
    tree = D.parse_rvnn(D.tree_to_rvnn_lines("abc", par, D.synth_bow(rng, 9, vocab=30)))["abc"]
    np.savez(tmp_path / "abc.npz", **D.graph_npz_dict(tree, 3, vocab=30))
    ds = D.BiGraphDataset(["abc"], {"abc": tree}, data_path=str(tmp_path))
    s, tid = ds[0]                                       # (Data, root tweet id): dataset.py:94-99
    assert s.x.shape == (9, 30) and int(s.y) == 3 and int(s.rootindex) == 0
    assert torch.equal(s.BU_edge_index, s.edge_index.flip(0))
    assert tid == "0"                                    # tweetids[rootindex] (graph_npz_dict: ids 0..n-1)
    # the DataLoader form of BiGCN_Twitter.py:168,174: (Batch, [root tweet ids])
    loader = torch.utils.data.DataLoader(ds, batch_size=2, collate_fn=D.collate_pairs)
    b, tids = next(iter(loader))
    assert tids == ["0"] and b.num_graphs == 1 and torch.equal(b.x, s.x)
    assert len(D.BiGraphDataset(["abc"], {"abc": tree}, lower=10, data_path=str(tmp_path))) == 0


def test_long_rows_and_spill_hints():
    """long_rows draws long posts (the reference caps no row, getTwittergraph.py:16-24);
    the batch carries its most non-zeros per row and the entries past the ELL cap (the
    spill pool's fill), bound to its x; collate sums the per-sample spill."""
    rng = np.random.default_rng(5)
    sizes = D.synth_tree_sizes(rng, 12, 50)
    b = D.synth_batch(rng, sizes, vocab=600, long_rows=(0.05, 40, 300, 3))
    nnz = (b.x != 0).sum(1)
    assert int(nnz.max()) > 40
    assert int((nnz[b.rootindex] > 32).sum()) >= 3
    assert b.x_nnz_hint() == int(nnz.max())
    assert b.x_spill_hint() == int((nnz - D.SPARSE_CAP).clamp_min(0).sum())
    b.x[0, 0] += 0.0                                     # an in-place write drops both hints
    assert b.x_nnz_hint() is None and b.x_spill_hint() is None
    b.set_x_nnz_max(int(nnz.max()), int((nnz - D.SPARSE_CAP).clamp_min(0).sum()))
    assert b.x_nnz_hint() == int(nnz.max())
    b.x = b.x.clone()                                   # a replaced x drops both hints
    assert b.x_nnz_hint() is None and b.x_spill_hint() is None
    # per-sample hints through make_sample / collate
    samples = []
    for n in (5, 9):
        x = np.zeros((n, 100), np.float32)
        x[0, :70] = 1.0                                  # one long row per sample: 38 spilled
        d = {"x": x, "edgeindex": np.stack([np.zeros(n - 1, np.int64), np.arange(1, n)]),
             "y": np.int64(1), "root": x[0], "rootindex": np.int64(0)}
        samples.append(D.make_sample(d))
    assert samples[0].x_nnz_max == 70 and samples[0].x_spill == 38
    c = D.collate(samples)
    assert c.x_nnz_hint() == 70 and c.x_spill_hint() == 76


def test_feature_path_policy_from_hints():
    """FusedTrainStep's "auto": BGCN_FEAT_SPARSE (no dense fallback launched) when every row
    fits the ELL or the spill fits the pool; the gated AUTO form without hints."""
    from bigcn_amd import _lib
    from bigcn_amd.train import _step_feat_mode
    b = D.Batch(x=torch.zeros(10, 5000))
    assert _step_feat_mode("auto", b) == _lib.BGCN_FEAT_AUTO          # no hints
    b.set_x_nnz_max(20)
    assert _step_feat_mode("auto", b) == _lib.BGCN_FEAT_SPARSE
    b.set_x_nnz_max(300, 10 * _lib.BGCN_SPARSE_SPILL_PER_ROW)
    assert _step_feat_mode("auto", b) == _lib.BGCN_FEAT_SPARSE
    b.set_x_nnz_max(300, 10 * _lib.BGCN_SPARSE_SPILL_PER_ROW + 1)      # beyond the pool
    assert _step_feat_mode("auto", b) == _lib.BGCN_FEAT_AUTO
    b.set_x_nnz_max(300)                                                # spill unknown
    assert _step_feat_mode("auto", b) == _lib.BGCN_FEAT_AUTO
    assert _step_feat_mode("dense", b) == _lib.BGCN_FEAT_DENSE
    assert _step_feat_mode("sparse", b) == _lib.BGCN_FEAT_SPARSE
