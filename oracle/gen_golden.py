"""Generate the committed golden fixtures under tests/golden/ (TEST INFRASTRUCTURE).

Run in the build container (needs /root/reference; never run on the GPU box):

    python oracle/gen_golden.py

1. ``format_trees.npz`` - PINNED BY THE REFERENCE ITSELF: synthetic trees written as RvNN
   text lines, parsed the way ``Process/getTwittergraph.py:main`` does (``:77-84``) and
   turned into graphs by the reference's own ``constructMat`` / ``getfeature``
   (``Process/getTwittergraph.py:26-72``), imported from /root/reference.  The
   build's ``bigcn_amd.data.tree_to_graph`` must reproduce x / edgeindex / rootindex /
   rootfeat exactly.
2. ``bigcn_*.npz`` - the BiGCN step computed by the CPU oracle (``oracle/bigcn_oracle.py``,
   fp64 and fp32) on small fixed batches: inputs, parameters, intermediate stages,
   log-probs, loss and every parameter gradient, in eval mode and in training mode with
   an injected dropout mask, for both gcn_norm degree conventions.  torch_geometric is
   not installed here, so these are "parity unpinned" against PyG itself (see
   oracle/bigcn_oracle.py).
Fixtures store only data (numpy arrays, no pickles); X is stored sparse.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

from bigcn_amd import data as D  # noqa: E402
from oracle import bigcn_oracle as O  # noqa: E402

REF = "/root/reference"
OUT = os.path.join(ROOT, "tests", "golden")


def _ref_graph_fns():
    sys.path.insert(0, REF)
    from Process import getTwittergraph as G  # the reference's own preprocessing
    return G.constructMat, G.getfeature


def _ref_parse(lines):
    """The tree dictionary ``getTwittergraph.main`` builds from the RvNN lines
    (``Process/getTwittergraph.py:77-84``): tree id -> {child index: {parent (str, "None"
    for the root), max_degree, maxL, vec (the "word:count" string)}}."""
    trees = {}
    for raw in lines:
        fields = raw.rstrip().split("\t")
        node = {"parent": fields[1], "max_degree": int(fields[3]), "maxL": int(fields[4]), "vec": fields[5]}
        trees.setdefault(fields[0], {})[int(fields[2])] = node
    return trees


def format_fixture():
    constructMat, getfeature = _ref_graph_fns()
    rng = np.random.default_rng(20250205)
    shapes = [("chain", 6), ("star", 9), ("random", 25), ("pair", 2), ("rootmid", 12), ("random", 40)]
    out = {}
    lines_all = []
    for t, (kind, n) in enumerate(shapes):
        if kind == "chain":
            par = np.arange(-1, n - 1)
        elif kind == "star":
            par = np.array([-1] + [0] * (n - 1))
        else:
            par = D.synth_parents(rng, n)
        bow = D.synth_bow(rng, n)
        eid = f"t{t}"
        lines = D.tree_to_rvnn_lines(eid, par, bow, root_pos=5 if kind == "rootmid" else 0)
        lines_all += lines
        tree = _ref_parse(lines)[eid]
        x_word, x_index, edgematrix, rootfeat, rootindex = constructMat(tree)
        x = getfeature(x_word, x_index)
        r, c = np.nonzero(x)
        out[f"{eid}_x_rows"], out[f"{eid}_x_cols"], out[f"{eid}_x_vals"] = r, c, x[r, c]
        out[f"{eid}_n"] = np.array(x.shape[0])
        out[f"{eid}_edgeindex"] = np.array(edgematrix, dtype=np.int64).reshape(2, -1)
        rr = np.nonzero(rootfeat[0])[0]
        out[f"{eid}_rootfeat_cols"], out[f"{eid}_rootfeat_vals"] = rr, rootfeat[0, rr]
        out[f"{eid}_rootindex"] = np.array(rootindex)
    out["lines"] = np.array(lines_all)
    out["eids"] = np.array([f"t{t}" for t in range(len(shapes))])
    np.savez_compressed(os.path.join(OUT, "format_trees.npz"), **out)
    print("format_trees.npz:", len(shapes), "trees")


def _batch(rng, kind, F, droprates=(0.0, 0.0)):
    """Small collated batches covering the edge cases of SURVEY.md 4."""
    samples = []
    if kind == "mixed":
        specs = [("chain", 5), ("star", 7), ("random", 11), ("pair", 2), ("random", 9)]
    elif kind == "single":
        specs = [("random", 13)]
    elif kind == "stars":
        specs = [("star", 40), ("star", 3), ("chain", 4)]
    elif kind == "rootmid":
        specs = [("random", 8), ("random", 10), ("chain", 6)]
    else:
        raise ValueError(kind)
    for t, (shape, n) in enumerate(specs):
        if shape == "chain":
            par = np.arange(-1, n - 1)
        elif shape == "star":
            par = np.array([-1] + [0] * (n - 1))
        else:
            par = D.synth_parents(rng, n)
        bow = D.synth_bow(rng, n, vocab=F, mean_extra=3.0)
        lines = D.tree_to_rvnn_lines(f"b{t}", par, bow, root_pos=(n // 2 if kind == "rootmid" else 0))
        tree = D.parse_rvnn(lines)[f"b{t}"]
        d = D.graph_npz_dict(tree, y=int(rng.integers(0, 4)), vocab=F)
        import random as _r
        samples.append(D.make_sample(d, *droprates, rnd=_r.Random(1000 + t)))
    return D.collate(samples)


def model_fixture(name, kind, F, training, degree_on, droprates=(0.0, 0.0), seed=0):
    rng = np.random.default_rng(7 + seed)
    b = _batch(rng, kind, F, droprates)
    p = O.make_params(F, 64, 64, 4, seed=seed, dtype=torch.float64)
    N = b.x.size(0)
    g = torch.Generator().manual_seed(99 + seed)
    td_mask = torch.rand(N, 64 + F, generator=g) < 0.5 if training else None
    bu_mask = torch.rand(N, 64 + F, generator=g) < 0.5 if training else None
    batch = {"x": b.x.double(), "edge_index": b.edge_index, "BU_edge_index": b.BU_edge_index,
             "batch": b.batch, "rootindex": b.rootindex, "y": b.y}
    stages = {}
    loss, logp, grads = O.reference_grads(p, batch, training, td_mask, bu_mask, degree_on, stages)
    out = {}
    xr, xc = torch.nonzero(b.x, as_tuple=True)
    out["x_rows"], out["x_cols"], out["x_vals"] = xr.numpy(), xc.numpy(), b.x[xr, xc].numpy()
    out["num_nodes"], out["in_feats"], out["num_graphs"] = np.array(N), np.array(F), np.array(b.num_graphs)
    for k in ("edge_index", "BU_edge_index", "batch", "rootindex", "y"):
        out[k] = getattr(b, k).numpy()
    out["training"], out["degree_on"] = np.array(int(training)), np.array(degree_on)
    if training:
        out["td_keep"] = td_mask.numpy()
        out["bu_keep"] = bu_mask.numpy()
    for k, v in p.items():
        out["param:" + k] = v.float().numpy()   # fp32 parameters (what the GPU path uses)
    # recompute the expected values from the fp32-rounded parameters in fp64
    p32 = {k: v.float().double() for k, v in p.items()}
    stages = {}
    loss, logp, grads = O.reference_grads(p32, batch, training, td_mask, bu_mask, degree_on, stages)
    out["logp"], out["loss"] = logp.numpy(), loss.numpy()
    for k, v in stages.items():
        out["stage:" + k] = v.numpy()
    for k, v in grads.items():
        out["grad:" + k] = v.numpy()
    np.savez_compressed(os.path.join(OUT, f"bigcn_{name}.npz"), **out)
    print(f"bigcn_{name}.npz: N={N} F={F} E={b.edge_index.size(1)}/{b.BU_edge_index.size(1)} training={training}")


def main():
    os.makedirs(OUT, exist_ok=True)
    format_fixture()
    model_fixture("eval_mixed", "mixed", 96, False, "col")
    model_fixture("train_mixed", "mixed", 96, True, "col", seed=1)
    model_fixture("train_dropedge", "mixed", 100, True, "col", droprates=(0.2, 0.2), seed=2)
    model_fixture("eval_stars_rowdeg", "stars", 64, False, "row", seed=3)
    model_fixture("train_rootmid", "rootmid", 132, True, "col", seed=4)
    model_fixture("eval_single", "single", 40, False, "col", seed=5)
    model_fixture("train_alldropped", "mixed", 96, True, "col", droprates=(0.99, 0.99), seed=6)


if __name__ == "__main__":
    main()
