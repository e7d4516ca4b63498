"""Host-side input path of the BiGCN hot path: tree formats, dataset, collation.

* RvNN tree text (``data/<name>/data.TD_RvNN.vol_5000.txt``, one line per post:
  ``eid \\t indexP \\t indexC \\t max_degree \\t maxL \\t idx:cnt ...``) as parsed by
  ``Process/process.py:7-19`` / ``Process/getTwittergraph.py:75-86``.
* Per-tree ``.npz`` (``x, root, edgeindex, rootindex, y`` + the ``cls, tweetids`` keys
  ``BiGraphDataset`` reads) as written by ``Process/getTwittergraph.py:26-72,128``:
  node i = indexC - 1, ``edgeindex`` sorted by (parent, child), ``rootindex`` = root indexC - 1.
* :class:`BiGraphDataset` - ``Process/dataset.py:45-99``: DropEdge sampled independently
  for TD and BU (``random.sample`` + sort), BU = flipped *undropped* TD edges.
* :func:`collate` - PyG ``Batch.from_data_list``: concatenate, offset every key that
  contains ``"index"`` (``edge_index``, ``BU_edge_index``, ``rootindex``) by the running
  node count, build ``batch`` and ``ptr``.
* Synthetic generators (the real trees are absent: ``.MISSING_LARGE_BLOBS:4-6``) with the
  shape of SURVEY.md 8(d): node k >= 1 attaches to the root with p = 0.5, otherwise to a
  uniform earlier non-root node; rows are bag-of-words with 1 + Poisson(11) distinct
  vocabulary ids and counts in {1, 2, 3}.
"""
from __future__ import annotations

import os
import random
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

VOCAB = 5000


# ----------------------------------------------------------------------------- synthetic trees
def synth_parents(rng: np.random.Generator, n: int, root_p: float = 0.5) -> np.ndarray:
    """parents[k] for k in [0, n); parents[0] = -1 (root)."""
    par = np.full(n, -1, dtype=np.int64)
    if n > 1:
        k = np.arange(1, n)
        to_root = rng.random(n - 1) < root_p
        other = (rng.random(n - 1) * np.maximum(k - 1, 1)).astype(np.int64) + 1
        par[1:] = np.where(to_root | (k == 1), 0, np.minimum(other, k - 1))
    return par


def synth_bow(rng: np.random.Generator, n: int, vocab: int = VOCAB, mean_extra: float = 11.0):
    """List of (indices, counts) per node: 1 + Poisson(mean_extra) distinct ids in [0, vocab)."""
    out = []
    nnz = np.minimum(1 + rng.poisson(mean_extra, size=n), vocab)
    for i in range(n):
        idx = np.sort(rng.choice(vocab, size=int(nnz[i]), replace=False))
        cnt = rng.integers(1, 4, size=idx.size).astype(np.float64)
        out.append((idx, cnt))
    return out


def synth_tree_sizes(rng: np.random.Generator, count: int, mean: float, sigma: float = 0.8,
                     lo: int = 2, hi: int = 8192) -> np.ndarray:
    """LogNormal(sigma) tree sizes scaled to ``mean`` and clamped to [lo, hi]."""
    mu = np.log(mean) - sigma * sigma / 2
    return np.clip(np.round(rng.lognormal(mu, sigma, size=count)), lo, hi).astype(np.int64)


def tree_to_rvnn_lines(eid: str, parents: np.ndarray, bow, root_pos: int = 0) -> List[str]:
    """RvNN text lines for one tree.  ``root_pos`` permutes ids so the root gets indexC
    root_pos + 1 (exercises a non-zero ``rootindex``)."""
    n = len(parents)
    perm = np.arange(n)
    if root_pos:
        perm[[0, root_pos]] = perm[[root_pos, 0]]  # node k gets id perm[k]
    lines = []
    for k in range(n):
        idxc = int(perm[k]) + 1
        p = "None" if parents[k] < 0 else str(int(perm[parents[k]]) + 1)
        vec = " ".join(f"{int(i)}:{int(c)}" for i, c in zip(*bow[k]))
        lines.append(f"{eid}\t{p}\t{idxc}\t1\t1\t{vec}")
    return lines


def parse_rvnn(lines: Sequence[str]) -> Dict[str, dict]:
    """``loadTree`` (``Process/process.py:9-19``): treeDic[eid][indexC] = {parent, vec, ...}."""
    tree: Dict[str, dict] = {}
    for line in lines:
        line = line.rstrip()
        f = line.split("\t")
        eid, indexP, indexC = f[0], f[1], int(f[2])
        tree.setdefault(eid, {})[indexC] = {"parent": indexP, "max_degree": int(f[3]),
                                            "maxL": int(f[4]), "vec": f[5]}
    return tree


def tree_to_graph(tree: dict, vocab: int = VOCAB):
    """Restates ``constructMat`` + ``getfeature`` (``Process/getTwittergraph.py:26-72``)
    vectorised: returns (x [n, vocab] float64, edgeindex [2, n-1], rootfeat [1, vocab],
    rootindex)."""
    n = len(tree)
    x = np.zeros((n, vocab))
    rows, cols = [], []
    rootindex, rootfeat = None, np.zeros((1, vocab))
    for c in sorted(tree):
        node = tree[c]
        idx, cnt = [], []
        for pair in node["vec"].split(" "):
            if not pair:
                continue
            i, v = pair.split(":")
            if int(i) <= vocab:                      # str2matrix keeps index <= 5000
                idx.append(int(i)); cnt.append(float(v))
        if idx:
            x[c - 1, np.array(idx)] = np.array(cnt)
        if node["parent"] == "None":
            rootindex = c - 1
            if idx:
                rootfeat[0, np.array(idx)] = np.array(cnt)
        else:
            rows.append(int(node["parent"]) - 1)
            cols.append(c - 1)
    order = np.lexsort((np.array(cols, dtype=np.int64), np.array(rows, dtype=np.int64)))
    edge = np.array([np.array(rows, dtype=np.int64)[order], np.array(cols, dtype=np.int64)[order]])
    if edge.size == 0:
        edge = np.zeros((2, 0), dtype=np.int64)
    return x, edge, rootfeat, rootindex


def graph_npz_dict(tree: dict, y: int, vocab: int = VOCAB) -> dict:
    x, edge, rootfeat, rootindex = tree_to_graph(tree, vocab)
    n = x.shape[0]
    return {"x": x, "root": rootfeat, "edgeindex": edge, "rootindex": np.array(rootindex),
            "y": np.array(y), "cls": np.zeros((n, 1)), "tweetids": np.arange(n).astype(str)}


SPARSE_CAP = 32   # = libbgcn's BGCN_SPARSE_CAP (ELL entries per row; the rest spill)


# ----------------------------------------------------------------------------- dataset
@dataclass
class Sample:
    x: torch.Tensor
    edge_index: torch.Tensor
    BU_edge_index: torch.Tensor
    y: torch.Tensor
    root: torch.Tensor
    rootindex: torch.Tensor
    cls: Optional[torch.Tensor] = None
    tweetids: Optional[torch.Tensor] = None
    x_nnz_max: Optional[int] = None     # most non-zeros in one row of x (feature-path hint)
    x_spill: Optional[int] = None       # sum over rows of max(nnz - BGCN_SPARSE_CAP, 0)


def _drop(row: np.ndarray, col: np.ndarray, rate: float, rnd: random.Random):
    """``random.sample(range(length), int(length * (1 - rate)))`` then sorted (``dataset.py:69-76``)."""
    length = len(row)
    pos = sorted(rnd.sample(range(length), int(length * (1 - rate))))
    return row[pos], col[pos]


def make_sample(d: dict, tddroprate: float = 0.0, budroprate: float = 0.0,
                rnd: Optional[random.Random] = None) -> Sample:
    """``BiGraphDataset.__getitem__`` (``Process/dataset.py:64-99``) on one npz dict."""
    rnd = rnd or random
    edge = np.asarray(d["edgeindex"], dtype=np.int64).reshape(2, -1)
    row, col = edge[0], edge[1]
    if tddroprate > 0:
        row, col = _drop(row, col, tddroprate, rnd)
    burow, bucol = edge[1], edge[0]                    # BU = flip of the UNdropped TD edges
    if budroprate > 0:
        burow, bucol = _drop(burow, bucol, budroprate, rnd)
    tweetids = None
    if "tweetids" in d:
        tweetids = torch.tensor([int(v) for v in d["tweetids"]], dtype=torch.int64)
    x = torch.tensor(d["x"], dtype=torch.float32)
    nnz = (x != 0).sum(1)
    return Sample(
        x=x,
        x_nnz_max=int(nnz.max()) if x.numel() else 0,
        x_spill=int((nnz - SPARSE_CAP).clamp_min(0).sum()) if x.numel() else 0,
        edge_index=torch.as_tensor(np.stack([row, col]), dtype=torch.int64),
        BU_edge_index=torch.as_tensor(np.stack([burow, bucol]), dtype=torch.int64),
        y=torch.tensor([int(d["y"])], dtype=torch.int64),
        root=torch.as_tensor(np.asarray(d["root"]), dtype=torch.int64),
        rootindex=torch.tensor([int(d["rootindex"])], dtype=torch.int64),
        cls=torch.tensor(np.asarray(d["cls"]), dtype=torch.float32) if "cls" in d else None,
        tweetids=tweetids)


class BiGraphDataset(torch.utils.data.Dataset):
    """``Process/dataset.py:45-99`` over ``<data_path>/<eid>.npz`` (size filter ``lower=2``,
    ``upper=100000`` against ``treeDic``).  npz files are read with ``allow_pickle=False``.

    An item is ``(sample, root tweet id)`` as the reference returns ``(Data(...),
    data['tweetids'][rootindex])`` (``dataset.py:94-99``); a DataLoader with
    ``collate_fn=collate_pairs`` then yields ``(Batch, [root tweet ids])`` like the loop at
    ``BiGCN_Twitter.py:174`` unpacks (``for Batch_data, tweetid in train_loader``).  The
    root tweet id is None for npz files without ``tweetids`` (the Twitter/Weibo
    preprocessors write none, ``getTwittergraph.py:128``).  The host-fed fast path
    (compacted features, one buffer per batch) is :mod:`bigcn_amd.feed`."""

    def __init__(self, fold_x, treeDic=None, lower=2, upper=100000, tddroprate=0.0, budroprate=0.0,
                 data_path=os.path.join("..", "..", "data", "Weibograph")):
        if treeDic is not None:
            fold_x = [i for i in fold_x if i in treeDic and lower <= len(treeDic[i]) <= upper]
        self.fold_x = list(fold_x)
        self.data_path = data_path
        self.tddroprate, self.budroprate = tddroprate, budroprate

    def __len__(self):
        return len(self.fold_x)

    def __getitem__(self, index):
        eid = self.fold_x[index]
        with np.load(os.path.join(self.data_path, eid + ".npz"), allow_pickle=False) as f:
            d = {k: f[k] for k in f.files}
        root_tid = None
        if "tweetids" in d:
            root_tid = d["tweetids"][int(d["rootindex"])]
        return make_sample(d, self.tddroprate, self.budroprate), root_tid


# ----------------------------------------------------------------------------- batch
class Batch:
    """PyG ``Batch`` stand-in carrying exactly the keys the BiGCN path reads."""

    def __init__(self, **kw):
        self.__dict__.update(kw)

    @property
    def num_nodes(self) -> int:
        return int(self.x.size(0))

    def to(self, device, non_blocking: bool = False):
        hinted = self._hint_ok()
        for k, v in list(self.__dict__.items()):
            if isinstance(v, torch.Tensor) and not k.startswith("_"):
                self.__dict__[k] = v.to(device, non_blocking=non_blocking)
        self.__dict__.pop("_bgcn_graphs", None)
        if hinted:
            self._x_nnz_of, self._x_nnz_ver = self.x, self.x._version
        return self

    # Host-side feature-path hints: the most non-zeros in one row of x and the entries past
    # the ELL cap summed over the rows (what the spill pool must hold).  They are bound to
    # the x tensor they were computed for (its identity and version counter) and ignored
    # once x is replaced or modified in place.
    def set_x_nnz_max(self, n: int, spill: Optional[int] = None) -> None:
        self.x_nnz_max = int(n)
        self.x_spill = None if spill is None else int(spill)
        self._x_nnz_of, self._x_nnz_ver = self.x, self.x._version

    def _hint_ok(self) -> bool:
        x = self.__dict__.get("x")
        return (x is not None and self.__dict__.get("_x_nnz_of") is x
                and self.__dict__.get("_x_nnz_ver") == x._version)

    def x_nnz_hint(self):
        return self.__dict__.get("x_nnz_max") if self._hint_ok() else None

    def x_spill_hint(self):
        return self.__dict__.get("x_spill") if self._hint_ok() else None

    def keys(self):
        return [k for k in self.__dict__ if not k.startswith("_")]


def collate(samples: Sequence[Sample]) -> Batch:
    """PyG ``Batch.from_data_list``: keys containing "index" are offset by the running
    node count (so ``rootindex`` becomes a global node id), ``batch``/``ptr`` built."""
    sizes = [int(s.x.size(0)) for s in samples]
    offs = np.concatenate([[0], np.cumsum(sizes)])
    off_t = torch.as_tensor(offs[:-1], dtype=torch.int64)
    kw = {
        "x": torch.cat([s.x for s in samples], 0),
        "edge_index": torch.cat([s.edge_index + int(o) for s, o in zip(samples, offs)], 1),
        "BU_edge_index": torch.cat([s.BU_edge_index + int(o) for s, o in zip(samples, offs)], 1),
        "y": torch.cat([s.y for s in samples], 0),
        "root": torch.cat([s.root for s in samples], 0),
        "rootindex": torch.cat([s.rootindex for s in samples], 0) + off_t,
        "batch": torch.repeat_interleave(torch.arange(len(samples), dtype=torch.int64),
                                         torch.as_tensor(sizes, dtype=torch.int64)),
        "ptr": torch.as_tensor(offs, dtype=torch.int64),
        "num_graphs": len(samples),
    }
    if all(s.cls is not None for s in samples):
        kw["cls"] = torch.cat([s.cls for s in samples], 0)
    if all(s.tweetids is not None for s in samples):
        kw["tweetids"] = torch.cat([s.tweetids for s in samples], 0)
    out = Batch(**kw)
    if all(s.x_nnz_max is not None for s in samples):
        # host-side hint: FusedTrainStep skips the dense fallback when every row fits the
        # sparse feature path (BGCN_FEAT_SPARSE)
        spill = sum(s.x_spill for s in samples) if all(s.x_spill is not None for s in samples) else None
        out.set_x_nnz_max(max(s.x_nnz_max for s in samples), spill)
    return out


def collate_pairs(items):
    """collate_fn for :class:`BiGraphDataset` items ``(sample, root tweet id)``: PyG's
    ``Collater`` on tuples - ``(Batch, list of root tweet ids)``."""
    samples, tids = zip(*items)
    return collate(samples), list(tids)


# ----------------------------------------------------------------------------- bulk synthetic batches
def synth_batch(rng: np.random.Generator, sizes: Sequence[int], vocab: int = VOCAB,
                num_classes: int = 4, tddroprate: float = 0.0, budroprate: float = 0.0,
                device="cpu", root_random: bool = False, dtype=torch.float32,
                long_rows: Optional[tuple] = None) -> Batch:
    """A collated batch of synthetic trees built directly (vectorised), identical in
    layout to ``collate([make_sample(npz) ...])``.  X is materialised dense on ``device``.

    ``long_rows=(frac, lo, hi[, roots])``: a fraction ``frac`` of the rows draw their word
    count uniformly from [lo, hi] instead of 1 + Poisson(11) (long posts: the reference
    caps no row, ``getTwittergraph.py:16-24``); ``roots`` (optional) forces that many
    tree roots among them."""
    sizes = np.asarray(sizes, dtype=np.int64)
    B = len(sizes)
    offs = np.concatenate([[0], np.cumsum(sizes)])
    N = int(offs[-1])
    td_rows, td_cols, bu_rows, bu_cols, roots = [], [], [], [], []
    for b, n in enumerate(sizes):
        n = int(n)
        par = synth_parents(rng, n)
        perm = rng.permutation(n) if root_random else np.arange(n)   # node k -> id perm[k]
        child = perm[np.arange(1, n)]
        parent = perm[par[1:]]
        order = np.lexsort((child, parent))                         # sorted by (parent, child)
        p_s, c_s = parent[order], child[order]
        roots.append(int(perm[0]) + int(offs[b]))
        E = len(p_s)
        keep_td = np.sort(rng.choice(E, size=int(E * (1 - tddroprate)), replace=False)) if tddroprate > 0 else np.arange(E)
        keep_bu = np.sort(rng.choice(E, size=int(E * (1 - budroprate)), replace=False)) if budroprate > 0 else np.arange(E)
        td_rows.append(p_s[keep_td] + offs[b]); td_cols.append(c_s[keep_td] + offs[b])
        bu_rows.append(c_s[keep_bu] + offs[b]); bu_cols.append(p_s[keep_bu] + offs[b])
    nnz = np.minimum(1 + rng.poisson(11.0, size=N), vocab)
    if long_rows is not None:
        frac, lo, hi = long_rows[:3]
        pick = rng.random(N) < frac
        if len(long_rows) > 3 and long_rows[3]:
            pick[np.asarray(roots[:int(long_rows[3])], dtype=np.int64)] = True
        nnz[pick] = np.minimum(rng.integers(int(lo), int(hi) + 1, size=int(pick.sum())), vocab)
    rows = np.repeat(np.arange(N, dtype=np.int64), nnz)
    # distinct ids per row: random ids, duplicates within a row collapse (set semantics);
    # the first draw of a duplicated (row, id) is kept, on the host, so x does not depend
    # on which duplicate a device scatter happens to write last
    cols = rng.integers(0, vocab, size=int(nnz.sum()), dtype=np.int64)
    vals = rng.integers(1, 4, size=int(nnz.sum())).astype(np.float32)
    _, first = np.unique(rows * vocab + cols, return_index=True)
    rows, cols, vals = rows[first], cols[first], vals[first]
    row_nnz = np.bincount(rows, minlength=N)                     # after duplicate collapse
    x = torch.zeros(N, vocab, dtype=dtype, device=device)
    x.index_put_((torch.as_tensor(rows, device=device), torch.as_tensor(cols, device=device)),
                 torch.as_tensor(vals, device=device).to(dtype))
    cat = lambda xs: torch.as_tensor(np.concatenate(xs) if xs else np.zeros(0, np.int64), dtype=torch.int64)
    ei = torch.stack([cat(td_rows), cat(td_cols)])
    bei = torch.stack([cat(bu_rows), cat(bu_cols)])
    rootindex = torch.as_tensor(roots, dtype=torch.int64)
    batch = torch.repeat_interleave(torch.arange(B, dtype=torch.int64), torch.as_tensor(sizes))
    y = torch.as_tensor(rng.integers(0, num_classes, size=B), dtype=torch.int64)
    # data.root ([B, vocab], dataset.py:97) is collated by the reference but never read
    # on the BiGCN path; it is omitted here.
    out = Batch(x=x, edge_index=ei, BU_edge_index=bei, y=y, rootindex=rootindex, batch=batch,
                ptr=torch.as_tensor(offs, dtype=torch.int64), num_graphs=B)
    out = out.to(device)
    out.set_x_nnz_max(int(row_nnz.max()) if N else 0,
                      int(np.maximum(row_nnz - SPARSE_CAP, 0).sum()) if N else 0)
    return out
