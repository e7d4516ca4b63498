"""Host-fed input path: DataLoader workers -> pinned memory -> H2D on
a copy stream -> the fused step, with the node features crossing PCIe compacted.

The reference moves every batch host -> device as PyG ``Batch`` tensors
(``model/Twitter/BiGCN_Twitter.py:168`` ``DataLoader(..., num_workers=5)``, ``:174-176``
``for Batch_data, tweetid in train_loader: Batch_data.to(device)``), with ``x`` dense:
``[N, 5000]`` fp32, 20 KB per node, ~590 MB per 128-tree batch - ~11 ms of PCIe per step,
40x the device step.  Here the same batch crosses as the CSR of its bag-of-words
non-zeros (~12 per row, ``Process/getTwittergraph.py:67-72``) plus the int64 index
tensors, ~4 MB in ONE copy, and the device builds the ELL / CSC of X from it
(``bgcn_batch.x_row_ptr``; the pass over a dense X disappears from the step).

Pieces:

* :class:`TreeStore` - the fold's trees packed once (the role of the per-tree ``.npz``
  files of ``Process/getTwittergraph.py:128``): per-node non-zero lists, per-tree edge
  lists (local ids, sorted by (parent, child)), ``rootindex``, ``y``, root tweet id.  Saved
  as plain ``.npy`` files and memory-mapped by the workers (no pickles).  Built from the
  reference's npz directory (:meth:`TreeStore.from_npz_dir`) or synthetically.
* :class:`PackedTreeDataset` - a map-style dataset over a store whose ``__getitems__``
  collates a whole batch into one shared-memory byte buffer (:class:`HostBatch`), so a
  ``torch.utils.data.DataLoader(ds, batch_size=128, shuffle=True, num_workers=5,
  collate_fn=host_collate, pin_memory=True)`` hands the main process one tensor per batch,
  pinned by the loader's pin thread.
* :class:`DeviceFeeder` - wraps the loader: each pinned batch is copied to the GPU on a
  dedicated stream ``depth`` batches ahead; the consumer's stream waits for the copy's
  event only when the batch is yielded (:class:`PackedBatch`, a ``Batch`` stand-in whose
  features stay compacted).

:class:`bigcn_amd.FusedTrainStep` takes a :class:`PackedBatch` as it takes a collated
``Batch`` (``next_data`` prefetch included) and computes the same bits as from the dense x
of the same trees (``tests/test_gpu_feed.py``).
"""
from __future__ import annotations

import ctypes
import json
import os
import weakref
from collections import deque
from typing import List, Optional, Sequence

import numpy as np
import torch

from .data import SPARSE_CAP, VOCAB, synth_parents, synth_tree_sizes

_ALIGN = 256
SPILL_PER_ROW = 32   # = BGCN_SPARSE_SPILL_PER_ROW
# the byte sections of a packed batch, in order (dtype, element count key)
_SECTIONS = (("x_row_ptr", np.int32), ("x_col", np.int32), ("x_val", np.float32),
             ("edge_index", np.int64), ("BU_edge_index", np.int64), ("batch", np.int64),
             ("rootindex", np.int64), ("y", np.int64), ("ptr", np.int64))


def _pad(n: int) -> int:
    return (n + _ALIGN - 1) // _ALIGN * _ALIGN


def _layout(N: int, B: int, nnz: int, Etd: int, Ebu: int):
    """{section: (byte offset, element count)} and the total bytes of a packed batch."""
    counts = {"x_row_ptr": N + 1, "x_col": nnz, "x_val": nnz, "edge_index": 2 * Etd,
              "BU_edge_index": 2 * Ebu, "batch": N, "rootindex": B, "y": B, "ptr": B + 1}
    lay, off = {}, 0
    for name, dt in _SECTIONS:
        lay[name] = (off, counts[name])
        off += _pad(counts[name] * np.dtype(dt).itemsize)
    return lay, off


# ----------------------------------------------------------------------------- the store
class TreeStore:
    """A fold's trees, packed: node ``k`` of tree ``t`` is store node ``tree_node[t] + k``.

    Arrays (all plain numpy, ``.npy`` on disk):
      ``tree_node [T+1]`` int64 - node offsets; ``node_nnz [Nall]`` int32 - non-zeros per
      node; ``entry_off [T+1]`` int64 - non-zero offsets per tree; ``cols [nnz]`` int32,
      ``vals [nnz]`` float32 - each node's non-zeros in ascending column order (the
      ``idx:count`` pairs of the RvNN line, ``getTwittergraph.py:16-24``);
      ``tree_edge [T+1]`` int64, ``edges [2, Eall]`` int32 - (parent, child) in local ids,
      sorted by (parent, child) (``getTwittergraph.py:56-61``); ``rootindex [T]`` int32
      (local), ``y [T]`` int64, ``root_tweetid [T]`` int64.  ``eids`` (json) names the
      trees."""

    _ARRAYS = ("tree_node", "node_nnz", "entry_off", "cols", "vals", "tree_edge", "edges",
               "rootindex", "y", "root_tweetid")

    def __init__(self, **arrays):
        for k in self._ARRAYS:
            setattr(self, k, arrays[k])
        self.eids: List[str] = list(arrays.get("eids") or [str(i) for i in range(len(self.y))])
        self.in_feats = int(arrays.get("in_feats", VOCAB))

    def __len__(self) -> int:
        return int(self.y.shape[0])

    # -- persistence (plain .npy + json: nothing that unpickles)
    def save(self, path: str) -> str:
        os.makedirs(path, exist_ok=True)
        for k in self._ARRAYS:
            np.save(os.path.join(path, k + ".npy"), np.ascontiguousarray(getattr(self, k)))
        with open(os.path.join(path, "meta.json"), "w") as f:
            json.dump({"eids": self.eids, "in_feats": self.in_feats}, f)
        return path

    @classmethod
    def load(cls, path: str, mmap: bool = True) -> "TreeStore":
        arrays = {k: np.load(os.path.join(path, k + ".npy"), mmap_mode="r" if mmap else None,
                             allow_pickle=False) for k in cls._ARRAYS}
        with open(os.path.join(path, "meta.json")) as f:
            meta = json.load(f)
        return cls(eids=meta["eids"], in_feats=meta["in_feats"], **arrays)

    # -- builders
    @classmethod
    def from_trees(cls, trees, in_feats: int = VOCAB) -> "TreeStore":
        """``trees``: iterable of dicts {x_rows: [(cols, vals)] per node, edges: [2, E] local
        (parent, child), rootindex, y, root_tweetid, eid}."""
        tree_node, node_nnz, cols, vals, tree_edge, edges = [0], [], [], [], [0], []
        rootindex, ys, rt, eids = [], [], [], []
        for t in trees:
            for c, v in t["x_rows"]:
                c = np.asarray(c, dtype=np.int64)
                v = np.asarray(v, dtype=np.float32)
                order = np.argsort(c, kind="stable")
                c, v = c[order], v[order]
                if c.size and (c[0] < 0 or c[-1] >= in_feats):
                    raise ValueError(f"tree {len(eids)}: a feature column outside [0, {in_feats})")
                if c.size > 1 and not np.all(c[1:] > c[:-1]):
                    raise ValueError(f"tree {len(eids)}: a feature column repeated within a node's row")
                keep = v != 0
                node_nnz.append(int(keep.sum()))
                cols.append(c[keep].astype(np.int32))
                vals.append(v[keep])
            tree_node.append(tree_node[-1] + len(t["x_rows"]))
            e = np.asarray(t["edges"], dtype=np.int64).reshape(2, -1)
            order = np.lexsort((e[1], e[0]))
            edges.append(e[:, order].astype(np.int32))
            tree_edge.append(tree_edge[-1] + e.shape[1])
            rootindex.append(int(t["rootindex"]))
            ys.append(int(t["y"]))
            rt.append(int(t.get("root_tweetid", -1)))
            eids.append(str(t.get("eid", len(eids))))
        node_nnz = np.asarray(node_nnz, dtype=np.int32)
        entry_node = np.concatenate([[0], np.cumsum(node_nnz, dtype=np.int64)])
        return cls(tree_node=np.asarray(tree_node, dtype=np.int64), node_nnz=node_nnz,
                   entry_off=entry_node[np.asarray(tree_node, dtype=np.int64)],
                   cols=np.concatenate(cols) if cols else np.zeros(0, np.int32),
                   vals=np.concatenate(vals) if vals else np.zeros(0, np.float32),
                   tree_edge=np.asarray(tree_edge, dtype=np.int64),
                   edges=np.concatenate(edges, 1) if edges else np.zeros((2, 0), np.int32),
                   rootindex=np.asarray(rootindex, dtype=np.int32), y=np.asarray(ys, dtype=np.int64),
                   root_tweetid=np.asarray(rt, dtype=np.int64), eids=eids, in_feats=in_feats)

    @classmethod
    def from_npz_dir(cls, data_path: str, eids: Sequence[str], in_feats: int = VOCAB) -> "TreeStore":
        """Pack the reference's per-tree npz files (``Process/getTwittergraph.py:128``: dense
        ``x``, ``edgeindex``, ``rootindex``, ``y``, ``tweetids``), read with
        ``allow_pickle=False``; the dense rows are compacted to their non-zeros here, once."""
        def gen():
            for eid in eids:
                with np.load(os.path.join(data_path, eid + ".npz"), allow_pickle=False) as f:
                    x = np.asarray(f["x"])
                    ri = int(f["rootindex"])
                    tid = -1
                    if "tweetids" in f.files:
                        tid = int(f["tweetids"][ri])
                    rows = [(np.nonzero(r)[0], r[np.nonzero(r)[0]]) for r in x]
                    yield {"x_rows": rows, "edges": np.asarray(f["edgeindex"]).reshape(2, -1), "rootindex": ri,
                           "y": int(f["y"]), "root_tweetid": tid, "eid": eid}
        return cls.from_trees(gen(), in_feats)

    @classmethod
    def synthetic(cls, count: int, mean_nodes: float, seed: int = 0, in_feats: int = VOCAB,
                  num_classes: int = 4, root_random: bool = False) -> "TreeStore":
        """Synthetic trees of SURVEY.md 8(d)'s shape (the real trees are absent,
        ``.MISSING_LARGE_BLOBS``): LogNormal(0.8) sizes of mean ``mean_nodes`` in [2, 8192],
        star-heavy attachment, rows of 1 + Poisson(11) distinct words with counts {1,2,3}."""
        rng = np.random.default_rng(seed)
        sizes = synth_tree_sizes(rng, count, mean_nodes)
        tree_node = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        Nall = int(tree_node[-1])
        edges, tree_edge, rootindex = [], [0], []
        for n in sizes:
            n = int(n)
            par = synth_parents(rng, n)
            perm = rng.permutation(n) if root_random else np.arange(n)
            child, parent = perm[1:], perm[par[1:]]
            order = np.lexsort((child, parent))
            edges.append(np.stack([parent[order], child[order]]).astype(np.int32))
            tree_edge.append(tree_edge[-1] + n - 1)
            rootindex.append(int(perm[0]))
        nnz = np.minimum(1 + rng.poisson(11.0, size=Nall), in_feats)
        rows = np.repeat(np.arange(Nall, dtype=np.int64), nnz)
        cols = rng.integers(0, in_feats, size=int(nnz.sum()), dtype=np.int64)
        vals = rng.integers(1, 4, size=int(nnz.sum())).astype(np.float32)
        key, first = np.unique(rows * in_feats + cols, return_index=True)   # sorted by (row, col)
        rows, cols, vals = key // in_feats, key % in_feats, vals[first]
        node_nnz = np.bincount(rows, minlength=Nall).astype(np.int32)
        entry_node = np.concatenate([[0], np.cumsum(node_nnz, dtype=np.int64)])
        return cls(tree_node=tree_node, node_nnz=node_nnz, entry_off=entry_node[tree_node],
                   cols=cols.astype(np.int32), vals=vals, tree_edge=np.asarray(tree_edge, dtype=np.int64),
                   edges=np.concatenate(edges, 1), rootindex=np.asarray(rootindex, dtype=np.int32),
                   y=rng.integers(0, num_classes, size=count).astype(np.int64),
                   root_tweetid=rng.integers(10**17, 10**18, size=count).astype(np.int64),
                   eids=[f"synth{seed}_{i}" for i in range(count)], in_feats=in_feats)

    # -- views of one tree / one batch
    def tree_rows(self, t: int):
        """(cols, vals) per node of tree t (local order)."""
        a, b = int(self.tree_node[t]), int(self.tree_node[t + 1])
        cnt = np.asarray(self.node_nnz[a:b], dtype=np.int64)
        off = int(self.entry_off[t]) + np.concatenate([[0], np.cumsum(cnt)])
        return [(np.asarray(self.cols[off[k]:off[k + 1]]), np.asarray(self.vals[off[k]:off[k + 1]]))
                for k in range(b - a)]

    def dense_x(self, trees: Sequence[int], dtype=np.float32) -> np.ndarray:
        """The collated dense ``x`` [N, in_feats] of ``trees`` (the reference's data.x)."""
        parts = []
        for t in trees:
            a, b = int(self.tree_node[t]), int(self.tree_node[t + 1])
            x = np.zeros((b - a, self.in_feats), dtype=dtype)
            for k, (c, v) in enumerate(self.tree_rows(t)):
                x[k, c] = v
            parts.append(x)
        return np.concatenate(parts, 0)


# ----------------------------------------------------------------------------- batches
def _drop_positions(rng: np.random.Generator, E_t: np.ndarray, rate: float) -> np.ndarray:
    """DropEdge of ``Process/dataset.py:68-90`` for a whole batch at once: per tree a uniform
    subset of exactly ``int(E_t * (1 - rate))`` edges, in edge order (the reference draws
    ``random.sample`` per tree; same distribution, a different stream).  Returns the kept
    positions into the concatenated list."""
    tot = int(E_t.sum())
    if tot == 0:
        return np.zeros(0, np.int64)
    tree = np.repeat(np.arange(E_t.size), E_t)
    order = np.lexsort((rng.random(tot), tree))          # by tree, random within a tree
    start = np.concatenate([[0], np.cumsum(E_t)[:-1]])
    rank = np.empty(tot, np.int64)
    rank[order] = np.arange(tot) - start[tree[order]]
    k = (E_t * (1.0 - rate)).astype(np.int64)            # int(length * (1 - rate))
    return np.nonzero(rank < k[tree])[0]


class HostBatch:
    """One collated batch as a single byte buffer (+ its sizes), what a DataLoader worker
    hands to the main process: either the buffer itself (pinned by the loader's pin thread
    through ``pin_memory()``), or - packed into a :class:`PinnedSlotRing` slot - only the
    slot number and the batch's sequence number (``buf`` is None until the main process
    binds the slot's view)."""

    __slots__ = ("buf", "meta", "root_tweetids", "slot", "seq")

    def __init__(self, buf: Optional[torch.Tensor], meta: dict, root_tweetids: np.ndarray,
                 slot: Optional[int] = None, seq: Optional[int] = None):
        self.buf, self.meta, self.root_tweetids, self.slot, self.seq = buf, meta, root_tweetids, slot, seq

    def pin_memory(self, device=None):
        if self.buf is None or self.slot is not None:
            return self
        return HostBatch(self.buf.pin_memory(), self.meta, self.root_tweetids)

    def section(self, name: str) -> np.ndarray:
        off, n = self.meta["layout"][name]
        dt = dict(_SECTIONS)[name]
        return self.buf.numpy()[off:off + n * np.dtype(dt).itemsize].view(dt)


def _shared_bytes(n: int) -> torch.Tensor:
    """A byte tensor allocated in shared memory (the worker -> main hand-off then sends a
    file descriptor instead of copying the batch)."""
    try:
        st = torch.UntypedStorage._new_shared(max(n, 1))
        return torch.empty(0, dtype=torch.uint8).set_(st)[:n]
    except Exception:   # pragma: no cover - other torch builds
        return torch.empty(n, dtype=torch.uint8)


def pack_batch(store: TreeStore, trees: Sequence[int], tddroprate: float = 0.0, budroprate: float = 0.0,
               rng: Optional[np.random.Generator] = None, shared: bool = False,
               bf16_values: bool = False, out: Optional[torch.Tensor] = None) -> HostBatch:
    """Collate ``trees`` of ``store`` as PyG's ``Batch.from_data_list`` does (every key
    containing "index" offset by the running node count, ``batch``/``ptr`` built; the BU
    list is the flip of the UNdropped TD list, ``dataset.py:80-90``) into one byte buffer,
    with ``x`` as the CSR of its non-zeros.  ``tddroprate`` / ``budroprate`` > 0 apply
    DropEdge on the host (vectorised; :func:`_drop_positions`); leave them 0 to draw it on
    the device (``FusedTrainStep(tddroprate=...)``).  ``out``: a byte tensor to pack into
    (a slot of a :class:`PinnedSlotRing`); the returned batch's ``buf`` is then its prefix."""
    t = np.asarray(trees, dtype=np.int64)
    B = int(t.size)
    n0, n1 = store.tree_node[t], store.tree_node[t + 1]
    sizes = (n1 - n0).astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(sizes)])
    N = int(offs[-1])
    e0, e1 = store.entry_off[t], store.entry_off[t + 1]
    nnz = int((e1 - e0).sum())
    g0, g1 = store.tree_edge[t], store.tree_edge[t + 1]
    E_t = (g1 - g0).astype(np.int64)
    Eall = int(E_t.sum())
    par = np.empty(Eall, np.int64)
    chi = np.empty(Eall, np.int64)
    np.concatenate([store.edges[0, a:b] for a, b in zip(g0, g1)] or [np.zeros(0, np.int32)], out=par,
                   casting="unsafe")
    np.concatenate([store.edges[1, a:b] for a, b in zip(g0, g1)] or [np.zeros(0, np.int32)], out=chi,
                   casting="unsafe")
    eoff = np.repeat(offs[:-1], E_t)
    par += eoff
    chi += eoff
    td_keep = bu_keep = None
    if tddroprate > 0 or budroprate > 0:
        rng = rng if rng is not None else np.random.default_rng()
        if tddroprate > 0:
            td_keep = _drop_positions(rng, E_t, tddroprate)
        if budroprate > 0:
            bu_keep = _drop_positions(rng, E_t, budroprate)
    Etd = Eall if td_keep is None else int(td_keep.size)
    Ebu = Eall if bu_keep is None else int(bu_keep.size)
    lay, total = _layout(N, B, nnz, Etd, Ebu)
    if out is not None:
        if out.numel() < total:
            raise ValueError(f"batch of {total} bytes does not fit the {out.numel()}-byte slot")
        buf = out[:total]
    else:
        buf = _shared_bytes(total) if shared else torch.empty(total, dtype=torch.uint8)
    raw = buf.numpy()

    def sec(name):
        off, n = lay[name]
        dt = dict(_SECTIONS)[name]
        return raw[off:off + n * np.dtype(dt).itemsize].view(dt)

    cnt = np.concatenate([store.node_nnz[a:b] for a, b in zip(n0, n1)] or [np.zeros(0, np.int32)])
    rp = sec("x_row_ptr")
    rp[0] = 0
    np.cumsum(cnt, out=rp[1:])
    xc = sec("x_col")
    np.concatenate([store.cols[a:b] for a, b in zip(e0, e1)] or [np.zeros(0, np.int32)], out=xc)
    if nnz and (int(xc.min()) < 0 or int(xc.max()) >= store.in_feats):
        raise ValueError(f"a feature column outside [0, {store.in_feats}) in the store")
    xv = sec("x_val")
    np.concatenate([store.vals[a:b] for a, b in zip(e0, e1)] or [np.zeros(0, np.float32)], out=xv)
    if bf16_values:   # the bf16 configuration: values as the bf16 x holds them
        xv[:] = torch.from_numpy(xv).to(torch.bfloat16).float().numpy()
    ei = sec("edge_index").reshape(2, Etd)
    bei = sec("BU_edge_index").reshape(2, Ebu)
    if td_keep is None:
        ei[0], ei[1] = par, chi
    else:
        ei[0], ei[1] = par[td_keep], chi[td_keep]
    if bu_keep is None:
        bei[0], bei[1] = chi, par
    else:
        bei[0], bei[1] = chi[bu_keep], par[bu_keep]
    sec("batch")[:] = np.repeat(np.arange(B, dtype=np.int64), sizes)
    sec("rootindex")[:] = store.rootindex[t].astype(np.int64) + offs[:-1]
    sec("y")[:] = store.y[t]
    sec("ptr")[:] = offs
    spill = int(np.maximum(cnt.astype(np.int64) - SPARSE_CAP, 0).sum()) if N else 0
    meta = {"N": N, "B": B, "nnz": nnz, "Etd": Etd, "Ebu": Ebu, "in_feats": store.in_feats,
            "bf16_values": bool(bf16_values),
            "nnz_max": int(cnt.max()) if N else 0, "spill": spill, "layout": lay, "bytes": total}
    return HostBatch(buf, meta, np.asarray(store.root_tweetid[t]))


def _per_tree_bytes(store: TreeStore) -> np.ndarray:
    """Bytes tree t adds to a packed batch (without the sections' padding)."""
    n = np.diff(store.tree_node)
    nnz = np.diff(store.entry_off)
    E = np.diff(store.tree_edge)
    return 4 * n + 8 * nnz + 32 * E + 8 * n + 24


class PinnedSlotRing:
    """``nslots`` fixed-size batch slots in one shared-memory region.

    DataLoader workers (forked after the ring exists, so they share its mapping) pack their
    batches straight into a slot; the main process page-locks the whole region once
    (``hipHostRegister`` through torch's runtime binding, :meth:`register`) and the
    :class:`DeviceFeeder` copies each batch to the GPU from its slot.  No batch bytes travel
    through the worker -> main queue and no pin-thread copy runs.  A slot is handed to the
    next batch only after the copy out of it has completed (:class:`SlotBatchSampler`)."""

    def __init__(self, nslots: int, slot_bytes: int):
        self.nslots = int(nslots)
        self.slot_bytes = _pad(int(slot_bytes))
        self.buf = _shared_bytes(self.nslots * self.slot_bytes)
        self.buf.zero_()                       # fault the pages in before workers fork
        self.events = [None] * self.nslots     # copy-out event of the batch in each slot
        self.seqs = [-1] * self.nslots         # ... and that batch's sequence number
        self._registered = None

    @staticmethod
    def slot_bytes_for(store: TreeStore, batch_size: int) -> int:
        """An upper bound of any ``batch_size``-tree batch of ``store`` (its largest trees)."""
        per = np.sort(_per_tree_bytes(store))[::-1][:batch_size]
        return int(per.sum()) + 8 * (batch_size + 2) + len(_SECTIONS) * _ALIGN

    def slot(self, s: int) -> torch.Tensor:
        return self.buf[s * self.slot_bytes:(s + 1) * self.slot_bytes]

    def register(self) -> None:
        """Page-lock the region for DMA (main process, once; after the workers forked)."""
        if self._registered is not None:
            return
        ptr, n = self.buf.data_ptr(), self.buf.numel()
        rt = torch.cuda.cudart()
        rc = rt.cudaHostRegister(ptr, n, 0)
        if int(rc) != 0:
            raise RuntimeError(f"hipHostRegister of the {n}-byte slot ring failed ({rc})")
        self._registered = rt

    def close(self) -> None:
        if self._registered is not None:
            torch.cuda.synchronize()
            self._registered.cudaHostUnregister(self.buf.data_ptr())
            self._registered = None

    def __del__(self):
        try:
            self.close()
        except Exception:   # interpreter shutdown
            pass

    def __getstate__(self):   # a spawned worker gets the region (shared by fd), not the events
        return {"nslots": self.nslots, "slot_bytes": self.slot_bytes, "buf": self.buf,
                "events": [None] * self.nslots, "seqs": [-1] * self.nslots, "_registered": None}

    def quiesce(self) -> None:
        """Wait for every issued copy out of the ring and forget the slots' batches: a new
        pass of the loader (after a DataLoader reset - a `break` out of the previous pass -
        whose packed-but-never-copied batches the loader discarded) starts from an empty
        ring with sequence numbers from 0."""
        for e in self.events:
            if e is not None:
                e.synchronize()
        self.events = [None] * self.nslots
        self.seqs = [-1] * self.nslots

    def free_for(self, s: int, seq: int) -> None:
        """Block until slot s may take batch ``seq``: the batch ``seq - nslots`` that used it
        has been copied out (its copy issued - else the ring is too small - and complete)."""
        prev = seq - self.nslots
        if prev < 0:
            return
        if self.seqs[s] != prev:
            raise RuntimeError(f"slot ring too small: batch {seq} would overwrite batch {prev} before its copy "
                               f"was issued (nslots = {self.nslots}; use >= prefetch_factor * num_workers + 2)")
        self.events[s].synchronize()


class SlotBatch(list):
    """A batch's tree indices plus its slot and sequence number (what the DataLoader sends a
    worker; the dataset packs into that slot)."""

    def __init__(self, idx, slot: int, seq: int):
        super().__init__(idx)
        self.slot, self.seq = slot, seq

    def __reduce__(self):
        return (SlotBatch, (list(self), self.slot, self.seq))


class SlotBatchSampler:
    """``batch_sampler`` for a DataLoader over a ring-backed :class:`PackedTreeDataset`: the
    batches of ``torch.utils.data.BatchSampler(Random/SequentialSampler)`` (shuffle as
    ``DataLoader(shuffle=True)``), each tagged with the next slot of the ring in turn; runs in
    the main process, where it waits for a slot's previous copy before reusing it."""

    def __init__(self, n: int, batch_size: int, ring: PinnedSlotRing, shuffle: bool = True,
                 drop_last: bool = False, generator=None, epochs: int = 1):
        base = (torch.utils.data.RandomSampler(range(n), generator=generator) if shuffle
                else torch.utils.data.SequentialSampler(range(n)))
        self.inner = torch.utils.data.BatchSampler(base, batch_size, drop_last)
        self.ring = ring
        self.epochs = int(epochs)   # passes over the data per iterator (reshuffled each pass)
        self._seq = 0

    def __len__(self) -> int:
        return len(self.inner) * self.epochs

    def __iter__(self):
        # runs at the first prefetch of a loader pass: with persistent workers that is after
        # the DataLoader's reset has drained the workers, so no worker still packs into a
        # slot of the previous pass
        self.ring.quiesce()
        self._seq = 0
        for _ in range(self.epochs):
            for idx in self.inner:
                seq = self._seq
                s = seq % self.ring.nslots
                self.ring.free_for(s, seq)
                self._seq += 1
                yield SlotBatch(idx, s, seq)


class PackedTreeDataset(torch.utils.data.Dataset):
    """Map-style dataset over a :class:`TreeStore` (the BiGraphDataset role,
    ``Process/dataset.py:45-99``, for the host-fed path).  ``__getitems__`` (called by the
    DataLoader's fetcher with the batch's indices) collates the whole batch into one
    shared-memory buffer; use ``collate_fn=host_collate``.  DropEdge: 0 here and the rates on
    ``FusedTrainStep`` (drawn on the device), or ``host_drop=True`` to draw it in the
    workers.  ``store`` may be a directory (loaded memory-mapped in each worker)."""

    def __init__(self, store, tddroprate: float = 0.0, budroprate: float = 0.0, host_drop: bool = False,
                 bf16_values: bool = False, indices: Optional[Sequence[int]] = None,
                 ring: Optional[PinnedSlotRing] = None):
        self.ring = ring
        self._path = store if isinstance(store, str) else None
        self._store = None if isinstance(store, str) else store
        n = len(self.store) if indices is None else len(indices)
        self.indices = np.arange(n) if indices is None else np.asarray(indices, dtype=np.int64)
        self.tddroprate, self.budroprate = float(tddroprate), float(budroprate)
        self.host_drop = bool(host_drop)
        self.bf16_values = bool(bf16_values)
        self._rng = None

    @property
    def store(self) -> TreeStore:
        if self._store is None:
            self._store = TreeStore.load(self._path, mmap=True)
        return self._store

    def __len__(self) -> int:
        return int(self.indices.size)

    def __getstate__(self):
        d = dict(self.__dict__)
        if self._path is not None:
            d["_store"] = None     # workers memory-map the directory themselves
        return d

    def _gen(self) -> np.random.Generator:
        if self._rng is None:
            info = torch.utils.data.get_worker_info()
            self._rng = np.random.default_rng(info.seed if info is not None else torch.initial_seed())
        return self._rng

    def __getitems__(self, idx) -> HostBatch:
        trees = self.indices[np.asarray(idx, dtype=np.int64)]
        drop = self.host_drop and (self.tddroprate > 0 or self.budroprate > 0)
        slot = getattr(idx, "slot", None) if self.ring is not None else None
        hb = pack_batch(self.store, trees, self.tddroprate if drop else 0.0, self.budroprate if drop else 0.0,
                        rng=self._gen() if drop else None,
                        shared=slot is None and torch.utils.data.get_worker_info() is not None,
                        bf16_values=self.bf16_values, out=None if slot is None else self.ring.slot(slot))
        if slot is not None:   # the bytes stay in the slot: send only where they are
            return HostBatch(None, hb.meta, hb.root_tweetids, slot, idx.seq)
        return hb

    def __getitem__(self, i) -> HostBatch:
        return self.__getitems__([i])


def host_collate(b):
    """collate_fn for :class:`PackedTreeDataset`: the batch is collated already."""
    return b


# ----------------------------------------------------------------------------- device side
class PackedBatch:
    """A collated batch on the device whose features stay compacted (the ``Batch`` a
    :class:`DeviceFeeder` yields).  Tensor attributes (``edge_index``, ``BU_edge_index``,
    ``batch``, ``rootindex``, ``y``, ``ptr``, ``x_row_ptr``, ``x_col``, ``x_val``) are views
    of one device buffer; ``x`` expands the dense features on first access
    (``bgcn_csr_to_dense``, for per-op code that reads them)."""

    def __init__(self, dbuf: torch.Tensor, meta: dict, root_tweetids=None, event=None, x_dtype=torch.float32):
        self.buf = dbuf
        self.meta = meta
        self.root_tweetids = root_tweetids
        self.event = event
        self.x_dtype = x_dtype
        self.num_graphs = meta["B"]
        self.in_feats = meta["in_feats"]
        self._views = {}
        self._x = None
        base = dbuf.data_ptr()
        self._ptr = {name: base + off for name, (off, _) in meta["layout"].items()}

    @property
    def num_nodes(self) -> int:
        return self.meta["N"]

    @property
    def device(self):
        return self.buf.device

    @property
    def fits_sparse(self) -> bool:
        """The rows fit the sparse path's ELL + spill pool (the step runs BGCN_FEAT_SPARSE)."""
        return self.in_feats <= 5120 and self.meta["spill"] <= self.meta["N"] * SPILL_PER_ROW

    def x_nnz_hint(self):
        return self.meta["nnz_max"]

    def x_spill_hint(self):
        return self.meta["spill"]

    def _view(self, name: str) -> torch.Tensor:
        v = self._views.get(name)
        if v is None:
            off, n = self.meta["layout"][name]
            dt = {np.int32: torch.int32, np.int64: torch.int64, np.float32: torch.float32}[dict(_SECTIONS)[name]]
            v = self.buf[off:off + n * torch.empty(0, dtype=dt).element_size()].view(dt)
            if name in ("edge_index", "BU_edge_index"):
                v = v.view(2, -1)
            self._views[name] = v
        return v

    def __getattr__(self, name):
        if name in dict(_SECTIONS):
            return self._view(name)
        raise AttributeError(name)

    @property
    def x(self) -> torch.Tensor:
        """The dense features [N, in_feats] (expanded on the device, once)."""
        if self._x is None:
            from . import _lib
            N, F = self.meta["N"], self.in_feats
            x = torch.empty(N, F, dtype=self.x_dtype, device=self.buf.device)
            st = torch.zeros(1, dtype=torch.int32, device=self.buf.device)
            _lib.check(_lib.lib().bgcn_csr_to_dense(self._ptr["x_row_ptr"], self._ptr["x_col"], self._ptr["x_val"],
                                                    N, F, x.data_ptr(), F,
                                                    _lib.BGCN_DTYPE_BF16 if self.x_dtype == torch.bfloat16
                                                    else _lib.BGCN_DTYPE_F32, st.data_ptr(), _lib.stream_handle()))
            if int(st.item()) & 1:   # (one host read, on the first access only)
                raise IndexError("a feature column outside [0, in_feats) in the batch's x_col")
            self._x = x
        return self._x

    def fill_desc(self, d) -> None:
        """bgcn_batch fields of this batch (features compacted: x = NULL)."""
        from . import _lib
        p, m = self._ptr, self.meta
        d.x, d.ldx = None, self.in_feats
        d.num_nodes, d.num_graphs = m["N"], m["B"]
        d.batch, d.rootindex = p["batch"], p["rootindex"]
        d.td_edge_index, d.td_num_edges = p["edge_index"], m["Etd"]
        d.bu_edge_index, d.bu_num_edges = p["BU_edge_index"], m["Ebu"]
        d.x_dtype = _lib.BGCN_DTYPE_BF16 if self.x_dtype == torch.bfloat16 else _lib.BGCN_DTYPE_F32
        d.x_row_ptr, d.x_col, d.x_val = p["x_row_ptr"], p["x_col"], p["x_val"]

    def keys(self):
        return [name for name, _ in _SECTIONS] + ["num_graphs"]


class DeviceFeeder:
    """Iterate a loader of :class:`HostBatch` (pinned) as device :class:`PackedBatch` es.

    Each batch is copied host -> device on ``copy_stream`` as soon as it is fetched, ``depth``
    batches ahead of the one being yielded; the yielding thread's current stream waits on
    the copy's event (a device-side wait, no host sync).  Device buffers are recycled: when
    a yielded batch is released (its last reference dropped) the buffer returns to the
    feeder's pool; once no view of it is left either, a later copy into it waits for an
    event recorded on the consumer stream at that point (no allocation, no ``record_stream``
    per batch: those cost ~20 us of host time per batch).  A :class:`NativeLoader` makes one
    pass (``epochs`` of them inside it): iterating a feeder over an exhausted one raises.  ``timing=True`` records start/end events around
    every copy (:meth:`copy_stats`)."""

    def __init__(self, loader, device=None, depth: int = 3, x_dtype=torch.float32, timing: bool = False,
                 ring: Optional[PinnedSlotRing] = None):
        self.loader = loader
        self.ring = ring if ring is not None else getattr(getattr(loader, "dataset", None), "ring", None)
        self.device = torch.device(device if device is not None else "cuda")
        self.depth = max(1, int(depth))
        self.x_dtype = x_dtype
        self.copy_stream = torch.cuda.Stream(device=self.device)
        self.timing = timing
        self._events = []
        self.bytes_copied = 0
        self.batches = 0
        self._free = []          # (device buffer, release event) ready for reuse
        self._consumer = None

    @staticmethod
    def _views_alive(buf: torch.Tensor) -> bool:
        """Whether a tensor other than the pool's own references views ``buf`` (a kept
        ``batch.y``).  Unknown (no use-count query in this torch) counts as alive."""
        try:
            return torch._C._storage_Use_Count(buf.untyped_storage()._cdata) > 2
        except (AttributeError, RuntimeError):
            return True

    def _release(self, buf: torch.Tensor) -> None:
        # the buffer returns to the pool when its batch dies; a view of it may outlive the
        # batch (a kept `batch.y`) and be read by kernels queued later, so the event its
        # reuse waits for is recorded when it is TAKEN: by then no view is left (checked),
        # so every kernel that read it is already enqueued on the consumer stream
        self._free.append((buf, None))

    def _take(self, nbytes: int):
        for k, (buf, ev) in enumerate(self._free):
            # reused only once no tensor of the caller still views it
            if buf.numel() >= nbytes and not self._views_alive(buf):
                del self._free[k]
                if ev is None:
                    ev = torch.cuda.Event()
                    ev.record(self._consumer)
                return buf, ev
        # a new buffer (with headroom: batches vary in size), allocated on the consumer stream
        # and marked used by the copy stream once, so that when the pool drops it the caching
        # allocator still orders its reuse behind the copies; the pool grows to the number of
        # batches alive at once (depth + the consumer's)
        buf = torch.empty(int(nbytes * 1.25) + 4096, dtype=torch.uint8, device=self.device)
        buf.record_stream(self.copy_stream)
        return buf, None

    def _issue(self, hb: HostBatch, consumer) -> PackedBatch:
        # the bf16 configuration has two knobs that must agree: the workers round x_val to
        # bf16 (PackedTreeDataset(bf16_values=True)) exactly when the step's x is bf16 (the
        # dense bf16 path and bgcn_csr_to_dense round the same values)
        if hb.meta.get("bf16_values", False) != (self.x_dtype == torch.bfloat16):
            raise ValueError(f"DeviceFeeder(x_dtype={self.x_dtype}) over batches packed with bf16_values="
                             f"{hb.meta.get('bf16_values', False)}: set both for the bf16 configuration")
        ring = self.ring
        if hb.slot is not None:
            ring.register()
            src = ring.slot(hb.slot)[:hb.meta["bytes"]]
        else:
            src = hb.buf if hb.buf.is_pinned() else hb.buf.pin_memory()
        cs = self.copy_stream
        pool, free_ev = self._take(src.numel())
        d = pool[:src.numel()]
        with torch.cuda.stream(cs):
            if free_ev is not None:
                cs.wait_event(free_ev)
            t0 = None
            if self.timing:
                t0 = torch.cuda.Event(enable_timing=True)
                t0.record(cs)
            d.copy_(src, non_blocking=True)
            ev = torch.cuda.Event(enable_timing=self.timing)
            ev.record(cs)
        if hb.slot is not None:   # the slot may take a later batch once this copy is done
            ring.events[hb.slot], ring.seqs[hb.slot] = ev, hb.seq
        if self.timing:
            self._events.append((t0, ev))
        self.bytes_copied += src.numel()
        self.batches += 1
        pb = PackedBatch(d, hb.meta, hb.root_tweetids, ev, self.x_dtype)
        weakref.finalize(pb, self._release, pool).atexit = False
        return pb

    def _issue_native(self):
        """The next batch of a :class:`NativeLoader`: one library call (the loader's threads
        packed it) that issues the copy on the copy stream."""
        L = self.loader
        pool, free_ev = self._take(L.slot_bytes)
        cs = self.copy_stream
        if free_ev is not None:
            cs.wait_event(free_ev)
        t0 = None
        if self.timing:
            # the bracket holds the copy only: the host first waits for the batch's packing
            # (an event recorded before that wait timed the packing too)
            L.wait()
            t0 = torch.cuda.Event(enable_timing=True)
            t0.record(cs)
        got = L.next_into(pool, cs.cuda_stream)
        if got is None:
            self._free.append((pool, free_ev))
            return None
        meta, rt = got
        ev = torch.cuda.Event(enable_timing=self.timing)
        ev.record(cs)
        if self.timing:
            self._events.append((t0, ev))
        self.bytes_copied += meta["bytes"]
        self.batches += 1
        pb = PackedBatch(pool[:meta["bytes"]], meta, rt, ev, self.x_dtype)
        weakref.finalize(pb, self._release, pool).atexit = False
        return pb

    def _iter_native(self, consumer):
        q = deque()
        while len(q) < self.depth:
            pb = self._issue_native()
            if pb is None:
                break
            q.append(pb)
        while q:
            pb = q.popleft()
            nxt = self._issue_native()   # keep `depth` copies in flight
            if nxt is not None:
                q.append(nxt)
            consumer.wait_event(pb.event)
            yield pb

    def __iter__(self):
        consumer = torch.cuda.current_stream(self.device)
        self._consumer = consumer
        if isinstance(self.loader, NativeLoader):
            if self.loader.bf16_values != (self.x_dtype == torch.bfloat16):
                raise ValueError(f"DeviceFeeder(x_dtype={self.x_dtype}) over a NativeLoader with bf16_values="
                                 f"{self.loader.bf16_values}: set both for the bf16 configuration")
            if self.loader.exhausted:
                raise RuntimeError("this NativeLoader has handed out all its batches (one pass per loader: "
                                   "ask for several epochs with NativeLoader(..., epochs=E), or make a new one)")
            yield from self._iter_native(consumer)
            return
        it = iter(self.loader)
        q = deque()
        for hb in it:
            q.append(self._issue(hb, consumer))
            if len(q) >= self.depth:
                break
        while q:
            pb = q.popleft()
            for hb in it:          # keep `depth` copies in flight
                q.append(self._issue(hb, consumer))
                break
            consumer.wait_event(pb.event)
            yield pb

    def copy_stats(self, reset: bool = True):
        """(copies, mean bytes, mean copy ms) of the timed copies so far (synchronises)."""
        if not self._events:
            return 0, 0.0, 0.0
        self._events[-1][1].synchronize()
        ms = [a.elapsed_time(b) for a, b in self._events]
        n = len(ms)
        out = (n, self.bytes_copied / max(self.batches, 1), float(np.mean(ms)))
        if reset:
            self._events.clear()
        return out


class _TreeStoreArgs(ctypes.Structure):
    """bgcn_tree_store (include/bgcn.h)."""
    _fields_ = [("num_trees", ctypes.c_int64), ("in_feats", ctypes.c_int64), ("tree_node", ctypes.c_void_p),
                ("node_nnz", ctypes.c_void_p), ("entry_off", ctypes.c_void_p), ("cols", ctypes.c_void_p),
                ("vals", ctypes.c_void_p), ("tree_edge", ctypes.c_void_p), ("edges", ctypes.c_void_p),
                ("edges_ld", ctypes.c_int64), ("rootindex", ctypes.c_void_p), ("y", ctypes.c_void_p)]


class _LoaderBatch(ctypes.Structure):
    """bgcn_loader_batch (include/bgcn.h)."""
    _fields_ = [("num_nodes", ctypes.c_int64), ("num_graphs", ctypes.c_int64), ("nnz", ctypes.c_int64),
                ("td_num_edges", ctypes.c_int64), ("bu_num_edges", ctypes.c_int64), ("nnz_max", ctypes.c_int64),
                ("spill", ctypes.c_int64), ("bytes", ctypes.c_int64), ("off", ctypes.c_int64 * 9),
                ("seq", ctypes.c_int64)]


class _LoaderStats(ctypes.Structure):
    """bgcn_loader_stats (include/bgcn.h)."""
    _fields_ = [("packs", ctypes.c_int64), ("pack_ms", ctypes.c_double), ("slot_wait_ms", ctypes.c_double),
                ("caller_wait_ms", ctypes.c_double), ("threads", ctypes.c_int64),
                ("copy_call_ms", ctypes.c_double), ("copy_call_ms_max", ctypes.c_double),
                ("record_call_ms_max", ctypes.c_double)]


_SECTION_NAMES = tuple(name for name, _ in _SECTIONS)


class NativeLoader:
    """The host-fed loader in libbgcn (``bgcn_loader_*``): ``num_workers`` C++ threads collate
    each batch of a :class:`TreeStore` into a page-locked slot exactly as :func:`pack_batch`
    does (byte for byte, ``tests/test_feed.py``), and :class:`DeviceFeeder` copies it to the
    device with one call per batch - the role of the reference's ``DataLoader(traindata_list,
    batch_size=128, shuffle=True, num_workers=5)`` (``BiGCN_Twitter.py:168``) without a
    Python worker protocol: :func:`host_fed_loader`'s torch DataLoader spent ~170 us of the
    main process per batch on its index queue, result unpickling, sampler and copy
    bookkeeping.  Batches come in a Fisher-Yates order per epoch from ``seed`` (or in order
    with ``shuffle=False``); DropEdge is drawn on the device (``FusedTrainStep``).
    ``pinned=False``: plain host slots and no copy (``next_host``, tests)."""

    def __init__(self, store, batch_size: int = 128, num_workers: int = 5, shuffle: bool = True,
                 drop_last: bool = True, seed: Optional[int] = None, epochs: int = 1, bf16_values: bool = False,
                 indices: Optional[Sequence[int]] = None, nslots: Optional[int] = None, pinned: bool = True):
        from . import _lib
        st = TreeStore.load(store, mmap=True) if isinstance(store, str) else store
        self.store = st
        self.bf16_values = bool(bf16_values)
        self.batch_size = int(batch_size)

        def arr(a, dt):
            return np.ascontiguousarray(np.asarray(a), dtype=dt)
        # the arrays the threads read, kept alive (and in the dtypes bgcn_tree_store names)
        self._arrays = {
            "tree_node": arr(st.tree_node, np.int64), "node_nnz": arr(st.node_nnz, np.int32),
            "entry_off": arr(st.entry_off, np.int64), "cols": arr(st.cols, np.int32),
            "vals": arr(st.vals, np.float32), "tree_edge": arr(st.tree_edge, np.int64),
            "edges": arr(st.edges, np.int32).reshape(2, -1), "rootindex": arr(st.rootindex, np.int32),
            "y": arr(st.y, np.int64)}
        a = self._arrays
        s = _TreeStoreArgs()
        s.num_trees, s.in_feats = len(st), int(st.in_feats)
        for k in ("tree_node", "node_nnz", "entry_off", "cols", "vals", "tree_edge", "edges", "rootindex", "y"):
            setattr(s, k, a[k].ctypes.data)
        s.edges_ld = a["edges"].shape[1]
        self._store_args = s
        self._indices = None if indices is None else arr(indices, np.int64)
        n = 0 if self._indices is None else self._indices.size
        # the host-only form needs no device (its threads only pack)
        self._L = _lib.lib() if pinned else _lib.load_library()
        h = ctypes.c_void_p()
        seed = int(torch.initial_seed() if seed is None else seed) & (2**64 - 1)
        nslots = int(nslots) if nslots is not None else max(2 * num_workers, 4) + 4
        _lib.check(self._L.bgcn_loader_create(ctypes.addressof(s), None if self._indices is None
                                                 else self._indices.ctypes.data, n, self.batch_size,
                                                 int(drop_last), int(shuffle), seed, int(epochs),
                                                 max(1, int(num_workers)), nslots, int(bf16_values),
                                                 int(pinned), ctypes.byref(h)))
        self._h = h
        self._lib = _lib
        self.slot_bytes = int(self._L.bgcn_loader_slot_bytes(h))
        self._out = _LoaderBatch()
        self._trees = np.empty(self.batch_size, np.int64)
        self.exhausted = False      # every batch handed out (the loader makes one pass)

    def __len__(self) -> int:
        return int(self._L.bgcn_loader_len(self._h))

    def _meta(self, o) -> dict:
        N, B, nnz, E = o.num_nodes, o.num_graphs, o.nnz, o.td_num_edges
        counts = (N + 1, nnz, nnz, 2 * E, 2 * E, N, B, B, B + 1)
        return {"N": N, "B": B, "nnz": nnz, "Etd": E, "Ebu": o.bu_num_edges, "in_feats": self.store.in_feats,
                "bf16_values": self.bf16_values, "nnz_max": o.nnz_max, "spill": o.spill,
                "layout": dict(zip(_SECTION_NAMES, zip(o.off, counts))), "bytes": o.bytes}

    def next_into(self, dst: torch.Tensor, stream_handle):
        """The next batch copied into device memory ``dst`` on ``stream_handle``: (meta, root
        tweet ids), or None after the last batch."""
        o = self._out
        rc = self._L.bgcn_loader_next(self._h, dst.data_ptr(), dst.numel(), stream_handle,
                                              ctypes.addressof(o), self._trees.ctypes.data, self._trees.size, None)
        if rc == 1:
            self.exhausted = True
            return None
        self._lib.check(rc)
        B = o.num_graphs
        return self._meta(o), self.store.root_tweetid[self._trees[:B]]

    def wait(self) -> bool:
        """Block until the next batch is packed (without taking it); False after the last."""
        rc = self._L.bgcn_loader_wait(self._h)
        if rc == 1:
            return False
        self._lib.check(rc)
        return True

    def stats(self, reset: bool = False) -> dict:
        """Where the loader's time went (bgcn_loader_get_stats): batches packed, mean ms per pack
        (one thread), thread-ms waiting for a slot's turn, caller ms waiting for packed
        batches, threads."""
        o = _LoaderStats()
        self._lib.check(self._L.bgcn_loader_get_stats(self._h, ctypes.addressof(o), int(reset)))
        n = max(int(o.packs), 1)
        return {"packs": int(o.packs), "pack_ms_per_batch": round(o.pack_ms / n, 4),
                "slot_wait_ms_per_batch": round(o.slot_wait_ms / n, 4),
                "caller_wait_ms_total": round(o.caller_wait_ms, 3), "threads": int(o.threads),
                "copy_call_ms_per_batch": round(o.copy_call_ms / n, 4),
                "memcpy_call_ms_max": round(o.copy_call_ms_max, 3),
                "record_call_ms_max": round(o.record_call_ms_max, 3)}

    def next_host(self) -> Optional[HostBatch]:
        """(``pinned=False``) the next batch as a :class:`HostBatch` over a copy of its bytes."""
        o = self._out
        p = ctypes.c_void_p()
        rc = self._L.bgcn_loader_next(self._h, None, 0, None, ctypes.addressof(o), self._trees.ctypes.data,
                                              self._trees.size, ctypes.byref(p))
        if rc == 1:
            self.exhausted = True
            return None
        self._lib.check(rc)
        raw = np.ctypeslib.as_array((ctypes.c_uint8 * o.bytes).from_address(p.value)).copy()
        self.last_trees = self._trees[:o.num_graphs].copy()
        return HostBatch(torch.from_numpy(raw), self._meta(o), self.store.root_tweetid[self.last_trees])

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            self._L.bgcn_loader_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:   # interpreter shutdown
            pass


class prepare_ahead:
    """The drop-in loop's data pipeline stage that prepares each batch one step ahead:

        for Batch_data in prepare_ahead(batches, model):      # batches: the reference's
            out_labels = model(Batch_data)                     # DataLoader + .to(device)
            loss = F.nll_loss(out_labels, Batch_data.y)        # (BiGCN_Twitter.py:174-189,
            optimizer.zero_grad(); loss.backward(); optimizer.step()   # the body untouched)

    When batch k is handed out, batch k+1's weight-independent preparation
    (``ops.prepare_batch``: DropEdge-free K1 of both directions, tree items, the ELL / CSC
    of X - the HBM-bound pass over X) is queued on a side stream behind everything the
    caller has queued so far, so it runs beside step k on the device; the model's forward
    finds it on ``Batch_data._bgcn_prep`` and skips K1 and the pass over X.  The loop body
    is the reference's; the batches are dense-x device batches (collated ``Batch``).
    ``slots`` prepared buffers are reused in turn: a preparation into a slot waits for the
    caller's stream, so the step that read the slot's previous batch has finished, and it
    retires the slot's previous preparation (a batch run again after its slot was reused
    is prepared inline by its forward: ``PreparedBatch.matches``).  The batch's tensors are
    marked as used by the side stream (``record_stream``), so a batch dropped before its
    preparation ends keeps its memory until then; when the iteration ends the caller's
    stream is ordered behind the side stream."""

    def __init__(self, batches, model, slots: int = 2):
        if slots < 2:
            raise ValueError("prepare_ahead needs at least two buffers")
        self.batches, self.model, self.slots = batches, model, slots
        self._bufs = [None] * slots
        self._gens = [[0] for _ in range(slots)]   # per slot: generation of its current batch
        self._stream = None
        self._main = None                           # the caller's stream (joined at the end)

    def _launch(self, data, slot: int):
        from .ops import prepare_batch
        main = torch.cuda.current_stream(data.x.device)
        self._main = main
        if self._stream is None:
            self._stream = torch.cuda.Stream(data.x.device)
        self._stream.wait_stream(main)          # the batch's tensors and the slot's last reader
        m = self.model
        feat = m._feat(data) if hasattr(m, "_feat") else "auto"
        gen = self._gens[slot]
        gen[0] += 1                             # the slot's previous preparation is stale now
        with torch.cuda.stream(self._stream):
            prep = prepare_batch(data, m.degree_on, feat, buf=self._bufs[slot], stream=self._stream)
        for t in prep._keep:                    # read by the side stream: freed only after it
            t.record_stream(self._stream)
        prep._slot = (gen, gen[0])
        self._bufs[slot] = prep.buf
        data._bgcn_prep = prep

    def __iter__(self):
        it = iter(self.batches)
        try:
            cur = next(it)
        except StopIteration:
            return
        try:
            self._launch(cur, 0)
            k = 0
            while True:
                try:
                    nxt = next(it)
                except StopIteration:
                    nxt = None
                if nxt is not None:
                    self._launch(nxt, (k + 1) % self.slots)
                yield cur
                if nxt is None:
                    return
                cur = nxt
                k += 1
        finally:
            # a preparation no forward consumed (the loop broke early, or its batch no
            # longer matched) is joined: nothing still writes a buffer the caller drops
            if self._stream is not None:
                self._main.wait_stream(self._stream)


def host_fed_loader(store, batch_size: int = 128, num_workers: int = 5, shuffle: bool = True,
                    drop_last: bool = True, prefetch_factor: int = 2, seed: Optional[int] = None,
                    epochs: int = 1, **ds_kw):
    """The host-fed loader: a ``torch.utils.data.DataLoader`` with worker processes (the
    reference's ``DataLoader(traindata_list, batch_size=batchsize, shuffle=True,
    num_workers=5)``, ``BiGCN_Twitter.py:168``) over a :class:`PackedTreeDataset` whose
    workers pack each batch into a slot of a :class:`PinnedSlotRing`.  Returns the loader;
    wrap it in :class:`DeviceFeeder` for device batches.  ``store``: a :class:`TreeStore`
    or a saved store's directory.  ``epochs``: passes over the store per iteration of the
    loader (one pipeline across epoch boundaries: no drain and refill of the workers)."""
    if isinstance(store, str):
        st = TreeStore.load(store, mmap=True)
    else:
        st = store
    nslots = prefetch_factor * max(num_workers, 1) + 4
    ring = PinnedSlotRing(nslots, PinnedSlotRing.slot_bytes_for(st, batch_size))
    ds = PackedTreeDataset(store, ring=ring, **ds_kw)
    gen = torch.Generator().manual_seed(int(seed)) if seed is not None else None
    sampler = SlotBatchSampler(len(ds), batch_size, ring, shuffle=shuffle, drop_last=drop_last, generator=gen,
                               epochs=epochs)
    kw = {"prefetch_factor": prefetch_factor, "persistent_workers": True} if num_workers > 0 else {}
    return torch.utils.data.DataLoader(ds, batch_sampler=sampler, num_workers=num_workers,
                                       collate_fn=host_collate, **kw)
