"""CPU tests of the host-fed input path (bigcn_amd.feed): the packed store and the
one-buffer batches against the reference-format path (per-tree npz -> BiGraphDataset item
-> PyG-style collate, Process/dataset.py:64-99), DropEdge counts, the DataLoader with
worker processes, and the store's .npy persistence."""
import os

import numpy as np
import pytest
import torch

from bigcn_amd import data as D
from bigcn_amd import feed as FD


def _npz_trees(tmp_path, count=6, vocab=64, seed=3):
    """Reference-format npz files (getTwittergraph.py:128 keys) of random trees, some with a
    non-zero rootindex and a long row."""
    rng = np.random.default_rng(seed)
    eids = []
    for t in range(count):
        n = int(rng.integers(1, 12))
        par = D.synth_parents(rng, n)
        bow = D.synth_bow(rng, n, vocab=vocab, mean_extra=4.0)
        if t == 2 and n > 1:
            bow[1] = (np.arange(40), np.full(40, 2.0))       # a row over the ELL cap
        lines = D.tree_to_rvnn_lines(f"e{t}", par, bow, root_pos=(n - 1 if t % 2 else 0))
        tree = D.parse_rvnn(lines)[f"e{t}"]
        d = D.graph_npz_dict(tree, int(rng.integers(0, 4)), vocab=vocab)
        d["tweetids"] = np.array([str(1000 * t + k) for k in range(n)])
        np.savez(tmp_path / f"e{t}.npz", **d)
        eids.append(f"e{t}")
    return eids


def _csr_dense(hb, N, F):
    rp, col, val = hb.section("x_row_ptr"), hb.section("x_col"), hb.section("x_val")
    x = np.zeros((N, F), np.float32)
    for i in range(N):
        x[i, col[rp[i]:rp[i + 1]]] = val[rp[i]:rp[i + 1]]
        assert np.all(np.diff(col[rp[i]:rp[i + 1]]) > 0)         # ascending, no duplicates
        assert np.all(val[rp[i]:rp[i + 1]] != 0)                 # non-zeros only
    return x


def test_pack_matches_reference_collation(tmp_path):
    eids = _npz_trees(tmp_path)
    store = FD.TreeStore.from_npz_dir(str(tmp_path), eids, in_feats=64)
    ds = D.BiGraphDataset(eids, None, data_path=str(tmp_path))
    order = [4, 0, 2, 5, 1]
    ref = D.collate([ds[i][0] for i in order])
    hb = FD.pack_batch(store, order)
    m = hb.meta
    N = ref.x.size(0)
    assert (m["N"], m["B"], m["in_feats"]) == (N, len(order), 64)
    assert np.array_equal(_csr_dense(hb, N, 64), ref.x.numpy())
    assert m["nnz"] == int((ref.x != 0).sum())
    assert m["nnz_max"] == int((ref.x != 0).sum(1).max())
    assert m["spill"] == int(((ref.x != 0).sum(1) - D.SPARSE_CAP).clamp_min(0).sum()) > 0
    for name in ("edge_index", "BU_edge_index"):
        assert np.array_equal(hb.section(name).reshape(2, -1), getattr(ref, name).numpy()), name
    for name in ("batch", "rootindex", "y", "ptr"):
        assert np.array_equal(hb.section(name), getattr(ref, name).numpy()), name
    # root tweet ids: the reference's second item element (dataset.py:99), as int
    assert [str(v) for v in hb.root_tweetids] == [ds[i][1] for i in order]
    # the collated buffer: 256-byte aligned sections, the sizes the layout says
    for name, (off, _) in m["layout"].items():
        assert off % 256 == 0, name
    assert hb.buf.numel() == m["bytes"]


def test_store_save_load_mmap(tmp_path):
    store = FD.TreeStore.synthetic(40, 30, seed=7, in_feats=300)
    path = store.save(str(tmp_path / "store"))
    back = FD.TreeStore.load(path, mmap=True)
    assert isinstance(back.cols, np.memmap) and back.eids == store.eids and back.in_feats == 300
    a = FD.pack_batch(store, [3, 9, 1])
    b = FD.pack_batch(back, [3, 9, 1])
    assert a.meta == b.meta
    for name in a.meta["layout"]:
        assert np.array_equal(a.section(name), b.section(name)), name
    # every tree's edges: n - 1 (parent, child) pairs sorted by (parent, child), local ids
    for t in range(len(store)):
        e = store.edges[:, store.tree_edge[t]:store.tree_edge[t + 1]]
        n = int(store.tree_node[t + 1] - store.tree_node[t])
        assert e.shape[1] == n - 1
        assert np.array_equal(np.lexsort((e[1], e[0])), np.arange(e.shape[1]))
        assert sorted(e[1].tolist()) == sorted(set(range(n)) - {int(store.rootindex[t])})


def test_synthetic_store_dense_equals_packed():
    store = FD.TreeStore.synthetic(25, 20, seed=2, in_feats=128, root_random=True)
    trees = list(range(0, 25, 2))
    hb = FD.pack_batch(store, trees)
    assert np.array_equal(_csr_dense(hb, hb.meta["N"], 128), store.dense_x(trees))
    assert not np.array_equal(hb.section("rootindex"), hb.section("ptr")[:-1])   # roots moved


@pytest.mark.parametrize("rate", [0.2, 0.5])
def test_host_dropedge_counts(rate):
    """dataset.py:68-90: per tree exactly int(E_t * (1 - rate)) edges kept, in edge order,
    TD and BU drawn independently, BU from the undropped TD list."""
    store = FD.TreeStore.synthetic(30, 25, seed=11, in_feats=64)
    trees = list(range(30))
    full = FD.pack_batch(store, trees)
    hb = FD.pack_batch(store, trees, rate, rate, rng=np.random.default_rng(0))
    E_t = (store.tree_edge[1:] - store.tree_edge[:-1])[trees]
    fe = full.section("edge_index").reshape(2, -1)
    for name in ("edge_index", "BU_edge_index"):
        e = hb.section(name).reshape(2, -1)
        src = e[0] if name == "edge_index" else e[1]              # the parent side
        bt = full.section("batch")[src]
        assert np.array_equal(np.bincount(bt, minlength=30), (E_t * (1 - rate)).astype(np.int64))
        # a subsequence of the full list, in order
        ref = fe if name == "edge_index" else fe[::-1]
        key_full = ref[0] * 10**6 + ref[1]
        key = e[0] * 10**6 + e[1]
        pos = np.searchsorted(key_full, key) if np.all(np.diff(key_full) > 0) else None
        if pos is not None:
            assert np.all(np.diff(pos) > 0)
    assert not np.array_equal(hb.section("edge_index").reshape(2, -1),
                              hb.section("BU_edge_index").reshape(2, -1)[::-1])


def test_dataloader_with_workers(tmp_path):
    """The loader of the host-fed bench: batch_size trees per item, worker processes, one
    shared-memory buffer per batch (the reference's DataLoader(..., num_workers=5))."""
    store = FD.TreeStore.synthetic(50, 20, seed=5, in_feats=200)
    path = store.save(str(tmp_path / "s"))
    ds = FD.PackedTreeDataset(path)
    loader = torch.utils.data.DataLoader(ds, batch_size=8, shuffle=True, num_workers=2,
                                         collate_fn=FD.host_collate, drop_last=True,
                                         generator=torch.Generator().manual_seed(0))
    seen = []
    for hb in loader:
        assert isinstance(hb, FD.HostBatch) and hb.meta["B"] == 8
        ptr = hb.section("ptr")
        seen.append(int(ptr[-1]))
        assert hb.meta["N"] == int(ptr[-1])
        assert np.array_equal(hb.section("batch"), np.repeat(np.arange(8), np.diff(ptr)))
    assert len(seen) == 6 and sum(seen) <= int(store.tree_node[-1])


def test_bf16_values_round():
    store = FD.TreeStore.synthetic(5, 10, seed=1, in_feats=64)
    store.vals = store.vals * np.float32(1.0 + 2.0 ** -10)    # not bf16-exact
    hb = FD.pack_batch(store, [0, 1], bf16_values=True)
    v = torch.from_numpy(hb.section("x_val").copy())
    assert torch.equal(v, v.to(torch.bfloat16).float())


class _DoneEvent:
    def synchronize(self):
        pass


def test_slot_ring_loader_packs_in_place(tmp_path):
    """host_fed_loader: workers pack each batch straight into a shared slot; only (slot,
    sequence, sizes) cross the worker queue; a slot is reused only after its batch's copy
    (emulated here: the feeder records a completed event per slot)."""
    store = FD.TreeStore.synthetic(60, 15, seed=8, in_feats=100)
    path = store.save(str(tmp_path / "s"))
    loader = FD.host_fed_loader(path, batch_size=4, num_workers=2, shuffle=False, prefetch_factor=2)
    ring = loader.dataset.ring
    assert ring.nslots == 8 and ring.slot_bytes >= FD.pack_batch(store, range(56, 60)).meta["bytes"]
    for epoch in range(2):   # > nslots batches per epoch: every slot is reused
        for k, hb in enumerate(loader):
            assert hb.buf is None and hb.slot == hb.seq % ring.nslots and hb.seq == k
            ref = FD.pack_batch(store, range(4 * k, 4 * k + 4))
            assert hb.meta == ref.meta
            view = FD.HostBatch(ring.slot(hb.slot)[:hb.meta["bytes"]], hb.meta, hb.root_tweetids)
            for name in ref.meta["layout"]:
                assert np.array_equal(view.section(name), ref.section(name)), name
            ring.events[hb.slot], ring.seqs[hb.slot] = _DoneEvent(), hb.seq
    # a feeder that never copies a batch out: the sampler refuses to overwrite it
    ring.seqs = [-1] * ring.nslots
    with pytest.raises(RuntimeError, match="slot ring too small"):
        for hb in loader:
            pass


def test_slot_ring_loader_break_and_reiterate(tmp_path):
    """A `break` out of a pass (early stopping, islice) and a new pass over the same
    persistent-worker loader: the batches the DataLoader discarded at its reset never had
    their copies issued, and the new pass must not wait for them (it starts from an empty
    ring, sequence numbers from 0)."""
    store = FD.TreeStore.synthetic(60, 15, seed=9, in_feats=100)
    loader = FD.host_fed_loader(store, batch_size=4, num_workers=2, shuffle=False, prefetch_factor=2)
    ring = loader.dataset.ring
    for k, hb in enumerate(loader):
        ring.events[hb.slot], ring.seqs[hb.slot] = _DoneEvent(), hb.seq
        if k == 2:
            break
    seen = []
    for k, hb in enumerate(loader):
        assert hb.seq == k
        ref = FD.pack_batch(store, range(4 * k, 4 * k + 4))
        view = FD.HostBatch(ring.slot(hb.slot)[:hb.meta["bytes"]], hb.meta, hb.root_tweetids)
        assert np.array_equal(view.section("x_col"), ref.section("x_col"))
        ring.events[hb.slot], ring.seqs[hb.slot] = _DoneEvent(), hb.seq
        seen.append(k)
    assert seen == list(range(15))


def test_store_rejects_bad_feature_columns():
    rows = [(np.array([3, 7]), np.array([1.0, 2.0], np.float32))]
    tree = {"x_rows": rows, "edges": np.zeros((2, 0), np.int64), "rootindex": 0, "y": 0}
    FD.TreeStore.from_trees([tree], in_feats=8)
    with pytest.raises(ValueError, match="outside"):
        FD.TreeStore.from_trees([tree], in_feats=7)
    dup = dict(tree, x_rows=[(np.array([3, 3]), np.array([1.0, 2.0], np.float32))])
    with pytest.raises(ValueError, match="repeated"):
        FD.TreeStore.from_trees([dup], in_feats=8)
    store = FD.TreeStore.synthetic(4, 10, seed=2, in_feats=64)
    store.in_feats = 32          # a store whose columns reach past in_feats
    with pytest.raises(ValueError, match="outside"):
        FD.pack_batch(store, [0, 1, 2, 3])


@pytest.mark.parametrize("bf16", [False, True])
def test_native_loader_bytes_equal_pack_batch(tmp_path, bf16):
    """The native loader (libbgcn's bgcn_loader_*: C++ threads collating into slots) packs
    every batch byte for byte as pack_batch does (sections, offsets, sizes, bf16 rounding),
    hands them out in order, and each epoch visits every tree once in a fresh order - on a
    saved, memory-mapped store with rows over the ELL cap."""
    eids = _npz_trees(tmp_path, count=9)
    st = FD.TreeStore.from_npz_dir(str(tmp_path), eids, in_feats=64)
    st = FD.TreeStore.load(st.save(str(tmp_path / "store")), mmap=True)
    big = FD.TreeStore.synthetic(200, 40, seed=5, in_feats=5000, num_classes=4)
    for store, bs in ((st, 4), (big, 16)):
        L = FD.NativeLoader(store, batch_size=bs, num_workers=3, seed=11, epochs=3, pinned=False,
                            bf16_values=bf16, drop_last=True)
        per = len(store) // bs
        assert len(L) == 3 * per
        got = []
        while True:
            hb = L.next_host()
            if hb is None:
                break
            ref = FD.pack_batch(store, L.last_trees, bf16_values=bf16)
            assert hb.meta["layout"] == ref.meta["layout"]
            for k in ("N", "B", "nnz", "Etd", "Ebu", "nnz_max", "spill", "bytes"):
                assert hb.meta[k] == ref.meta[k], k
            for name, _ in FD._SECTIONS:
                assert np.array_equal(hb.section(name), ref.section(name)), name
            assert np.array_equal(hb.root_tweetids, np.asarray(store.root_tweetid)[L.last_trees])
            got.append(L.last_trees)
        assert len(got) == 3 * per
        for e in range(3):   # every tree at most once per epoch, all of the kept batches distinct
            ep = np.concatenate(got[e * per:(e + 1) * per])
            assert len(np.unique(ep)) == ep.size == per * bs
        assert not all(np.array_equal(a, b) for a, b in zip(got[:per], got[per:2 * per]))
        L.close()


def test_native_loader_order_and_indices():
    """shuffle=False keeps the given tree order; indices restrict the dataset; a bad index
    is refused; the same seed gives the same batches."""
    st = FD.TreeStore.synthetic(40, 20, seed=2, in_feats=64, num_classes=4)
    idx = np.arange(5, 35)
    L = FD.NativeLoader(st, batch_size=7, num_workers=2, shuffle=False, drop_last=False, indices=idx, pinned=False)
    out = []
    while (hb := L.next_host()) is not None:
        out.append(L.last_trees)
    assert np.array_equal(np.concatenate(out), idx) and [len(o) for o in out] == [7, 7, 7, 7, 2]
    assert L.exhausted and L.next_host() is None      # one pass per loader
    ls = L.stats()                                    # bgcn_loader_get_stats (ABI 12)
    assert ls["packs"] == 5 and ls["threads"] == 2 and ls["pack_ms_per_batch"] >= 0.0
    assert ls["copy_call_ms_per_batch"] == 0.0       # host-only: no copies issued
    assert L.stats(reset=True)["packs"] == 5 and L.stats()["packs"] == 0
    assert not L.wait()                               # bgcn_loader_wait: past the last batch
    L.close()
    L = FD.NativeLoader(FD.TreeStore.synthetic(16, 10, seed=3, in_feats=64, num_classes=4),
                        batch_size=4, num_workers=2, shuffle=False, pinned=False)
    assert L.wait() and L.wait()                      # waits for batch 0 without taking it
    assert L.next_host() is not None and L.last_trees.tolist() == [0, 1, 2, 3]
    L.close()
    with pytest.raises(Exception):
        FD.NativeLoader(st, batch_size=4, indices=[0, 40], pinned=False)
    runs = []
    for _ in range(2):
        L = FD.NativeLoader(st, batch_size=8, num_workers=4, seed=99, pinned=False)
        runs.append([L.next_host() and L.last_trees for _ in range(len(L))])
        L.close()
    assert all(np.array_equal(a, b) for a, b in zip(*runs))


def test_prepare_ahead_order_and_slots(monkeypatch):
    """prepare_ahead hands out every batch in order, queues batch k+1's preparation before it
    hands out batch k (so it runs beside step k), and takes the buffers in turn (a slot is
    reused two batches later, after the caller has queued the step that read it)."""
    from bigcn_amd.feed import prepare_ahead
    log = []
    monkeypatch.setattr(prepare_ahead, "_launch", lambda self, data, slot: log.append(("prep", data, slot)))
    pa = prepare_ahead(range(5), model=None)
    for b in pa:
        log.append(("use", b))
    assert log == [("prep", 0, 0), ("prep", 1, 1), ("use", 0), ("prep", 2, 0), ("use", 1), ("prep", 3, 1),
                   ("use", 2), ("prep", 4, 0), ("use", 3), ("use", 4)]
    log.clear()
    assert list(prepare_ahead([], model=None)) == [] and log == []
    assert list(prepare_ahead([7], model=None)) == [7] and log == [("prep", 7, 0)]
    log.clear()
    assert list(prepare_ahead(range(4), model=None, slots=3)) == [0, 1, 2, 3]
    assert [s for _, _, s in [e for e in log if e[0] == "prep"]] == [0, 1, 2, 0]
    with pytest.raises(ValueError):
        prepare_ahead([], model=None, slots=1)
