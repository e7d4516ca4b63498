"""GPU parity of the host-fed input path (bigcn_amd.feed).

A batch whose node features cross PCIe as the CSR of their non-zeros (bgcn_batch.x_row_ptr;
the prepare pass fills the ELL / spill pool / CSC of X from it) must train to exactly the
same bits as the same trees with the dense x of the reference (Process/dataset.py:94
``x=torch.tensor(data['x'])``): bit-exact losses, gradients and Adam updates, with device
DropEdge and next-batch prefetch, at the full Twitter15 batch size, with long rows in the
spill pool, and with rows that overflow the pool (the dense fallback from the expanded x)."""
import numpy as np
import pytest
import torch

from bigcn_amd import data as D
from bigcn_amd import feed as FD
from oracle import bigcn_oracle as O

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _dense_batch(store, trees, dtype=torch.float32):
    """The reference-format collated batch of ``trees`` (dense x) from the same store."""
    hb = FD.pack_batch(store, trees)
    t = {name: torch.from_numpy(hb.section(name).copy()) for name in hb.meta["layout"]}
    b = D.Batch(x=torch.from_numpy(store.dense_x(trees)).to(dtype), edge_index=t["edge_index"].view(2, -1),
                BU_edge_index=t["BU_edge_index"].view(2, -1), batch=t["batch"], rootindex=t["rootindex"],
                y=t["y"], ptr=t["ptr"], num_graphs=len(trees))
    b = b.to(DEV)
    nnz = (b.x != 0).sum(1)
    b.set_x_nnz_max(int(nnz.max()), int((nnz - D.SPARSE_CAP).clamp_min(0).sum()))
    return b


def _packed(store, trees, x_dtype=torch.float32):
    hb = FD.pack_batch(store, trees, bf16_values=x_dtype == torch.bfloat16)
    return FD.PackedBatch(hb.buf.to(DEV), hb.meta, hb.root_tweetids, None, x_dtype)


def _model(F, seed, classes=4):
    from bigcn_amd import BiGCN, Net
    p = O.make_params(F, 64, 64, classes, seed=seed)
    m = (BiGCN if classes == 4 else Net)(F, 64, 64).to(DEV)
    m.load_state_dict({k: v.float() for k, v in p.items()})
    m.train()
    return m


def _run(batches, F, classes=4, steps=None, drop=0.2):
    """Full training steps (step + fused Adam) with next-batch prefetch and device DropEdge;
    returns per-step (loss, gradients) and the final parameters."""
    from bigcn_amd import FusedTrainStep
    m = _model(F, 5, classes)
    st = FusedTrainStep(m, tddroprate=drop, budroprate=drop, drop_seed=1234)
    out = []
    n = len(batches) if steps is None else steps
    for k in range(n):
        b = batches[k % len(batches)]
        nxt = batches[(k + 1) % len(batches)] if k + 1 < n else None
        loss = st(b, seed=100 + k, next_data=nxt)
        out.append((loss.clone(), [g.clone() for g in st.grads().values()]))
    torch.cuda.synchronize()
    st.check_status()
    assert st.run_report() == {"status": 0, "invalid_steps": 0}
    return out, [p.detach().clone() for p in m.parameters()]


def _assert_same(a, b):
    (ra, pa), (rb, pb) = a, b
    for (la, ga), (lb, gb) in zip(ra, rb):
        assert torch.equal(la, lb), (float(la), float(lb))
        for x, y in zip(ga, gb):
            assert torch.equal(x, y)
    for x, y in zip(pa, pb):
        assert torch.equal(x, y)


def test_compacted_input_bitwise_equals_dense_full_twitter15():
    """Two full Twitter15-size batches (128 trees of mean 256 nodes, 5000-dim BoW), three
    steps each way: compacted-input steps == dense-x steps, bit for bit."""
    store = FD.TreeStore.synthetic(256, 256, seed=21, in_feats=5000, root_random=True)
    trees = [list(range(0, 128)), list(range(128, 256))]
    dense = [_dense_batch(store, t) for t in trees]
    packed = [_packed(store, t) for t in trees]
    assert all(p.fits_sparse for p in packed)
    _assert_same(_run(dense, 5000, steps=3), _run(packed, 5000, steps=3))


def test_compacted_input_long_rows_in_the_spill_pool():
    """Rows of 40-300 words (the reference caps none, getTwittergraph.py:16-24) go to the
    spill pool from the CSR exactly as from the dense rows."""
    store = FD.TreeStore.synthetic(40, 60, seed=22, in_feats=2000)
    rng = np.random.default_rng(3)
    rows = []
    for t in range(len(store)):
        rows.append([(c, v) for c, v in store.tree_rows(t)])
        for k in rng.choice(len(rows[-1]), size=min(3, len(rows[-1])), replace=False):
            c = np.sort(rng.choice(2000, size=int(rng.integers(33, 300)), replace=False))
            rows[-1][k] = (c, rng.integers(1, 4, size=c.size).astype(np.float32))
    trees = []
    for t in range(len(store)):
        a, b = int(store.tree_edge[t]), int(store.tree_edge[t + 1])
        trees.append({"x_rows": rows[t], "edges": np.asarray(store.edges[:, a:b]), "rootindex": int(store.rootindex[t]),
                      "y": int(store.y[t])})
    long = FD.TreeStore.from_trees(trees, in_feats=2000)
    tr = [list(range(0, 20)), list(range(20, 40))]
    packed = [_packed(long, t) for t in tr]
    assert all(p.fits_sparse and p.meta["spill"] > 0 for p in packed)
    _assert_same(_run([_dense_batch(long, t) for t in tr], 2000, steps=3), _run(packed, 2000, steps=3))


def test_pool_overflow_trains_from_the_expanded_x():
    """A batch whose spill exceeds the pool (over 64 words per row on average) cannot stay
    compacted: FusedTrainStep expands its x on the device (bgcn_csr_to_dense) and takes the
    dense fallback, like the dense batch of the same trees."""
    trees = []
    rng = np.random.default_rng(4)
    for t in range(6):
        n = 5
        rows = []
        for k in range(n):
            c = np.sort(rng.choice(512, size=100, replace=False))
            rows.append((c, rng.integers(1, 4, size=100).astype(np.float32)))
        trees.append({"x_rows": rows, "edges": np.array([[0, 0, 1, 1], [1, 2, 3, 4]]), "rootindex": 0,
                      "y": t % 4})
    store = FD.TreeStore.from_trees(trees, in_feats=512)
    pk = _packed(store, range(6))
    assert not pk.fits_sparse
    _assert_same(_run([_dense_batch(store, range(6))], 512, steps=2), _run([pk], 512, steps=2))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_csr_to_dense(dtype):
    store = FD.TreeStore.synthetic(30, 40, seed=23, in_feats=5000)
    pk = _packed(store, range(30), dtype)
    want = torch.from_numpy(store.dense_x(range(30))).to(dtype)
    assert torch.equal(pk.x.cpu(), want)


def test_bf16_compacted_equals_dense_bf16():
    """The bf16 configuration (Weibo, configs[2]): compacted values are the bf16 x's."""
    store = FD.TreeStore.synthetic(64, 200, seed=24, in_feats=5000, num_classes=2)
    tr = [list(range(32)), list(range(32, 64))]
    dense = [_dense_batch(store, t, torch.bfloat16) for t in tr]
    packed = [_packed(store, t, torch.bfloat16) for t in tr]
    _assert_same(_run(dense, 5000, classes=2, steps=2, drop=0.0),
                 _run(packed, 5000, classes=2, steps=2, drop=0.0))


def test_feeder_end_to_end_matches_dense(tmp_path):
    """DataLoader workers -> shared pinned slots -> H2D on the copy stream -> steps with
    prefetch: the same bits as feeding the dense batches of the same trees in the same
    order; the root tweet ids travel with each batch (dataset.py:99)."""
    store = FD.TreeStore.synthetic(48, 100, seed=25, in_feats=5000)
    path = store.save(str(tmp_path / "store"))
    loader = FD.host_fed_loader(path, batch_size=8, num_workers=2, shuffle=False)
    feeder = FD.DeviceFeeder(loader, DEV, depth=2, timing=True)
    got = list(feeder)
    assert [int(b.num_graphs) for b in got] == [8] * 6
    for k, b in enumerate(got):
        assert np.array_equal(b.root_tweetids, store.root_tweetid[8 * k:8 * k + 8])
    n, mean_bytes, ms = feeder.copy_stats()
    assert n == 6 and mean_bytes > 0 and ms > 0
    dense = [_dense_batch(store, range(8 * k, 8 * k + 8)) for k in range(6)]
    _assert_same(_run(dense, 5000), _run(got, 5000))
    loader.dataset.ring.close()


def test_native_loader_feeder_end_to_end_matches_dense(tmp_path):
    """libbgcn's native loader (C++ collating threads -> page-locked slots -> one H2D copy per
    batch on the copy stream, feed.NativeLoader) through DeviceFeeder, in order: the device
    bytes equal pack_batch's, the steps the same bits as the dense batches of the same trees
    in the same order, the root tweet ids travel with each batch; recycled device buffers are
    never overwritten while a batch (or a view of one) is alive."""
    store = FD.TreeStore.synthetic(48, 100, seed=25, in_feats=5000)
    path = store.save(str(tmp_path / "store"))
    loader = FD.NativeLoader(path, batch_size=8, num_workers=3, shuffle=False, epochs=2, nslots=4)
    feeder = FD.DeviceFeeder(loader, DEV, depth=2, timing=True)
    got = []
    views = []
    for k, b in enumerate(feeder):
        if k < 6:
            got.append(b)
        else:
            views.append(b.y)          # a view kept past its batch's life
    assert [int(b.num_graphs) for b in got] == [8] * 6
    for k, b in enumerate(got):
        assert np.array_equal(b.root_tweetids, store.root_tweetid[8 * k:8 * k + 8])
        ref = FD.pack_batch(store, list(range(8 * k, 8 * k + 8)))
        for name, _ in FD._SECTIONS:
            assert np.array_equal(getattr(b, name).cpu().numpy().reshape(-1), ref.section(name)), name
    torch.cuda.synchronize()
    for k, v in enumerate(views):
        assert torch.equal(v.cpu(), torch.as_tensor(store.y[8 * k:8 * k + 8]))
    n, mean_bytes, ms = feeder.copy_stats()
    assert n == 12 and mean_bytes > 0 and ms > 0
    dense = [_dense_batch(store, range(8 * k, 8 * k + 8)) for k in range(6)]
    _assert_same(_run(dense, 5000), _run(got, 5000))
    # one pass per loader: a second pass over the exhausted loader raises (it used to
    # yield nothing, silently)
    assert loader.exhausted
    with pytest.raises(RuntimeError):
        next(iter(FD.DeviceFeeder(loader, DEV)))
    loader.close()


@pytest.mark.parametrize("bad", ["range", "order", "negative"])
def test_bad_feature_columns_reject_the_step(bad):
    """Host-fed lists are checked on the device: a column outside [0, F), columns out of
    ascending order or a negative row count set status bit 0 (the step is invalid and the
    fused Adam skips it), never an out-of-bounds access."""
    from bigcn_amd import FusedTrainStep
    store = FD.TreeStore.synthetic(16, 40, seed=26, in_feats=1000)
    pk = _packed(store, range(16))
    rp = pk.x_row_ptr
    col = pk.x_col
    r = 7                                            # a row of >= 2 entries
    while int(rp[r + 1] - rp[r]) < 2:
        r += 1
    a = int(rp[r])
    if bad == "range":
        col[a + 1] = 1000 + 17
    elif bad == "order":
        col[a + 1] = col[a]
    else:
        rp[r + 1] = rp[r] - 1
    m = _model(1000, 5)
    before = [p.detach().clone() for p in m.parameters()]
    st = FusedTrainStep(m, tddroprate=0.2, budroprate=0.2, drop_seed=3)
    st(pk, seed=1)
    torch.cuda.synchronize()
    with pytest.raises(IndexError):
        st.check_status()
    assert st.run_report()["invalid_steps"] == 1
    for p, q in zip(m.parameters(), before):
        assert torch.equal(p.detach(), q)           # the update was skipped

