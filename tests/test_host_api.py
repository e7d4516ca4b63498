"""Host-side API contracts that need no GPU: argument validation of the drop-in
modules and the fused step (no kernel is launched)."""
import pytest
import torch

from bigcn_amd import BiGCN, GCNConv, Net
from bigcn_amd.ops import degree_code


def test_degree_on_values_are_validated():
    assert degree_code("col") == 0 and degree_code("row") == 1
    for bad in ("rows", "COL", "target", ""):
        with pytest.raises(ValueError):
            degree_code(bad)
        with pytest.raises(ValueError):
            GCNConv(8, 4, degree_on=bad)
        with pytest.raises(ValueError):
            BiGCN(8, 64, 64, degree_on=bad)


def test_degree_on_is_model_wide():
    m = Net(16, 64, 64, degree_on="row")
    assert m.degree_on == "row"
    convs = (m.TDrumorGCN.conv1, m.TDrumorGCN.conv2, m.BUrumorGCN.conv1, m.BUrumorGCN.conv2)
    assert all(c.degree_on == "row" for c in convs)
    m.degree_on = "col"
    assert all(c.degree_on == "col" for c in convs)
    with pytest.raises(ValueError):
        m.degree_on = "source"
    m.TDrumorGCN.conv2.degree_on = "row"          # edited behind the model's back
    with pytest.raises(ValueError, match="disagree"):
        _ = m.degree_on


def test_fused_step_takes_the_models_degree_convention():
    from bigcn_amd import FusedTrainStep
    m = BiGCN(16, 64, 64, degree_on="row")
    assert FusedTrainStep(m).degree_on == 1
    assert FusedTrainStep(m, degree_on="row").degree_on == 1
    with pytest.raises(ValueError, match="model"):
        FusedTrainStep(m, degree_on="col")


def test_fused_step_bucket_carries_the_status_slot():
    """Layout [early gradients | status slot | conv1 weight gradients]: part a (flat_a)
    holds every gradient the deferred-dW1 step finishes first and the status slot, part b
    (flat_b) exactly the two conv1 weight gradients."""
    from bigcn_amd import FusedTrainStep
    m = BiGCN(16, 64, 64)
    st = FusedTrainStep(m)
    b = st.bucket
    n = sum(p.numel() for p in m.parameters())
    assert b.flag.numel() == 1
    assert b.flat_a.numel() + b.flat_b.numel() == b.flat.numel()
    assert b.flat_a.data_ptr() <= b.flag.data_ptr() < b.flat_a.data_ptr() + 4 * b.flat_a.numel()
    enc = list(m.encoder_params())
    late = {id(enc[0]), id(enc[4])}
    lo, hi = b.flat_b.data_ptr(), b.flat_b.data_ptr() + 4 * b.flat_b.numel()
    for p, v in zip(b.params, b.views()):
        inside = lo <= v.data_ptr() < hi
        assert inside == (id(p) in late), tuple(p.shape)
    assert b.flat_b.numel() == enc[0].numel() + enc[4].numel()
    assert sum(v.numel() for v in b.views()) == n


def test_bucket_views_are_16_byte_aligned():
    """Net's 2-class head bias would misalign every later view of a packed bucket: the
    views start on 16-byte boundaries (float4 paths of the step and the fused Adam), the
    gaps stay zero, reduce_sum fills the views."""
    from bigcn_amd import FusedTrainStep, Net
    m = Net(16, 64, 64)
    st = FusedTrainStep(m)
    b = st.bucket
    assert all(v.data_ptr() % 16 == 0 for v in b.views())
    for p in b.params:
        p.grad = torch.full_like(p, 2.0)
    views = b.reduce_sum()
    assert all(bool((v == 2.0).all()) for v in views)
    assert float(b.flat.sum()) - float(b.flag.sum()) == 2.0 * sum(p.numel() for p in b.params)
