"""Training-trajectory parity: twenty consecutive FusedTrainStep updates (device DropEdge
0.2 / 0.2, in-kernel dropout 0.5, the fused three-group Adam) against the fp64 oracle
training from the same initial parameters with torch.optim.Adam on the same batches - the
reference's epoch loop (model/Twitter/BiGCN_Twitter.py:160-189: model -> nll_loss ->
backward -> Adam(lr 5e-4, wd 1e-4, BU convs at lr / 5)) for twenty batches.

The oracle gets the same inputs every step: the DropEdge lists its restatement keeps for the
step's drop seed (O.drop_edges), the in-kernel dropout draw (keep_words) and the kernel's
relu' decisions (from the step's saved H1 / H2; every decision differing from the fp64
sign must be a tie, |h| <= 1e-6 max|h|, as in test_gpu_fullsize).  The two runs then differ
by arithmetic only, and the test measures how that difference grows over the updates.

Bars (fp32 / bf16-split kernels vs fp64):
  * the loss of every step: |a - b| <= 1e-4 * |b|;
  * every gradient of every step: max-scaled 1e-4 (the single-step bar);
  * every parameter after every update: max|a - b| <= 1e-4 * max|b| (max-scaled).
The per-step error growth is written to gpurun_out/parity/trajectory_twitter15.json (kept as
profiles/r05_trajectory_twitter15.json)."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import bigcn_oracle as O
from test_gpu_bigcn import DEV
from test_gpu_fullsize import TIE_WINDOW, _oracle_batch, errors
from test_gpu_train import KEYS, _model

pytestmark = pytest.mark.gpu
TOL = 1e-4
STEPS = 20


def test_twenty_updates_track_the_fp64_oracle():
    from bigcn_amd import FusedTrainStep
    from bigcn_amd.data import synth_batch, synth_tree_sizes
    from bigcn_amd.ops import keep_words, unpack_keep
    F, drops = 5000, (0.2, 0.2)
    batches = []
    for s in (51, 52):
        rng = np.random.default_rng(s)
        batches.append(synth_batch(rng, synth_tree_sizes(rng, 32, 128), F, 4, 0.0, 0.0, device=DEV))
    p = O.make_params(F, 64, 64, 4, seed=61)
    m = _model(p)
    m.train()
    st = FusedTrainStep(m, tddroprate=drops[0], budroprate=drops[1], drop_seed=9100)
    q = {k: v.double().clone().requires_grad_(True) for k, v in p.items()}
    opt = O.make_optimizer(q)
    rows = []
    for k in range(STEPS):
        b = batches[k % 2]
        seed = 500 + k
        loss = st(b, seed=seed)
        grads = [st.grads()[prm].detach().clone().cpu() for prm in st.step_params]
        h1, h2 = (t.clone().cpu() for t in st.saved_activations())
        torch.cuda.synchronize()
        st.check_status()
        N = b.x.size(0)
        mk = unpack_keep(keep_words(seed, N, F, DEV), 64 + F).cpu()
        ref = _oracle_batch(b, drops, st.last_drop_seed)
        masks = {d: (h1[:, 64 * j:64 * (j + 1)] > 0, h2[:, 64 * j:64 * (j + 1)] > 0)
                 for j, d in enumerate(("TDrumorGCN", "BUrumorGCN"))}
        stages = {}
        logp = O.bigcn_forward(q, ref.x.double().cpu(), ref.edge_index.cpu(), ref.BU_edge_index.cpu(),
                               ref.batch.cpu(), ref.rootindex.cpu(), True, mk[0], mk[1], "col", stages, masks)
        rloss = O.bigcn_loss(logp, ref.y.cpu())
        opt.zero_grad()
        rloss.backward()
        rgrads = {key: q[key].grad.detach().clone() for key in KEYS}
        opt.step()
        # relu' decisions that differ from the fp64 sign are ties
        for j, d in enumerate(("TDrumorGCN", "BUrumorGCN")):
            for name, mine in (("h1", h1), ("h2", h2)):
                r = stages[f"{d}.{name}"]
                got = mine[:, 64 * j:64 * (j + 1)]
                flip = (got > 0) != (r > 0)
                if bool(flip.any()):
                    depth = float(r[flip].abs().max() / r.abs().max())
                    assert depth <= TIE_WINDOW, f"step {k} {d}.{name}: relu' flip at {depth:.2e} of max|h|"
        row = {"step": k, "N": N, "loss": float(rloss), "loss_rel": abs(float(loss) - float(rloss)) / abs(float(rloss))}
        row["grads"] = {key: errors(g, rgrads[key])[0] for key, g in zip(KEYS, grads)}
        sd = m.state_dict()
        row["params"] = {key: errors(sd[key], q[key].detach())[0] for key in KEYS}
        rows.append(row)
        del mk, stages, logp
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "parity")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "trajectory_twitter15.json"), "w") as f:
        json.dump({"what": "FusedTrainStep x20 (device DropEdge, in-kernel dropout, fused Adam) vs the fp64 oracle "
                           "with torch Adam: per step the relative loss error and the max-scaled errors of every "
                           "gradient and of every parameter after the update", "tol": TOL, "rows": rows}, f, indent=1)
    print()
    for r in rows:
        print(f"step {r['step']:2d} loss {r['loss']:.5f} rel {r['loss_rel']:.1e}  grad max {max(r['grads'].values()):.1e}"
              f"  param max {max(r['params'].values()):.1e}")
    for r in rows:
        assert r["loss_rel"] <= TOL, r
        bad = {key: v for key, v in r["grads"].items() if v > TOL}
        assert not bad, (r["step"], bad)
        bad = {key: v for key, v in r["params"].items() if v > TOL}
        assert not bad, (r["step"], bad)
