// One training step of the reference loop body up to the optimiser, as ONE host call:
//
//   for Batch_data in train_loader:                          BiGCN_Twitter.py:183
//       out_labels = model(Batch_data)                       :184  (K1 + encoder + head)
//       loss = F.nll_loss(out_labels, Batch_data.y)          :186
//       optimizer.zero_grad(); loss.backward()               :187-188
//
// The weight-independent preparation (DropEdge, K1 = gcn_norm + CSR of TD and BU, the
// ELL / CSC of X) of the NEXT batch runs on the auxiliary lane beside this step's chain.
// The caller's stream forks only once per step: a fork's event record stalls the stream
// ~6 us, so small side reductions (db1, db2, the head's weight gradients) ride as extra
// blocks of launches the chain makes anyway.  The head (fc -> log_softmax -> nll mean,
// BiGCN_Twitter.py:129-130,186) is fused into the readout.  Every parameter gradient is
// written (not accumulated), so the
// caller's buffers can be views of a flat data-parallel bucket; the all-reduce and
// bgcn_adam_step follow.  No host sync anywhere: a bad edge index or label sets a bit
// of *status on the device.
#include "bgcn_internal.h"
#include "bgcn_sparse.h"

namespace bgcn {
namespace {

constexpr int H = 64;


struct StepWs {
  float *h1, *h2, *head, *dhead, *dz, *loss_row, *logp;
  void* enc; size_t enc_bytes;
};

void carve_csr(Carve& c, int64_t cap, int64_t N, bgcn_csr_out* g) {
  g->t_ptr = c.take<int32_t>(size_t(N + 1));
  g->t_row = c.take<int32_t>(size_t(cap));
  g->t_col = c.take<int32_t>(size_t(cap));
  g->t_w = c.take<float>(size_t(cap));
  g->s_ptr = c.take<int32_t>(size_t(N + 1));
  g->s_row = c.take<int32_t>(size_t(cap));
  g->s_col = c.take<int32_t>(size_t(cap));
  g->s_w = c.take<float>(size_t(cap));
}

size_t carve_step(Carve& c, int64_t N, int64_t B, int64_t F, int64_t C, StepWs* w) {
  StepWs t{};
  t.h1 = c.take<float>(size_t(N) * 2 * H);
  t.h2 = c.take<float>(size_t(N) * 2 * H);
  t.head = c.take<float>(size_t(B) * kHeadIn);
  t.dhead = c.take<float>(size_t(B) * kHeadIn);
  t.dz = c.take<float>(size_t(B) * C);
  t.loss_row = c.take<float>(size_t(B));
  t.logp = c.take<float>(size_t(B) * C);   // the evaluation step's log-probabilities (no caller buffer)
  t.enc_bytes = bigcn_ws_size(N, B, F, H);
  t.enc = c.take<char>(t.enc_bytes);
  if (w) *w = t;
  return c.off;
}

bgcn_graph_view view_of(const bgcn_csr_out& g, int64_t cap) {
  return bgcn_graph_view{g.t_ptr, g.t_row, g.t_col, g.t_w, g.s_ptr, g.s_row, g.s_col, g.s_w, cap};
}

int check_batch(const bgcn_batch* b) {
  BGCN_CHECK_ARG(b, "null batch");
  BGCN_CHECK_ARG(b->num_nodes > 0 && b->num_graphs > 0, "bad sizes");
  BGCN_CHECK_ARG(b->td_num_edges >= 0 && b->bu_num_edges >= 0, "bad edge counts");
  BGCN_CHECK_ARG(b->batch && b->rootindex, "null pointer");
  // features: the dense x, or (x == NULL) the host-fed CSR of its non-zeros
  BGCN_CHECK_ARG(b->x || (b->x_row_ptr && b->x_col && b->x_val), "null x (and no compacted features)");
  BGCN_CHECK_ARG((b->td_num_edges == 0 || b->td_edge_index) && (b->bu_num_edges == 0 || b->bu_edge_index),
                 "null edge_index");
  BGCN_CHECK_ARG(b->td_droprate < 1.0 && b->bu_droprate < 1.0, "droprate must be < 1");
  BGCN_CHECK_ARG(b->x_dtype == BGCN_DTYPE_F32 || b->x_dtype == BGCN_DTYPE_BF16, "bad x_dtype");
  BGCN_CHECK_ARG((reinterpret_cast<uintptr_t>(b->x) & 15) == 0, "x must be 16-byte aligned");
  return BGCN_OK;
}

// a batch whose features arrive compacted (bgcn_batch.x_row_ptr) has no dense x: only the
// sparse feature path (BGCN_FEAT_SPARSE, no dense fallback kernels) can train on it
int check_feat_input(const bgcn_batch* b, int feat_mode, int64_t F) {
  if (b->x) return BGCN_OK;
  BGCN_CHECK_ARG(feat_mode == BGCN_FEAT_SPARSE, "compacted features (x == NULL) need feat_mode BGCN_FEAT_SPARSE");
  BGCN_CHECK_ARG(F <= kSparseMaxFeat && b->num_nodes <= kSparseMaxN,
                 "compacted features: in_feats / num_nodes beyond the sparse path (expand with bgcn_csr_to_dense)");
  return BGCN_OK;
}

}  // namespace

size_t carve_prepared(Carve& c, int64_t N, int64_t B, int64_t F, int64_t Etd, int64_t Ebu,
                      Prepared* p) {
  Prepared t{};
  t.td_cap = Etd + N;
  t.bu_cap = Ebu + N;
  carve_csr(c, t.td_cap, N, &t.td);
  carve_csr(c, t.bu_cap, N, &t.bu);
  t.gws_bytes = bgcn_graph_pair_workspace_size(Etd, Ebu, N);
  t.gws = c.take<char>(t.gws_bytes);
  // K1 leaves each orientation's aggregation plan in its graph workspace
  if (p && c.base) graph_pair_plans(t.gws, t.gws_bytes, Etd, Ebu, N, t.plan[0], t.plan[1]);
  t.tree_ptr = c.take<int32_t>(size_t(B + 1));
  t.node_root = c.take<int32_t>(size_t(N));
  t.status = c.take<int32_t>(1);
  const int64_t max_items = N / kChunkItems + B + 1;
  t.item_tree = c.take<int32_t>(size_t(max_items));
  t.item_beg = c.take<int32_t>(size_t(max_items));
  t.item_end = c.take<int32_t>(size_t(max_items));
  t.item_root = c.take<int32_t>(size_t(max_items));
  t.tree_item0 = c.take<int32_t>(size_t(B + 1));
  t.x_flags = c.take<int32_t>(8);
  t.x_nnz = c.take<int32_t>(size_t(N));
  t.x_cols = c.take<int32_t>(size_t(N) * BGCN_SPARSE_CAP);
  t.x_vals = c.take<float>(size_t(N) * BGCN_SPARSE_CAP);
  t.x_ovf_off = c.take<int32_t>(size_t(N));
  t.x_long = c.take<int32_t>(size_t(N));
  t.ovf_cap = N * BGCN_SPARSE_SPILL_PER_ROW;
  t.x_ovf = c.take<uint2>(size_t(t.ovf_cap));
  const int64_t R = (N + kCscRowBlock - 1) / kCscRowBlock;
  t.hist = c.take<int32_t>(size_t(R) * size_t(F));
  t.col_total = c.take<int32_t>(size_t(F));
  t.col_start = c.take<int32_t>(size_t(F));
  t.col_end = c.take<int32_t>(size_t(F));
  t.csc = c.take<uint2>(size_t(N) * (BGCN_SPARSE_CAP + BGCN_SPARSE_SPILL_PER_ROW));
  t.td_drop = c.take<int64_t>(size_t(2 * Etd));
  t.bu_drop = c.take<int64_t>(size_t(2 * Ebu));
  t.dws_bytes = drop_ws_size(B);
  t.dws = c.take<char>(t.dws_bytes);
  if (p) *p = t;
  return c.off;
}

static size_t prepared_size(int64_t N, int64_t B, int64_t F, int64_t Etd, int64_t Ebu) {
  Carve c(nullptr, 0);
  return carve_prepared(c, N, B, F, Etd, Ebu, nullptr) + 256;
}

// The per-op encoder on a batch a data pipeline prepared ahead (bgcn_bigcn_args.prepared):
// the args with the prepared buffer's graphs, ELL of X and tree pointers in place of the
// caller's, then the same forward / backward bodies bgcn_train_step runs on its prepared
// batches (no K1, no pass over X, no CSC build in the call).
int bigcn_prepared_call(const bgcn_bigcn_args* a, void* ws, size_t ws_bytes, hipStream_t s, bool backward) {
  BGCN_CHECK_ARG(a && a->prepared, "null args / prepared buffer");
  const int64_t N = a->num_nodes, B = a->num_graphs, F = a->in_feats;
  BGCN_CHECK_ARG(N > 0 && B > 0 && F > 0 && a->td_num_edges >= 0 && a->bu_num_edges >= 0, "bad sizes");
  BGCN_CHECK_ARG(a->prepared_bytes >= prepared_size(N, B, F, a->td_num_edges, a->bu_num_edges),
                 "prepared buffer too small for these sizes");
  Prepared p;
  Carve cp(const_cast<void*>(a->prepared), a->prepared_bytes);
  carve_prepared(cp, N, B, F, a->td_num_edges, a->bu_num_edges, &p);
  bgcn_bigcn_args e = *a;
  e.td = view_of(p.td, p.td_cap);
  e.bu = view_of(p.bu, p.bu_cap);
  e.x_flags = p.x_flags; e.x_nnz = p.x_nnz; e.x_cols = p.x_cols; e.x_vals = p.x_vals;
  e.tree_ptr = p.tree_ptr;
  if (backward) return bigcn_backward_impl(&e, ws, ws_bytes, s, &p, false);
  return bigcn_forward_impl(&e, ws, ws_bytes, s, -1, nullptr, &p);
}

// gs: stream of the graph build (K1); the caller joins it before the graphs are used
static int prepare_into(const bgcn_batch* b, int64_t F, int degree_on, int feat_mode, void* buf,
                        size_t bytes, hipStream_t s, Prepared* out, hipStream_t gs, int lanes = 0) {
  BGCN_TRY(check_batch(b));
  BGCN_CHECK_ARG(F > 0 && F % 4 == 0 && b->ldx >= F && b->ldx % 4 == 0, "bad in_feats / ldx");
  const int64_t N = b->num_nodes, B = b->num_graphs;
  BGCN_CHECK_ARG(buf && bytes >= prepared_size(N, B, F, b->td_num_edges, b->bu_num_edges),
                 "prepared buffer too small");
  Prepared p;
  Carve c(buf, bytes);
  carve_prepared(c, N, B, F, b->td_num_edges, b->bu_num_edges, &p);
  BGCN_TRY(check_feat_input(b, feat_mode, F));
  const int mode = (feat_mode == BGCN_FEAT_DENSE || F > kSparseMaxFeat || N > kSparseMaxN) ? 1 : 0;
  // one stream: the six merged launches (DropEdge, K1, the pass over X and the CSC of X
  // side by side, bgcn_sparse.hip prep_pipeline).  BGCN_PREP_MERGED=0 (read per call)
  // selects the separate launches for A/B runs: the pass over X first (beside the
  // forward, whose gathers are L2-served, it costs the chain less than beside the
  // backward: 0.322 vs 0.329 ms per step), then DropEdge and K1, then the CSC.
  const char* me = std::getenv("BGCN_PREP_MERGED");
  if (s == gs && !(me && atoi(me) == 0)) {
    BGCN_TRY(prep_pipeline(p, b, F, degree_on, mode, s, true, lanes));
    if (out) *out = p;
    return BGCN_OK;
  }
  BGCN_CHECK_HIP(hipMemsetAsync(p.status, 0, sizeof(int32_t), gs));
  const bool x_first = s == gs;
  if (x_first)
    BGCN_TRY(sparse_prepare(p, N, B, F, mode, b->batch, b->rootindex, b->x, b->x_dtype, b->ldx, s, 1, b));
  const int64_t* td = b->td_edge_index;
  const int64_t* bu = b->bu_edge_index;
  if (b->td_droprate > 0.0 || b->bu_droprate > 0.0) {
    // DropEdge (dataset.py:68-90) in the masked form: dropped edges become self loops,
    // which K1 removes - same graphs as the compacted lists, no kept count on the host
    BGCN_TRY(drop_edges_impl(td, b->td_num_edges, p.td_drop, b->td_num_edges, b->td_droprate, bu,
                             b->bu_num_edges, p.bu_drop, b->bu_num_edges, b->bu_droprate, b->batch,
                             N, B, b->drop_seed, 1, nullptr, p.status, p.dws, p.dws_bytes, gs));
    if (td) td = p.td_drop;
    if (bu) bu = p.bu_drop;
  }
  BGCN_TRY(bgcn_build_graph_pair(td, b->td_num_edges, bu, b->bu_num_edges, N, degree_on, &p.td,
                                 &p.bu, b->batch, p.status, p.gws, p.gws_bytes,
                                 reinterpret_cast<bgcn_stream_t>(gs)));
  BGCN_TRY(sparse_prepare(p, N, B, F, mode, b->batch, b->rootindex, b->x, b->x_dtype, b->ldx, s,
                          x_first ? 2 : 3, b));
  if (out) *out = p;
  return BGCN_OK;
}

static int train_step_body(const bgcn_step_args* a, const Prepared& p, StepWs& w, hipStream_t s,
                           int graph_lane);

// bgcn_step_args.adam as the tail's fused form: its tensors must be exactly the ten step
// parameters (gradient pointers = the step's grads, torch's sizes), its images the step's
static bool tail_adam_args(const bgcn_step_args* a, const WeightImages* img, TailAdam& t) {
  const bgcn_adam_args* A = a->adam;
  const int64_t F = a->in_feats, C = a->num_classes;
  if (!A || A->count != kStepParams) return false;
  const int64_t want[kStepParams] = {H * F, H, H * (H + F), H, H * F, H, H * (H + F), H, C * 4 * H, C};
  for (int k = 0; k < kStepParams; ++k) {
    int j = 0;
    while (j < A->count && A->t[j].param != a->params[k]) ++j;
    if (j == A->count || A->t[j].grad != a->grads[k] || A->t[j].numel != want[k]) return false;
    t.p[k] = A->t[j].param;
    t.m[k] = A->t[j].exp_avg;
    t.v[k] = A->t[j].exp_avg_sq;
    t.g[k] = A->t[j].grad;
    t.lr[k] = A->t[j].lr;
    t.n[k] = want[k];
  }
  if (A->images) {
    if (A->images != a->images || A->images_in_feats != F || !img) return false;
    t.w1t = img->w1t;
    t.w2t = img->w2t;
    t.w2s = img->w2s;
    t.w2d = img->w2d;
  }
  t.b1 = A->beta1; t.b2 = A->beta2; t.wd = A->weight_decay; t.eps = A->eps;
  t.bc1 = A->bias_correction1; t.bc2s = A->bias_correction2_sqrt; t.gs = A->grad_scale;
  t.skip_flag = A->skip_flag;
  t.skip_count = A->skip_count;
  t.on = 1;
  return true;
}

size_t train_step_ws_size(int64_t N, int64_t B, int64_t F, int64_t C, int64_t Etd, int64_t Ebu) {
  (void)Etd; (void)Ebu;
  Carve c(nullptr, 0);
  return carve_step(c, N, B, F, C, nullptr) + 256;
}

int train_step_impl(const bgcn_step_args* a, void* ws, size_t ws_bytes, hipStream_t s) {
  BGCN_CHECK_ARG(a, "null args");
  BGCN_TRY(check_batch(&a->cur));
  const int64_t N = a->cur.num_nodes, B = a->cur.num_graphs, F = a->in_feats, C = a->num_classes;
  BGCN_CHECK_ARG(F > 0, "bad sizes");
  BGCN_TRY(check_feat_input(&a->cur, a->feat_mode, F));
  BGCN_CHECK_ARG(C >= 1 && C <= kMaxClasses, "num_classes must be in [1, 16]");
  BGCN_CHECK_ARG(a->y && a->loss, "null pointer");
  for (int k = 0; k < BGCN_STEP_PARAMS; ++k)
    BGCN_CHECK_ARG(a->params[k] && a->grads[k], "null parameter / gradient pointer");
  BGCN_CHECK_ARG(ws && ws_bytes >= train_step_ws_size(N, B, F, C, 0, 0), "workspace too small");
  BGCN_CHECK_ARG(a->prepared, "a prepared buffer is required (bgcn_prepare_workspace_size)");
  if (a->next) {
    BGCN_TRY(check_batch(a->next));
    BGCN_TRY(check_feat_input(a->next, a->feat_mode, F));
    BGCN_CHECK_ARG(a->next_prepared && a->next_prepared != a->prepared,
                   "next_prepared must be a separate buffer");
  }
  StepWs w;
  Carve c(ws, ws_bytes);
  carve_step(c, N, B, F, C, &w);
  BGCN_CHECK_ARG(c.ok(), "workspace too small");
  BGCN_CHECK_ARG(a->images || !a->images_current, "images_current without an image buffer");
  Prepared p;
  int graph_lane = -1;
  // the previous call's next-batch preparation (this call's batch) must be complete
  // before this stream uses it
  BGCN_TRY(aux_prep_wait(s));

  timing_begin(10, s);   // span classes: 8 next-batch preparation, 9 main chain, 10 step
  timing_begin(9, s);
  if (!a->prepared_ready) {
    // prepare the current batch first; without a next batch to prefetch, its K1 runs on
    // the side lane beside the pass over X (joined before the first propagate)
    hipStream_t g = s;
    if (!a->next) BGCN_TRY(aux_fork(s, kLaneSide, &g));
    BGCN_TRY(prepare_into(&a->cur, F, a->degree_on, a->feat_mode, a->prepared, a->prepared_bytes, s,
                          &p, g));
    if (g != s) graph_lane = kLaneSide;
  } else {
    BGCN_CHECK_ARG(a->prepared_bytes >= prepared_size(N, B, F, a->cur.td_num_edges, a->cur.bu_num_edges),
                   "prepared buffer too small");
    Carve cp(a->prepared, a->prepared_bytes);
    carve_prepared(cp, N, B, F, a->cur.td_num_edges, a->cur.bu_num_edges, &p);
  }
  if (a->next) {
    // the next batch's weight-independent preparation (K1, ELL and CSC of X: the HBM-
    // bound pass) runs on the side lane beside this step's latency-bound chain
    hipStream_t x;
    BGCN_TRY(aux_fork(s, kLaneSide, &x));
    timing_begin(8, x);
    BGCN_TRY(prepare_into(a->next, F, a->degree_on, a->feat_mode, a->next_prepared,
                          a->next_prepared_bytes, x, nullptr, x));
    timing_end(8, x);
    // waited for by the next call, not joined by this one: the step's chain ends without a
    // cross-stream wait (chain alone 197 -> 190 us; beside a preparation the join was
    // free, the side lane ends first)
    BGCN_TRY(aux_prep_done(s));
  }
  BGCN_TRY(train_step_body(a, p, w, s, graph_lane));
  timing_end(10, s);
  return BGCN_OK;
}

static int train_step_body(const bgcn_step_args* a, const Prepared& p, StepWs& w, hipStream_t s,
                           int graph_lane) {
  const int64_t N = a->cur.num_nodes, B = a->cur.num_graphs, F = a->in_feats, C = a->num_classes;
  // (*status is cleared by the forward's prologue)
  bgcn_bigcn_args e{};
  e.x = a->cur.x; e.x_dtype = a->cur.x_dtype;
  e.ldx = a->cur.ldx; e.num_nodes = N; e.num_graphs = B; e.in_feats = F; e.hid = H;
  e.batch = a->cur.batch; e.rootindex = a->cur.rootindex;
  e.td = view_of(p.td, p.td_cap);
  e.bu = view_of(p.bu, p.bu_cap);
  e.td_w1 = a->params[0]; e.td_b1 = a->params[1]; e.td_w2 = a->params[2]; e.td_b2 = a->params[3];
  e.bu_w1 = a->params[4]; e.bu_b1 = a->params[5]; e.bu_w2 = a->params[6]; e.bu_b2 = a->params[7];
  e.training = a->training; e.seed = a->seed; e.keep_words = nullptr;
  e.feat_mode = a->feat_mode;
  e.x_flags = p.x_flags; e.x_nnz = p.x_nnz; e.x_cols = p.x_cols; e.x_vals = p.x_vals;
  e.tree_ptr = p.tree_ptr; e.h1 = w.h1; e.h2 = w.h2; e.head_in = w.head; e.dhead_in = w.dhead;
  e.td_dw1 = a->grads[0]; e.td_db1 = a->grads[1]; e.td_dw2 = a->grads[2]; e.td_db2 = a->grads[3];
  e.bu_dw1 = a->grads[4]; e.bu_db1 = a->grads[5]; e.bu_dw2 = a->grads[6]; e.bu_db2 = a->grads[7];
  e.save_for_backward = 1;
  // forward with the head fused into the readout (fc, log_softmax, NLL row terms, dz,
  // dhead per tree); the prepared batch's K1 status is folded into *status
  const HeadArgs hd{a->params[8], a->params[9], a->y, int(C), a->logp, w.dz, w.loss_row, w.dhead,
                    a->status, p.status, a->feat_mode == BGCN_FEAT_SPARSE ? p.x_flags : nullptr};
  WeightImages im{};
  if (a->images) {
    Carve ci(a->images, bgcn_weight_images_size(F));
    carve_images(ci, F, &im);
  }
  const WeightImages* img = a->images ? &im : nullptr;
  BGCN_TRY(bigcn_forward_impl(&e, w.enc, w.enc_bytes, s, graph_lane, &hd, &p, img, a->images_current != 0));
  // fc weight/bias gradients, the loss mean and the validity flag: extra blocks of the
  // readout backward (joins the side lane at its end; with a next-batch preparation on
  // the side lane the dW2 chain stays on this stream, which balances the two)
  const HeadGradJob hj{w.head, w.dz, B, int(C), w.loss_row, a->grads[8], a->grads[9], a->loss,
                       a->status, a->status_flag, a->status_seen};
  TailAdam ta;
  const bool fuse = a->adam && !a->defer_dw1 && tail_adam_args(a, img, ta);
  bool done = false;
  BGCN_TRY(bigcn_backward_impl(&e, w.enc, w.enc_bytes, s, &p, a->next != nullptr, &hj, img, a->defer_dw1 != 0,
                               fuse ? &ta : nullptr, &done));
  // the optimiser step the tail did not take: its own launch (same bits)
  if (a->adam && !done) {
    BGCN_CHECK_ARG(!a->defer_dw1, "adam with defer_dw1: the update needs dW1 (run bgcn_adam_step after "
                                  "bgcn_train_step_dw1)");
    const int rc = bgcn_adam_step(a->adam, reinterpret_cast<bgcn_stream_t>(s));
    if (rc != BGCN_OK) return rc;
  }
  return BGCN_OK;
}

// One evaluation step (the test loop body, BiGCN_Twitter.py:207-222: model.eval();
// val_out = model(Batch_data); val_loss = F.nll_loss(val_out, y); val_pred = argmax;
// correct = val_pred.eq(y).sum()) as one call: the prepared batch's forward in eval mode
// (no dropout; the batch carries no DropEdge), the head fused into the readout, then the
// loss mean, the predictions and the correct count on the device.  No backward, no host
// sync; the next batch's preparation rides on the side lane as in the training step.
int eval_step_impl(const bgcn_step_args* a, int32_t* correct, int64_t* pred, void* ws, size_t ws_bytes,
                   hipStream_t s) {
  BGCN_CHECK_ARG(a, "null args");
  BGCN_TRY(check_batch(&a->cur));
  const int64_t N = a->cur.num_nodes, B = a->cur.num_graphs, F = a->in_feats, C = a->num_classes;
  BGCN_CHECK_ARG(F > 0, "bad sizes");
  BGCN_TRY(check_feat_input(&a->cur, a->feat_mode, F));
  BGCN_CHECK_ARG(C >= 1 && C <= kMaxClasses, "num_classes must be in [1, 16]");
  BGCN_CHECK_ARG(a->y && a->loss, "null pointer");
  BGCN_CHECK_ARG(a->training == 0, "the evaluation step runs in eval mode (training = 0)");
  BGCN_CHECK_ARG(a->cur.td_droprate == 0.0 && a->cur.bu_droprate == 0.0,
                 "the evaluation step drops no edges (the test set's BiGraphDataset)");
  for (int k = 0; k < BGCN_STEP_PARAMS; ++k) BGCN_CHECK_ARG(a->params[k], "null parameter pointer");
  BGCN_CHECK_ARG(ws && ws_bytes >= train_step_ws_size(N, B, F, C, 0, 0), "workspace too small");
  BGCN_CHECK_ARG(a->prepared, "a prepared buffer is required (bgcn_prepare_workspace_size)");
  if (a->next) {
    BGCN_TRY(check_batch(a->next));
    BGCN_TRY(check_feat_input(a->next, a->feat_mode, F));
    BGCN_CHECK_ARG(a->next_prepared && a->next_prepared != a->prepared, "next_prepared must be a separate buffer");
  }
  StepWs w;
  Carve c(ws, ws_bytes);
  carve_step(c, N, B, F, C, &w);
  BGCN_CHECK_ARG(c.ok(), "workspace too small");
  BGCN_CHECK_ARG(a->images || !a->images_current, "images_current without an image buffer");
  Prepared p;
  int graph_lane = -1;
  BGCN_TRY(aux_prep_wait(s));
  if (!a->prepared_ready) {
    hipStream_t g = s;
    if (!a->next) BGCN_TRY(aux_fork(s, kLaneSide, &g));
    BGCN_TRY(prepare_into(&a->cur, F, a->degree_on, a->feat_mode, a->prepared, a->prepared_bytes, s, &p, g));
    if (g != s) graph_lane = kLaneSide;
  } else {
    BGCN_CHECK_ARG(a->prepared_bytes >= prepared_size(N, B, F, a->cur.td_num_edges, a->cur.bu_num_edges),
                   "prepared buffer too small");
    Carve cp(a->prepared, a->prepared_bytes);
    carve_prepared(cp, N, B, F, a->cur.td_num_edges, a->cur.bu_num_edges, &p);
  }
  if (a->next) {
    hipStream_t x;
    BGCN_TRY(aux_fork(s, kLaneSide, &x));
    BGCN_TRY(prepare_into(a->next, F, a->degree_on, a->feat_mode, a->next_prepared, a->next_prepared_bytes, x,
                          nullptr, x));
    BGCN_TRY(aux_prep_done(s));
  }
  bgcn_bigcn_args e{};
  e.x = a->cur.x; e.x_dtype = a->cur.x_dtype;
  e.ldx = a->cur.ldx; e.num_nodes = N; e.num_graphs = B; e.in_feats = F; e.hid = H;
  e.batch = a->cur.batch; e.rootindex = a->cur.rootindex;
  e.td = view_of(p.td, p.td_cap);
  e.bu = view_of(p.bu, p.bu_cap);
  e.td_w1 = a->params[0]; e.td_b1 = a->params[1]; e.td_w2 = a->params[2]; e.td_b2 = a->params[3];
  e.bu_w1 = a->params[4]; e.bu_b1 = a->params[5]; e.bu_w2 = a->params[6]; e.bu_b2 = a->params[7];
  e.training = 0; e.seed = 0; e.keep_words = nullptr;
  e.feat_mode = a->feat_mode;
  e.x_flags = p.x_flags; e.x_nnz = p.x_nnz; e.x_cols = p.x_cols; e.x_vals = p.x_vals;
  e.tree_ptr = p.tree_ptr; e.h1 = w.h1; e.h2 = w.h2; e.head_in = w.head; e.dhead_in = w.dhead;
  e.save_for_backward = 0;
  float* logp = a->logp ? a->logp : w.logp;
  const HeadArgs hd{a->params[8], a->params[9], a->y, int(C), logp, w.dz, w.loss_row, w.dhead,
                    a->status, p.status, a->feat_mode == BGCN_FEAT_SPARSE ? p.x_flags : nullptr};
  WeightImages im{};
  if (a->images) {
    Carve ci(a->images, bgcn_weight_images_size(F));
    carve_images(ci, F, &im);
  }
  BGCN_TRY(bigcn_forward_impl(&e, w.enc, w.enc_bytes, s, graph_lane, &hd, &p, a->images ? &im : nullptr,
                              a->images_current != 0));
  return eval_finish_impl(w.loss_row, logp, a->y, B, int(C), a->loss, correct, pred, a->status, a->status_seen, s);
}

// the encoder arguments of a step (the dW1 call re-derives them from the same inputs)
static void step_encoder_args(const bgcn_step_args* a, const Prepared& p, const StepWs& w, bgcn_bigcn_args* e) {
  *e = bgcn_bigcn_args{};
  e->x = a->cur.x; e->x_dtype = a->cur.x_dtype;
  e->ldx = a->cur.ldx; e->num_nodes = a->cur.num_nodes; e->num_graphs = a->cur.num_graphs;
  e->in_feats = a->in_feats; e->hid = H;
  e->batch = a->cur.batch; e->rootindex = a->cur.rootindex;
  e->td = view_of(p.td, p.td_cap);
  e->bu = view_of(p.bu, p.bu_cap);
  e->td_w1 = a->params[0]; e->td_b1 = a->params[1]; e->td_w2 = a->params[2]; e->td_b2 = a->params[3];
  e->bu_w1 = a->params[4]; e->bu_b1 = a->params[5]; e->bu_w2 = a->params[6]; e->bu_b2 = a->params[7];
  e->training = a->training; e->seed = a->seed; e->keep_words = nullptr;
  e->feat_mode = a->feat_mode;
  e->x_flags = p.x_flags; e->x_nnz = p.x_nnz; e->x_cols = p.x_cols; e->x_vals = p.x_vals;
  e->tree_ptr = p.tree_ptr; e->h1 = w.h1; e->h2 = w.h2; e->head_in = w.head; e->dhead_in = w.dhead;
  e->td_dw1 = a->grads[0]; e->td_db1 = a->grads[1]; e->td_dw2 = a->grads[2]; e->td_db2 = a->grads[3];
  e->bu_dw1 = a->grads[4]; e->bu_db1 = a->grads[5]; e->bu_dw2 = a->grads[6]; e->bu_db2 = a->grads[7];
  e->save_for_backward = 1;
}

int train_step_dw1_impl(const bgcn_step_args* a, void* ws, size_t ws_bytes, hipStream_t s) {
  BGCN_CHECK_ARG(a, "null args");
  BGCN_TRY(check_batch(&a->cur));
  const int64_t N = a->cur.num_nodes, B = a->cur.num_graphs, F = a->in_feats, C = a->num_classes;
  BGCN_CHECK_ARG(a->defer_dw1, "bgcn_train_step_dw1 follows a step run with defer_dw1 = 1");
  BGCN_CHECK_ARG(a->grads[0] && a->grads[4], "null gradient pointer");
  BGCN_CHECK_ARG(ws && ws_bytes >= train_step_ws_size(N, B, F, C, 0, 0), "workspace too small");
  BGCN_CHECK_ARG(a->prepared && a->prepared_bytes >= prepared_size(N, B, F, a->cur.td_num_edges, a->cur.bu_num_edges),
                 "prepared buffer too small");
  StepWs w;
  Carve c(ws, ws_bytes);
  carve_step(c, N, B, F, C, &w);
  Prepared p;
  Carve cp(a->prepared, a->prepared_bytes);
  carve_prepared(cp, N, B, F, a->cur.td_num_edges, a->cur.bu_num_edges, &p);
  bgcn_bigcn_args e;
  step_encoder_args(a, p, w, &e);
  WeightImages im{};
  if (a->images) {
    Carve ci(a->images, bgcn_weight_images_size(F));
    carve_images(ci, F, &im);
  }
  return bigcn_backward_dw1(&e, w.enc, w.enc_bytes, s, &p, a->images ? &im : nullptr);
}

}  // namespace bgcn

extern "C" size_t bgcn_prepare_workspace_size(int64_t num_nodes, int64_t num_graphs, int64_t in_feats,
                                              int64_t td_num_edges, int64_t bu_num_edges) {
  return bgcn::prepared_size(num_nodes, num_graphs, in_feats, td_num_edges, bu_num_edges);
}

extern "C" int bgcn_prepare_batch(const bgcn_batch* batch, int64_t in_feats, int32_t degree_on,
                                  int32_t feat_mode, void* prepared, size_t prepared_bytes,
                                  bgcn_stream_t stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // one lane: a caller of this entry point already runs it off its critical path (e.g.
  // feed.prepare_ahead's side stream beside a host-bound per-op loop); forking the graph
  // build onto a second lane cost that caller's thread ~40 us of host time per batch
  // (two event records and waits) for no gain it could see (profiles/r06_prep_lanes_dropin.txt)
  return bgcn::prepare_into(batch, in_feats, degree_on, feat_mode, prepared, prepared_bytes, s, nullptr, s, 1);
}

extern "C" size_t bgcn_train_step_workspace_size(int64_t num_nodes, int64_t num_graphs,
                                                 int64_t in_feats, int64_t num_classes,
                                                 int64_t td_num_edges, int64_t bu_num_edges) {
  return bgcn::train_step_ws_size(num_nodes, num_graphs, in_feats, num_classes, td_num_edges,
                                  bu_num_edges);
}

extern "C" int bgcn_train_step_saved(void* workspace, size_t workspace_bytes, int64_t num_nodes,
                                     int64_t num_graphs, int64_t in_feats, int64_t num_classes, float** h1,
                                     float** h2) {
  using namespace bgcn;
  BGCN_CHECK_ARG(num_nodes > 0 && num_graphs > 0 && in_feats > 0 && num_classes >= 1, "bad sizes");
  BGCN_CHECK_ARG(workspace && h1 && h2 &&
                     workspace_bytes >= train_step_ws_size(num_nodes, num_graphs, in_feats, num_classes, 0, 0),
                 "workspace too small");
  StepWs w;
  Carve c(workspace, workspace_bytes);
  carve_step(c, num_nodes, num_graphs, in_feats, num_classes, &w);
  *h1 = w.h1;
  *h2 = w.h2;
  return BGCN_OK;
}

extern "C" int bgcn_train_step(const bgcn_step_args* args, void* workspace, size_t workspace_bytes,
                               bgcn_stream_t stream) {
  return bgcn::train_step_impl(args, workspace, workspace_bytes,
                               reinterpret_cast<hipStream_t>(stream));
}

extern "C" int bgcn_eval_step(const bgcn_step_args* args, int32_t* correct, int64_t* pred, void* workspace,
                              size_t workspace_bytes, bgcn_stream_t stream) {
  return bgcn::eval_step_impl(args, correct, pred, workspace, workspace_bytes, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int bgcn_train_step_dw1(const bgcn_step_args* args, void* workspace, size_t workspace_bytes,
                                   bgcn_stream_t stream) {
  return bgcn::train_step_dw1_impl(args, workspace, workspace_bytes, reinterpret_cast<hipStream_t>(stream));
}
