// One training step of the reference loop body up to the optimiser, as ONE host call:
//
//   for Batch_data in train_loader:                          BiGCN_Twitter.py:183
//       out_labels = model(Batch_data)                       :184  (K1 + encoder + head)
//       loss = F.nll_loss(out_labels, Batch_data.y)          :186
//       optimizer.zero_grad(); loss.backward()               :187-188
//
// K1 (gcn_norm + CSR of TD and BU) runs on the auxiliary lane, overlapped with the
// encoder's pass over X on the caller's stream; then the CSC of X (same lane) overlaps
// the second half of the forward, and the dW2 chain overlaps dH1 -> dZ1.  The head
// (fc -> log_softmax -> nll mean, BiGCN_Twitter.py:129-130,186) and its backward are
// two small kernels.  Every parameter gradient is written (not accumulated), so the
// caller's buffers can be views of a flat data-parallel bucket; the all-reduce and
// bgcn_adam_step follow.  No host sync anywhere: a bad edge index or label sets a bit
// of *status on the device.
#include "bgcn_internal.h"

namespace bgcn {
namespace {

constexpr int H = 64;


// Weight-side head backward: dW[c][k] = sum_b dz[b][c] head[b][k] (block c < C; 4
// quarters of the trees x 256 k, combined in quarter order) and in block C:
// db[c] = sum_b dz[b][c] and loss = sum_b loss_row[b] / B.  Fixed orders.
__global__ __launch_bounds__(1024) void k_head_wgrad(const float* __restrict__ head,
                                                     const float* __restrict__ dz, int64_t B, int C,
                                                     const float* __restrict__ loss_row,
                                                     float* __restrict__ dW, float* __restrict__ db,
                                                     float* __restrict__ loss) {
  __shared__ float red[4][kHeadIn];
  const int c = blockIdx.x, k = threadIdx.x & 255, q = threadIdx.x >> 8;
  const int64_t bq = (B + 3) / 4, b0 = q * bq, b1 = min<int64_t>(B, b0 + bq);
  if (c < C) {
    float acc = 0.f;
    int64_t b = b0;
    for (; b + 8 <= b1; b += 8) {
      float hv[8], gv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        hv[u] = head[(b + u) * kHeadIn + k];
        gv[u] = dz[(b + u) * C + c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = fmaf(gv[u], hv[u], acc);
    }
    for (; b < b1; ++b) acc = fmaf(dz[b * C + c], head[b * kHeadIn + k], acc);
    red[q][k] = acc;
    __syncthreads();
    if (q == 0) dW[int64_t(c) * kHeadIn + k] = ((red[0][k] + red[1][k]) + red[2][k]) + red[3][k];
    return;
  }
  float* lr = &red[0][0];   // 1024 partial sums of the loss rows
  float acc = 0.f;
  for (int64_t b = threadIdx.x; b < B; b += 1024) acc += loss_row[b];
  lr[threadIdx.x] = acc;
  if (threadIdx.x < C) {
    float s = 0.f;
    for (int64_t b = 0; b < B; ++b) s += dz[b * C + threadIdx.x];
    db[threadIdx.x] = s;
  }
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if (threadIdx.x < o) lr[threadIdx.x] += lr[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) *loss = lr[0] / float(B);
}

struct StepWs {
  bgcn_csr_out td, bu;
  void* gws; size_t gws_bytes;
  int32_t* x_flags; int32_t* x_nnz; int32_t* x_cols; float* x_vals;
  int32_t* tree_ptr;
  float *h1, *h2, *head, *dhead, *dz, *loss_row;
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

size_t carve_step(Carve& c, int64_t N, int64_t B, int64_t F, int64_t C, int64_t Etd, int64_t Ebu,
                  StepWs* w) {
  StepWs t{};
  carve_csr(c, Etd + N, N, &t.td);
  carve_csr(c, Ebu + N, N, &t.bu);
  t.gws_bytes = bgcn_graph_pair_workspace_size(Etd, Ebu, N);
  t.gws = c.take<char>(t.gws_bytes);
  t.x_flags = c.take<int32_t>(8);
  t.x_nnz = c.take<int32_t>(size_t(N));
  t.x_cols = c.take<int32_t>(size_t(N) * BGCN_SPARSE_CAP);
  t.x_vals = c.take<float>(size_t(N) * BGCN_SPARSE_CAP);
  t.tree_ptr = c.take<int32_t>(size_t(B + 1));
  t.h1 = c.take<float>(size_t(N) * 2 * H);
  t.h2 = c.take<float>(size_t(N) * 2 * H);
  t.head = c.take<float>(size_t(B) * kHeadIn);
  t.dhead = c.take<float>(size_t(B) * kHeadIn);
  t.dz = c.take<float>(size_t(B) * C);
  t.loss_row = c.take<float>(size_t(B));
  t.enc_bytes = bigcn_ws_size(N, B, F, H);
  t.enc = c.take<char>(t.enc_bytes);
  if (w) *w = t;
  return c.off;
}

bgcn_graph_view view_of(const bgcn_csr_out& g, int64_t cap) {
  return bgcn_graph_view{g.t_ptr, g.t_row, g.t_col, g.t_w, g.s_ptr, g.s_row, g.s_col, g.s_w, cap};
}

}  // namespace

static int train_step_body(const bgcn_step_args* a, StepWs& w, hipStream_t s);

size_t train_step_ws_size(int64_t N, int64_t B, int64_t F, int64_t C, int64_t Etd, int64_t Ebu) {
  Carve c(nullptr, 0);
  return carve_step(c, N, B, F, C, Etd, Ebu, nullptr) + 256;
}

int train_step_impl(const bgcn_step_args* a, void* ws, size_t ws_bytes, hipStream_t s) {
  BGCN_CHECK_ARG(a, "null args");
  const int64_t N = a->num_nodes, B = a->num_graphs, F = a->in_feats, C = a->num_classes;
  BGCN_CHECK_ARG(N > 0 && B > 0 && F > 0, "bad sizes");
  BGCN_CHECK_ARG(C >= 1 && C <= kMaxClasses, "num_classes must be in [1, 16]");
  BGCN_CHECK_ARG(a->td_num_edges >= 0 && a->bu_num_edges >= 0, "bad edge counts");
  BGCN_CHECK_ARG(a->y && a->loss, "null pointer");
  for (int k = 0; k < BGCN_STEP_PARAMS; ++k)
    BGCN_CHECK_ARG(a->params[k] && a->grads[k], "null parameter / gradient pointer");
  BGCN_CHECK_ARG(ws && ws_bytes >= train_step_ws_size(N, B, F, C, a->td_num_edges, a->bu_num_edges),
                 "workspace too small");
  StepWs w;
  Carve c(ws, ws_bytes);
  carve_step(c, N, B, F, C, a->td_num_edges, a->bu_num_edges, &w);
  BGCN_CHECK_ARG(c.ok(), "workspace too small");
  return train_step_body(a, w, s);
}

static int train_step_body(const bgcn_step_args* a, StepWs& w, hipStream_t s) {
  const int64_t N = a->num_nodes, B = a->num_graphs, F = a->in_feats, C = a->num_classes;
  if (a->status) BGCN_CHECK_HIP(hipMemsetAsync(a->status, 0, sizeof(int32_t), s));

  // K1 for both directions on the side lane (joined by the encoder right after its pass
  // over X, before the CSC of X is queued on the same lane), overlapped with that pass
  hipStream_t g;
  BGCN_TRY(aux_fork(s, kLaneSide, &g));
  BGCN_TRY(bgcn_build_graph_pair(a->td_edge_index, a->td_num_edges, a->bu_edge_index,
                                 a->bu_num_edges, N, a->degree_on, &w.td, &w.bu, a->status, w.gws,
                                 w.gws_bytes, reinterpret_cast<bgcn_stream_t>(g)));

  bgcn_bigcn_args e{};
  e.x = a->x; e.ldx = a->ldx; e.num_nodes = N; e.num_graphs = B; e.in_feats = F; e.hid = H;
  e.batch = a->batch; e.rootindex = a->rootindex;
  e.td = view_of(w.td, a->td_num_edges + N);
  e.bu = view_of(w.bu, a->bu_num_edges + N);
  e.td_w1 = a->params[0]; e.td_b1 = a->params[1]; e.td_w2 = a->params[2]; e.td_b2 = a->params[3];
  e.bu_w1 = a->params[4]; e.bu_b1 = a->params[5]; e.bu_w2 = a->params[6]; e.bu_b2 = a->params[7];
  e.training = a->training; e.seed = a->seed; e.keep_words = nullptr;
  e.feat_mode = a->feat_mode;
  e.x_flags = w.x_flags; e.x_nnz = w.x_nnz; e.x_cols = w.x_cols; e.x_vals = w.x_vals;
  e.tree_ptr = w.tree_ptr; e.h1 = w.h1; e.h2 = w.h2; e.head_in = w.head; e.dhead_in = w.dhead;
  e.td_dw1 = a->grads[0]; e.td_db1 = a->grads[1]; e.td_dw2 = a->grads[2]; e.td_db2 = a->grads[3];
  e.bu_dw1 = a->grads[4]; e.bu_db1 = a->grads[5]; e.bu_dw2 = a->grads[6]; e.bu_db2 = a->grads[7];
  e.save_for_backward = 1;
  // forward with the head fused into the readout (fc, log_softmax, NLL row terms, dz,
  // dhead per tree)
  const HeadArgs hd{a->params[8], a->params[9], a->y, int(C), a->logp, w.dz, w.loss_row, w.dhead,
                    a->status};
  BGCN_TRY(bigcn_forward_impl(&e, w.enc, w.enc_bytes, s, g == s ? -1 : kLaneSide, &hd));
  // fc weight/bias gradients and the loss mean are off the critical path: side lane
  hipStream_t x;
  BGCN_TRY(aux_fork(s, kLaneSide, &x));
  hipLaunchKernelGGL(k_head_wgrad, dim3(unsigned(C + 1)), dim3(1024), 0, x, w.head, w.dz, B, int(C),
                     w.loss_row, a->grads[8], a->grads[9], a->loss);
  BGCN_CHECK_LAUNCH();
  return bigcn_backward_impl(&e, w.enc, w.enc_bytes, s);   // joins the side lane at its end
}

}  // namespace bgcn

extern "C" size_t bgcn_train_step_workspace_size(int64_t num_nodes, int64_t num_graphs,
                                                 int64_t in_feats, int64_t num_classes,
                                                 int64_t td_num_edges, int64_t bu_num_edges) {
  return bgcn::train_step_ws_size(num_nodes, num_graphs, in_feats, num_classes, td_num_edges,
                                  bu_num_edges);
}

extern "C" int bgcn_train_step(const bgcn_step_args* args, void* workspace, size_t workspace_bytes,
                               bgcn_stream_t stream) {
  return bgcn::train_step_impl(args, workspace, workspace_bytes,
                               reinterpret_cast<hipStream_t>(stream));
}
