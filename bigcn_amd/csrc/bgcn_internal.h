// Internal (C++) entry points shared between the libbgcn translation units.
#pragma once

#include "bgcn_common.h"

namespace bgcn {

// ---- K3/K4 aggregation (bgcn_spmm.hip)
struct SpmmProb {
  const int32_t* ptr;
  const int32_t* row;
  const int32_t* col;
  const float* w;
  const float* in;
  int64_t ld_in;
  float* out;
  int64_t ld_out;
  const float* bias;
  float* part;  // [ngroups][2][F] partial rows of chunk-crossing rows
  int64_t ngroups;
  int64_t capacity;  // allocated entries; [ptr[rows], capacity) hold row = -1 (K1 writes them)
  SpmmPlan plan;     // F = 64 only; plan.bnd == nullptr -> merge-path chunks + fixup
};

// Readout-gradient input of the planned F = 64 aggregation (the fused step's dZ2 = A^T dH2
// with the readout backward folded in): when sgn != nullptr, problem d's input row j is
//   dH2_d[j][c] = [H2_d[j][c] > 0] * dhead[b][hoff_d + c] / cnt_b,   b = tree of j,
// (BiGCN_Twitter.py:57,65: relu then scatter_mean; hoff = 2H for TD, 0 for BU: the head
// input is cat(BU, TD), :128) read from the readout's H2 sign words: sgn[j][d] bit 16k + l
// = column 4l + k.  A tree's edges stay inside it, so row i's sum is
//   dZ2_d[i] = (dhead[b(i)][hoff_d ..] / cnt_b(i)) * sum_j w_ij [H2_d[j] > 0].
struct SpmmSign {
  const uint64_t* sgn;       // [rows][2] or nullptr
  const float* dhead;        // [B][kHeadIn]
  const int64_t* batch;      // [rows] node -> tree
  const int32_t* tree_ptr;   // [B + 1]
  int64_t B;
  // per problem (TD, BU): the graph build's status word; BGCN_STATUS_CROSS_TREE set = some
  // neighbour lies in another tree, so each gathered row takes its own tree's scale
  const int32_t* tree_status[2];
};

struct SpmmBatch {
  SpmmProb p[2];
  int64_t rows;
  int F;
  int epi;
  SpmmSign sg;   // sg.sgn != nullptr: readout-gradient input (planned F = 64 path only)
};

int spmm_batch_impl(SpmmBatch& sb, int count, hipStream_t stream);
bool spmm_planned(const SpmmBatch& sb, int count);   // whether the launch takes K1's plans
// the plans K1 left in a graph-pair workspace (bgcn_build_graph_pair layout)
void graph_pair_plans(void* ws, size_t ws_bytes, int64_t Etd, int64_t Ebu, int64_t N, SpmmPlan td[2],
                      SpmmPlan bu[2]);
int64_t spmm_groups(int64_t capacity, int32_t F);
size_t spmm_ws_size(int64_t capacity, int32_t F);
int spmm_impl(const int32_t* ptr, const int32_t* row, const int32_t* col, const float* w,
              int64_t rows, int64_t capacity, const float* in, int64_t ld_in, float* out,
              int64_t ld_out, int32_t F, const float* bias, int epi, void* ws, size_t ws_bytes,
              hipStream_t stream);

// ---- K2/K10 GEMMs (bgcn_gemm.hip)
// gate: see gate_closed() in bgcn_common.h (nullptr = always run)
int gemm_xwt_impl(const float* X, int64_t ldx, const float* W0, const float* W1, int64_t ldw,
                  int64_t split, float* Y, int64_t ldy, int64_t M, int64_t Nc, int64_t K,
                  hipStream_t stream, const int32_t* gate);
int gemm_tn_impl(const float* G, int64_t ldg, const float* X, int64_t ldx, float* C0, float* C1,
                 int64_t ldc, int64_t split, int64_t Mc, int64_t Nc, int64_t K, void* ws,
                 size_t ws_bytes, hipStream_t stream, int timing_cls, const int32_t* gate);
size_t tn_ws_size(int64_t Mc, int64_t Nc, int64_t K);
// the same GEMMs with the node features X as fp32 or bf16 (xdt: BGCN_DTYPE_*)
// fp32 X takes the six-product bf16-MFMA kernels (128-row tiles, about one block per CU)
// only from this many rows on: at PHEME's ~1.2k nodes per batch their 10-20 blocks leave the
// GPU idle, where the f32-MFMA kernels' 64-row tiles run twice the blocks (pheme768 conv2
// 34 vs 56-59 us)
constexpr int64_t kX6MinRows = 8192;
int gemm_xwt_x(const void* X, int xdt, int64_t ldx, const float* W0, const float* W1, int64_t ldw,
               int64_t split, float* Y, int64_t ldy, int64_t M, int64_t Nc, int64_t K,
               hipStream_t stream, const int32_t* gate);
int gemm_tn_x(const float* G, int64_t ldg, const void* X, int xdt, int64_t ldx, float* C0,
              float* C1, int64_t ldc, int64_t split, int64_t Mc, int64_t Nc, int64_t K, void* ws,
              size_t ws_bytes, hipStream_t stream, int timing_cls, const int32_t* gate);
int tn_splits(int64_t Mc, int64_t Nc, int64_t K);

// ---- classifier head fc -> log_softmax -> NLL (BiGCN_Twitter.py:129-130,186) and its
// row-local backward; evaluated per tree by one wave (shared by k_readout_fwd's fused
// form and bgcn_step.hip)
constexpr int kHeadIn = 256;       // cat(BU_x, TD_x)
constexpr int kMaxClasses = 16;
struct HeadArgs {
  const float* W;        // [C, 256] (nullptr: no head)
  const float* bias;     // [C]
  const int64_t* y;      // [B]
  int C;
  float* logp;           // [B, C] or nullptr
  float* dz;             // [B, C] dLoss/dlogits
  float* loss_row;       // [B]
  float* dhead;          // [B, 256]
  int32_t* status;       // bit 1: label out of range
  const int32_t* in_status;  // OR-ed into *status once (prepared batch's K1 flags), or nullptr
  const int32_t* in_xflags;  // BGCN_FEAT_SPARSE: the compaction's overflow flag (-> bit 2)
};

// One wave, row b of the head: h = head_in[b][4l .. 4l+3] held by lane l.
//   z = h W^T + bias ; logp = z - logsumexp(z) ; loss_row = -logp[y] ;
//   dz = (softmax - onehot(y)) / B ; dhead = dz W.  Dot products butterfly-reduced.
// The head's operands (W rows, bias, label) are loaded by head_load, unconditionally
// from clamped rows, so a caller can issue them long before the row is known: loaded
// inside the dependent chain each was one more full memory latency (C + 2 of them).
// MC: classes held in registers (>= hd.C): 4 covers Twitter (4) and Weibo (2) and holds 60
// fewer registers than kMaxClasses
template <int MC = kMaxClasses>
struct HeadRegs {
  float4 w[MC];
  float bias[MC];
  int64_t y;
};
template <int MC>
__device__ inline void head_load(const HeadArgs& hd, int64_t b, HeadRegs<MC>& r) {
  const int l = threadIdx.x & 63;
  const int cm = hd.C - 1;
#pragma unroll
  for (int c = 0; c < MC; ++c) {
    const int cc = c < cm ? c : cm;
    r.w[c] = ld4(hd.W + int64_t(cc) * kHeadIn + 4 * l);
    r.bias[c] = hd.bias[cc];
  }
  r.y = hd.y[b];
}
template <int MC>
__device__ inline void head_row(const HeadArgs& hd, int64_t b, int64_t B, float4 h, const HeadRegs<MC>& r) {
  const int l = threadIdx.x & 63;
  const int C = hd.C;
  float z[MC];
#pragma unroll
  for (int c = 0; c < MC; ++c) {
    z[c] = 0.f;
    if (c < C) {  // C is uniform: the shuffles stay convergent
      const float4 w = r.w[c];
      float p = fmaf(h.x, w.x, fmaf(h.y, w.y, fmaf(h.z, w.z, h.w * w.w)));
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) p += __shfl_xor(p, o);
      z[c] = p + r.bias[c];
    }
  }
  float m = z[0];
#pragma unroll
  for (int c = 1; c < MC; ++c)
    if (c < C) m = fmaxf(m, z[c]);
  float se = 0.f;
#pragma unroll
  for (int c = 0; c < MC; ++c)
    if (c < C) se += expf(z[c] - m);
  const float lse = m + logf(se);
  const int64_t yb = r.y;
  const bool yok = yb >= 0 && yb < C;
  if (!yok && l == 0 && hd.status) atomicOr(hd.status, 2);
  const float inv_b = 1.0f / float(B);
  float4 dh = f4zero();
#pragma unroll
  for (int c = 0; c < MC; ++c) {
    if (c < C) {
      const float lp = z[c] - lse;
      const float g = yok ? (expf(lp) - (c == yb ? 1.f : 0.f)) * inv_b : 0.f;
      if (l == 0) {
        if (hd.logp) hd.logp[b * C + c] = lp;
        hd.dz[b * C + c] = g;
        if (c == yb) hd.loss_row[b] = -lp;
      }
      dh = f4fma(g, r.w[c], dh);
    }
  }
  if (l == 0 && !yok) hd.loss_row[b] = 0.f;
  // the prepared batch's K1 flags: bits 0-3 (BGCN_STATUS_CROSS_TREE is information, the
  // readout backward handles such edges)
  if (l == 0 && b == 0 && hd.in_status && hd.status && (*hd.in_status & 15)) atomicOr(hd.status, *hd.in_status & 15);
  if (l == 0 && b == 0 && hd.in_xflags && hd.status && *hd.in_xflags) atomicOr(hd.status, 4);
  st4(hd.dhead + b * kHeadIn + 4 * l, dh);
}
__device__ inline void head_row(const HeadArgs& hd, int64_t b, int64_t B, float4 h) {
  HeadRegs<kMaxClasses> r;
  head_load(hd, b, r);
  head_row(hd, b, B, h, r);
}

// ---- small reductions carried by extra blocks of a launch the caller's stream makes
// anyway.  Forking them onto the side lane instead costs the caller's stream ~6 us per
// fork (the event record's barrier packet stalls the queue; measured on the step's
// kernel trace), more than the reductions themselves.

// out_td[c] = sum_p part[p][c], out_bu[c] = sum_p part[p][H + c] (c < 64): 16 threads
// per column stride the partials (p = g, g + 16, ...), the 16 group sums are then added
// in group order - a fixed order (deterministic).  Job block jb of kColsumGroups *
// blockDim.x / 16 ... : each block holds blockDim.x / 16 whole columns.
// One Adam element (torch semantics, amsgrad off, L2 weight decay in the gradient):
// bgcn_optim.hip's launch and the step's fused form (TailAdam) share it, so their bits agree.
struct AdamConst {
  float b1, b2, wd, eps, step, inv_bc2, gs;
};
// Every product and sum is spelled out (fmaf / __fmul_rn / __fadd_rn): with contraction
// left to the compiler, the inlined copies fused a * b + c * d differently per call site and
// the fused step's moments drifted an ulp from the separate launch's.
__device__ __forceinline__ void adam_elem(float& p, float gr, float& m, float& v, const AdamConst& c) {
  const float g = fmaf(c.wd, p, __fmul_rn(gr, c.gs));
  m = fmaf(1.0f - c.b1, __fsub_rn(g, m), m);                 // exp_avg.lerp_(grad, 1 - beta1)
  v = fmaf(1.0f - c.b2, __fmul_rn(g, g), __fmul_rn(v, c.b2));   // exp_avg_sq.mul_(beta2).addcmul_(g, g, 1 - beta2)
  const float denom = fmaf(sqrtf(v), c.inv_bc2, c.eps);
  p = fmaf(-c.step, __fdiv_rn(m, denom), p);
}

// The optimiser step fused into the backward's tail launch (bgcn_step_args.adam): per step
// parameter k (bgcn_step_args order: td_w1 td_b1 td_w2 td_b2 bu_w1 bu_b1 bu_w2 bu_b2 fc_w
// fc_b) its Adam state and step size; the images are the step's weight images.
constexpr int kStepParams = 10;
struct TailAdam {
  int on = 0;
  const float* skip_flag = nullptr;
  int32_t* skip_count = nullptr;
  float b1 = 0, b2 = 0, wd = 0, eps = 0, bc1 = 1, bc2s = 1, gs = 0;
  float* p[kStepParams] = {};
  float* m[kStepParams] = {};
  float* v[kStepParams] = {};
  const float* g[kStepParams] = {};
  float lr[kStepParams] = {};
  int64_t n[kStepParams] = {};
  float* w1t = nullptr;      // [F][128]
  float* w2t = nullptr;      // [2][64+F][64]
  __bf16* w2s = nullptr;     // [2][3][64 o][kW2sLd]
  __bf16* w2d = nullptr;     // [2][3][64 c][kW2dLd]
  // (the same expressions as k_adam's constants: the same bits)
  __device__ AdamConst c(int k) const { return AdamConst{b1, b2, wd, eps, lr[k] / bc1, 1.0f / bc2s, gs}; }
  __device__ bool skip() const { return skip_flag && *skip_flag != 0.0f; }
};

struct ColsumJob {
  const float* part;   // [P][128] or nullptr (no job)
  int P;
  float* out_td;
  float* out_bu;
};
constexpr int kColsumGroups = 16;
__host__ __device__ constexpr int colsum_job_blocks(int threads) {
  return 128 * kColsumGroups / threads;
}
// sm: kColsumSmem floats of the caller's shared memory (a merged launch passes its role
// buffer, so the job adds no LDS of its own to the launch)
constexpr int kColsumSmem = kColsumGroups * 64;
__device__ inline void colsum_job_block(const ColsumJob& j, int jb, float* sm, const TailAdam* ad = nullptr) {
  float* red = sm;
  const int cpb = int(blockDim.x) / kColsumGroups;    // columns per block (<= 64)
  const int cl = threadIdx.x % cpb, g = threadIdx.x / cpb;
  const int c = jb * cpb + cl;
  // the fused optimiser step (b1): the parameter's state requested before the sums
  const bool fa = ad && ad->on && g == 0 && !ad->skip();
  const int ka = c < 64 ? 1 : 5, ia = c & 63;
  float ap = 0.f, am = 0.f, av = 0.f;
  if (fa) {
    ap = ad->p[ka][ia];
    am = ad->m[ka][ia];
    av = ad->v[ka][ia];
  }
  float acc = 0.f;
  int p = g;
  for (; p + 3 * kColsumGroups < j.P; p += 4 * kColsumGroups) {   // 4 loads in flight
    const float v0 = j.part[int64_t(p) * 128 + c], v1 = j.part[int64_t(p + kColsumGroups) * 128 + c];
    const float v2 = j.part[int64_t(p + 2 * kColsumGroups) * 128 + c];
    const float v3 = j.part[int64_t(p + 3 * kColsumGroups) * 128 + c];
    acc += v0; acc += v1; acc += v2; acc += v3;
  }
  for (; p < j.P; p += kColsumGroups) acc += j.part[int64_t(p) * 128 + c];
  red[g * cpb + cl] = acc;
  __syncthreads();
  if (g == 0) {
    float s = red[cl];
    for (int q = 1; q < kColsumGroups; ++q) s += red[q * cpb + cl];
    if (c < 64) j.out_td[c] = s; else j.out_bu[c - 64] = s;
    if (fa) {
      adam_elem(ap, s, am, av, ad->c(ka));
      ad->p[ka][ia] = ap;
      ad->m[ka][ia] = am;
      ad->v[ka][ia] = av;
    }
  }
}

// The same sums with one 256-thread block per column (128 blocks): for many partials
// (the readout's per-item db2 partials, ~N/32: 3.3k at Weibo size, where the 16-group
// form above ran 23 us on 8 blocks at the end of the middle launch).  Lane t of the block
// sums partials p = t, t + 256, ...; the 256 lane sums are combined by a fixed
// butterfly in each wave and the four wave sums in wave order (deterministic).
constexpr int kColsumColBlocks = 128;
__device__ inline void colsum_col_block(const ColsumJob& j, int c, float* sm) {
  float acc = 0.f;
  int p = int(threadIdx.x);
  for (; p + 768 < j.P; p += 1024) {   // 4 loads in flight
    const float v0 = j.part[int64_t(p) * 128 + c], v1 = j.part[int64_t(p + 256) * 128 + c];
    const float v2 = j.part[int64_t(p + 512) * 128 + c], v3 = j.part[int64_t(p + 768) * 128 + c];
    acc += v0; acc += v1; acc += v2; acc += v3;
  }
  for (; p < j.P; p += 256) acc += j.part[int64_t(p) * 128 + c];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float s = ((sm[0] + sm[1]) + sm[2]) + sm[3];
    if (c < 64) j.out_td[c] = s; else j.out_bu[c - 64] = s;
  }
}

// Weight side of the classifier head's backward (bgcn_train_step), as C + 1 extra
// 256-thread blocks: block c < C: dW[c][k] = sum_b dz[b][c] head[b][k] (4 quarters of the
// trees x 64 float4 column groups, quarters combined in order); block C: db[c] =
// sum_b dz[b][c] (64 tree slices per class, combined in order), loss = sum_b loss_row[b]
// / B (fixed tree), and the step's validity flag float(status & 15) (every status bit is
// known once the readout / head has run).
struct HeadGradJob {
  const float* head;     // [B, 256] or nullptr (no job)
  const float* dz;       // [B, C]
  int64_t B;
  int C;
  const float* loss_row;  // [B]
  float* dW;             // [C, 256]
  float* db;             // [C]
  float* loss;           // [1]
  const int32_t* status;  // or nullptr
  float* status_flag;    // or nullptr
  int32_t* status_seen = nullptr;   // sticky OR of the step statuses, or nullptr
};
// sm: kHeadGradSmem floats of the caller's shared memory (16-byte aligned)
constexpr int kHeadGradSmem = 4 * 64 * 4 + 256 + kMaxClasses * 64;
__device__ inline void head_grad_block(const HeadGradJob& j, int hb, float* sm) {
  float4 (*r4)[64] = reinterpret_cast<float4 (*)[64]>(sm);
  float* ls = sm + 4 * 64 * 4;
  float (*dbp)[64] = reinterpret_cast<float (*)[64]>(sm + 4 * 64 * 4 + 256);
  const int t = threadIdx.x;
  const int64_t B = j.B;
  const int C = j.C;
  if (hb < C) {
    const int kq = t & 63, q = t >> 6;
    const int64_t bq = (B + 3) / 4, b0 = q * bq, b1 = min<int64_t>(B, b0 + bq);
    float4 acc = f4zero();
    int64_t b = b0;
    for (; b + 8 <= b1; b += 8) {
      float4 hv[8];
      float gv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        hv[u] = ld4(j.head + (b + u) * kHeadIn + 4 * kq);
        gv[u] = j.dz[(b + u) * C + hb];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = f4fma(gv[u], hv[u], acc);
    }
    for (; b < b1; ++b) acc = f4fma(j.dz[b * C + hb], ld4(j.head + b * kHeadIn + 4 * kq), acc);
    r4[q][kq] = acc;
    __syncthreads();
    if (q == 0)
      st4(j.dW + int64_t(hb) * kHeadIn + 4 * kq,
          f4add(f4add(f4add(r4[0][kq], r4[1][kq]), r4[2][kq]), r4[3][kq]));
    return;
  }
  float a = 0.f;
  for (int64_t b = t; b < B; b += 256) a += j.loss_row[b];
  ls[t] = a;
  for (int cc = t >> 6; cc < C; cc += 4) {
    const int sl = t & 63;
    float s = 0.f;
    for (int64_t b = sl; b < B; b += 64) s += j.dz[b * C + cc];
    dbp[cc][sl] = s;
  }
  __syncthreads();
  if (t < C) {
    float s = 0.f;
    for (int q = 0; q < 64; ++q) s += dbp[t][q];
    j.db[t] = s;
  }
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) ls[t] += ls[t + o];
    __syncthreads();
  }
  if (t == 0) {
    *j.loss = ls[0] / float(B);
    const int32_t st = j.status ? *j.status & 15 : 0;
    if (j.status_flag) *j.status_flag = float(st);
    if (j.status_seen && st) atomicOr(j.status_seen, st);
  }
}

// ---- fused encoder (bgcn_bigcn.hip); graph_lane: see bigcn_forward_impl
size_t bigcn_ws_size(int64_t N, int64_t B, int64_t F, int64_t hid);
struct Prepared;
struct WeightImages;
// img (bgcn_train_step): the caller's weight-image buffer replaces the workspace's copies;
// img_current: it already holds the current weights' images (no prologue launch)
int bigcn_forward_impl(const bgcn_bigcn_args* a, void* ws, size_t ws_bytes, hipStream_t s,
                       int graph_lane, const HeadArgs* head = nullptr,
                       const Prepared* prep = nullptr, const WeightImages* img = nullptr,
                       bool img_current = false);
// side_busy: the side lane carries other long work (a next-batch preparation); the dW2
// chain then stays on the caller's stream
// head (bgcn_train_step): the classifier head's weight gradients, run as extra blocks of
// the readout backward
int bigcn_backward_impl(const bgcn_bigcn_args* a, void* ws, size_t ws_bytes, hipStream_t s,
                        const Prepared* prep = nullptr, bool side_busy = false,
                        const HeadGradJob* head = nullptr, const WeightImages* img = nullptr,
                        bool defer_dw1 = false, const TailAdam* adam = nullptr, bool* adam_done = nullptr);
// the dW1 of a backward run with defer_dw1 (same arguments and buffers)
int bigcn_backward_dw1(const bgcn_bigcn_args* a, void* ws, size_t ws_bytes, hipStream_t s, const Prepared* prep,
                       const WeightImages* img);

// ---- prepared batch (bgcn_step.hip): the weight-independent state of one batch
// (sizes shared with bgcn_sparse.h: tree work items of kChunkItems nodes, CSC row blocks)
constexpr int kChunkItems = 256;
constexpr int kCscRowBlock = 256;
constexpr int64_t kSparseMaxFeat = 5120;   // widest X of the sparse path (one pass per row)
struct Prepared {
  bgcn_csr_out td, bu;
  SpmmPlan plan[2][2];                   // [td, bu][t (forward), s (backward)]
  int64_t td_cap, bu_cap;                // E + N
  int32_t *tree_ptr, *node_root, *status;
  int32_t *item_tree, *item_beg, *item_end, *item_root, *tree_item0;   // items: tree, node range, root
  int32_t *x_flags, *x_nnz, *x_cols;
  float* x_vals;
  int32_t* x_ovf_off;                    // [N] spill pool offsets (rows over the ELL cap)
  int32_t* x_long;                       // [N] list of the rows over the ELL cap
  uint2* x_ovf;                          // [ovf_cap] spilled (col, value bits)
  int64_t ovf_cap;
  int32_t *hist, *col_total, *col_start, *col_end;
  uint2* csc;   // [N * (kCap + kSpillPerRow)] (slot, value bits) grouped by column, rows in order
  void* gws;
  size_t gws_bytes;
  int64_t *td_drop, *bu_drop;            // [2, E] masked DropEdge lists (device DropEdge)
  void* dws;
  size_t dws_bytes;
};
size_t carve_prepared(Carve& c, int64_t N, int64_t B, int64_t F, int64_t Etd, int64_t Ebu,
                      Prepared* p);
// bgcn_bigcn_forward / _backward on a caller's prepared batch (bgcn_bigcn_args.prepared)
int bigcn_prepared_call(const bgcn_bigcn_args* a, void* ws, size_t ws_bytes, hipStream_t s, bool backward);

// ---- DropEdge (bgcn_drop.hip)
size_t drop_ws_size(int64_t B);
int drop_edges_impl(const int64_t* td, int64_t Etd, int64_t* td_out, int64_t ld_td, double td_rate,
                    const int64_t* bu, int64_t Ebu, int64_t* bu_out, int64_t ld_bu, double bu_rate,
                    const int64_t* batch, int64_t N, int64_t B, uint64_t seed, int masked,
                    int64_t* counts, int32_t* status, void* ws, size_t ws_bytes, hipStream_t s);

// ---- one training step (bgcn_step.hip)
size_t train_step_ws_size(int64_t N, int64_t B, int64_t F, int64_t C, int64_t Etd, int64_t Ebu);
int train_step_impl(const bgcn_step_args* a, void* ws, size_t ws_bytes, hipStream_t s);
// the evaluation loop's reductions after the head (bgcn_head.hip, k_eval_finish)
int eval_finish_impl(const float* loss_row, const float* logp, const int64_t* y, int64_t B, int32_t C, float* loss,
                     int32_t* correct, int64_t* pred, const int32_t* status, int32_t* status_seen, hipStream_t s);

}  // namespace bgcn
