// K9: the classifier head of BiGCN.forward for the per-op (autograd) path:
//   logp = log_softmax(head_in . fc_w^T + fc_b, dim=1)      (BiGCN_Twitter.py:129-130,
//                                                            BiGCN_Weibo.py:87-88)
// and its backward from an arbitrary dlogp (loss.backward() through F.nll_loss or any
// other loss on logp):
//   dz = dlogp - exp(logp) * rowsum(dlogp),  dhead = dz . fc_w,  dfc_w = dz^T . head_in,
//   dfc_b = colsum(dz).
// The rows are the B trees of a batch (128 x 256 at the reference batch) and C <= 16
// classes: launch-bound work, one launch each way.  The fused training step has this head
// inside its readout (bgcn_bigcn.hip); these entry points give the drop-in modules the
// same single launch instead of a library GEMM + log_softmax (+ three backward kernels).
#include "bgcn_internal.h"

namespace bgcn {
namespace {

constexpr int kHeadK = 256;   // cat(BU_x, TD_x) = 4 x 64 (hid = out = 64): lane l holds columns 4l .. 4l+3

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// one wave per tree row, four rows per 256-thread block
__global__ __launch_bounds__(256) void k_head_fwd(const float* __restrict__ head, const float* __restrict__ W,
                                                  const float* __restrict__ bias, int64_t B, int C,
                                                  float* __restrict__ logp) {
  const int64_t b = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int l = threadIdx.x & 63;
  if (b >= B) return;
  const float4 h = *reinterpret_cast<const float4*>(head + b * kHeadK + 4 * l);
  float z[kMaxClasses];
  float mx = -INFINITY;
#pragma unroll
  for (int c = 0; c < kMaxClasses; ++c) {
    if (c < C) {
      const float4 w = *reinterpret_cast<const float4*>(W + int64_t(c) * kHeadK + 4 * l);
      z[c] = wave_sum(h.x * w.x + h.y * w.y + h.z * w.z + h.w * w.w) + bias[c];
      mx = fmaxf(mx, z[c]);
    }
  }
  float se = 0.f;
#pragma unroll
  for (int c = 0; c < kMaxClasses; ++c)
    if (c < C) se += expf(z[c] - mx);
  const float lse = mx + logf(se);
#pragma unroll
  for (int c = 0; c < kMaxClasses; ++c)
    if (c < C && l == c) logp[b * C + c] = z[c] - lse;
}

// blocks [0, nrow): dhead, one wave per tree row; blocks [nrow, nrow + C): dfc_w row c
// over the 256 columns (one thread each) and, by thread 0, dfc_b[c] - both summed over
// the trees in index order (deterministic)
__global__ __launch_bounds__(256) void k_head_bwd(const float* __restrict__ head, const float* __restrict__ logp,
                                                  const float* __restrict__ dlogp, const float* __restrict__ W,
                                                  int64_t B, int C, int nrow, float* __restrict__ dhead,
                                                  float* __restrict__ dW, float* __restrict__ db) {
  if (int(blockIdx.x) < nrow) {
    const int64_t b = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
    const int l = threadIdx.x & 63;
    if (b >= B) return;
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += dlogp[b * C + c];
    float4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < C; ++c) {
      const float dz = dlogp[b * C + c] - expf(logp[b * C + c]) * s;
      const float4 w = *reinterpret_cast<const float4*>(W + int64_t(c) * kHeadK + 4 * l);
      acc.x += dz * w.x; acc.y += dz * w.y; acc.z += dz * w.z; acc.w += dz * w.w;
    }
    *reinterpret_cast<float4*>(dhead + b * kHeadK + 4 * l) = acc;
    return;
  }
  __shared__ float dzs[256];
  const int c = int(blockIdx.x) - nrow, j = threadIdx.x;
  float acc = 0.f, bsum = 0.f;
  for (int64_t b0 = 0; b0 < B; b0 += 256) {
    const int64_t b = b0 + threadIdx.x;
    float dz = 0.f;
    if (b < B) {
      float s = 0.f;
      for (int k = 0; k < C; ++k) s += dlogp[b * C + k];
      dz = dlogp[b * C + c] - expf(logp[b * C + c]) * s;
    }
    dzs[threadIdx.x] = dz;
    __syncthreads();
    const int nb = int(min<int64_t>(256, B - b0));
#pragma unroll 16   // sixteen independent head loads in flight (a dependent chain of 128 ran 9 us)
    for (int t = 0; t < nb; ++t) acc += dzs[t] * head[(b0 + t) * kHeadK + j];
    if (j == 0)
      for (int t = 0; t < nb; ++t) bsum += dzs[t];
    __syncthreads();
  }
  dW[int64_t(c) * kHeadK + j] = acc;
  if (j == 0) db[c] = bsum;
}

bool a16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// The evaluation loop's per-batch reductions (BiGCN_Twitter.py:218-222: val_loss =
// F.nll_loss(val_out, y); _, val_pred = val_out.max(dim=1); correct = val_pred.eq(y).sum())
// on the device, one 256-thread block: the mean NLL over the head's per-tree terms summed in
// the order the training step's loss uses (head_grad_block: strided thread sums, then a
// halving tree), the argmax per tree (the first maximal class, as torch's max), the count of
// correct predictions, and the step's status folded into status_seen.
__global__ __launch_bounds__(256) void k_eval_finish(const float* __restrict__ loss_row,
                                                     const float* __restrict__ logp,
                                                     const int64_t* __restrict__ y, int64_t B, int C,
                                                     float* __restrict__ loss, int32_t* __restrict__ correct,
                                                     int64_t* __restrict__ pred, const int32_t* status,
                                                     int32_t* status_seen) {
  __shared__ float ls[256];
  __shared__ int32_t cs[256];
  const int t = threadIdx.x;
  float a = 0.f;
  int32_t n = 0;
  for (int64_t b = t; b < B; b += 256) {
    a += loss_row[b];
    int best = 0;
    float bv = logp[b * C];
    for (int c = 1; c < C; ++c) {
      const float v = logp[b * C + c];
      if (v > bv) { bv = v; best = c; }
    }
    if (pred) pred[b] = best;
    n += (y[b] == int64_t(best)) ? 1 : 0;
  }
  ls[t] = a;
  cs[t] = n;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) {
      ls[t] += ls[t + o];
      cs[t] += cs[t + o];
    }
    __syncthreads();
  }
  if (t == 0) {
    *loss = ls[0] / float(B);
    if (correct) *correct = cs[0];
    const int32_t st = status ? *status & 15 : 0;
    if (status_seen && st) atomicOr(status_seen, st);
  }
}

}  // namespace

int eval_finish_impl(const float* loss_row, const float* logp, const int64_t* y, int64_t B, int32_t C, float* loss,
                     int32_t* correct, int64_t* pred, const int32_t* status, int32_t* status_seen, hipStream_t s) {
  BGCN_CHECK_ARG(B > 0 && C > 0 && C <= kMaxClasses, "need B > 0 and 0 < C <= 16");
  BGCN_CHECK_ARG(loss_row && logp && y && loss, "null pointer");
  hipLaunchKernelGGL(k_eval_finish, dim3(1), dim3(256), 0, s, loss_row, logp, y, B, C, loss, correct, pred, status,
                     status_seen);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

int head_fwd_impl(const float* head, const float* W, const float* bias, int64_t B, int32_t C, float* logp,
                  hipStream_t s) {
  BGCN_CHECK_ARG(B > 0 && C > 0 && C <= kMaxClasses, "need B > 0 and 0 < C <= 16");
  BGCN_CHECK_ARG(head && W && bias && logp, "null pointer");
  BGCN_CHECK_ARG(a16(head) && a16(W), "head_in / fc_w must be 16-byte aligned");
  hipLaunchKernelGGL(k_head_fwd, dim3(unsigned((B + 3) / 4)), dim3(256), 0, s, head, W, bias, B, C, logp);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

int head_bwd_impl(const float* head, const float* logp, const float* dlogp, const float* W, int64_t B,
                  int32_t C, float* dhead, float* dW, float* db, hipStream_t s) {
  BGCN_CHECK_ARG(B > 0 && C > 0 && C <= kMaxClasses, "need B > 0 and 0 < C <= 16");
  BGCN_CHECK_ARG(head && logp && dlogp && W && dhead && dW && db, "null pointer");
  BGCN_CHECK_ARG(a16(head) && a16(W) && a16(dhead), "head_in / fc_w / dhead must be 16-byte aligned");
  const int64_t nrow = (B + 3) / 4;
  BGCN_CHECK_ARG(nrow < (int64_t(1) << 30), "batch too large");
  hipLaunchKernelGGL(k_head_bwd, dim3(unsigned(nrow + C)), dim3(256), 0, s, head, logp, dlogp, W, B, C,
                     int(nrow), dhead, dW, db);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

}  // namespace bgcn

extern "C" int bgcn_head_forward(const float* head_in, const float* fc_w, const float* fc_b, int64_t num_graphs,
                                 int32_t num_classes, float* logp, bgcn_stream_t stream) {
  return bgcn::head_fwd_impl(head_in, fc_w, fc_b, num_graphs, num_classes, logp,
                             reinterpret_cast<hipStream_t>(stream));
}

extern "C" int bgcn_head_backward(const float* head_in, const float* logp, const float* dlogp, const float* fc_w,
                                  int64_t num_graphs, int32_t num_classes, float* dhead_in, float* fc_dw,
                                  float* fc_db, bgcn_stream_t stream) {
  return bgcn::head_bwd_impl(head_in, logp, dlogp, fc_w, num_graphs, num_classes, dhead_in, fc_dw, fc_db,
                             reinterpret_cast<hipStream_t>(stream));
}
