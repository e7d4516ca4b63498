// Fused multi-tensor Adam (one launch for every parameter of the model).
//
// Replaces the optimiser step of the reference's training loop:
//   torch.optim.Adam([{base}, {BU conv1, lr/5}, {BU conv2, lr/5}], lr, weight_decay)
//   (model/Twitter/BiGCN_Twitter.py:146-153, step at :189)
// with torch's Adam semantics (amsgrad = False, maximize = False, weight decay added to
// the gradient = L2):
//   g = grad * grad_scale + wd * p ; m = lerp(m, g, 1 - b1) ; v = b2 v + (1 - b2) g^2
//   p -= lr / (1 - b1^t) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
// grad_scale folds the 1/world of the data-parallel mean into the step, so the reduced
// flat gradient bucket is consumed in place.
#include "bgcn_common.h"
#include "bgcn_sparse.h"

namespace bgcn {
namespace {

constexpr int kChunkElems = 256 * 4;  // elements per block (256 threads x one float4)
constexpr int H = 64;                  // rows of the conv weights with images

// four consecutive elements from e (vector when the tensor's arrays are 16-byte aligned)
__device__ __forceinline__ void adam_quad(const bgcn_adam_tensor& T, int64_t e, int n, bool vec,
                                          const AdamConst& c, float out[4]) {
  if (vec && n == 4) {
    float4 p = ld4(T.param + e), g = ld4(T.grad + e);
    float4 m = ld4(T.exp_avg + e), v = ld4(T.exp_avg_sq + e);
    adam_elem(p.x, g.x, m.x, v.x, c);
    adam_elem(p.y, g.y, m.y, v.y, c);
    adam_elem(p.z, g.z, m.z, v.z, c);
    adam_elem(p.w, g.w, m.w, v.w, c);
    st4(T.param + e, p);
    st4(T.exp_avg + e, m);
    st4(T.exp_avg_sq + e, v);
    out[0] = p.x; out[1] = p.y; out[2] = p.z; out[3] = p.w;
    return;
  }
  for (int j = 0; j < 4; ++j) {
    out[j] = 0.f;
    if (j >= n) continue;
    float p = T.param[e + j], m = T.exp_avg[e + j], v = T.exp_avg_sq[e + j];
    adam_elem(p, T.grad[e + j], m, v, c);
    T.param[e + j] = p;
    T.exp_avg[e + j] = m;
    T.exp_avg_sq[e + j] = v;
    out[j] = p;
  }
}

// A conv weight with a weight image (BGCN_IMAGE_*): tiles of kImgRows rows (o) x kImgCols
// columns (k), one float4 per thread per pass, every load of the tile issued before the
// first store; the updated values are staged in LDS and written transposed - W1^T[k][d*64
// + o] or W2^T_d[k][o], kImgRows * 4 contiguous bytes per k - plus, for W2's columns k <
// 64, the bf16 split images (conv2's hi / mid / lo [o][k] and the middle launch's hi / lo
// [k][o]): what the step's prologue would otherwise derive from the parameters.  The tile
// shape trades the parameter side's piece size against the image side's
// (profiles/r02_adam_images_ab.txt, the launch alone: 7.6-8.2 us without images; with
// them 16 x 128: 8.6, 8 x 256: 9.0, 16 x 256: 9.7, 64 x 32: 13.0).
#ifndef BGCN_IMG_COLS
#define BGCN_IMG_COLS 128
#endif
#ifndef BGCN_IMG_ROWS
#define BGCN_IMG_ROWS 16
#endif
constexpr int kImgCols = BGCN_IMG_COLS;      // columns (k) per tile
constexpr int kImgRows = BGCN_IMG_ROWS;      // rows (o) per tile
constexpr int kImgTpr = kImgCols / 4;        // threads per row piece (one float4 each)
constexpr int kImgRpp = 256 / kImgTpr;       // rows per pass
constexpr int kImgPasses = kImgRows / kImgRpp;
constexpr int kImgTpk = kImgRows / 4;        // threads per image row piece (one float4 each)
constexpr int kImgKpp = 256 / kImgTpk;       // image rows per pass
static_assert(kImgPasses >= 1 && kImgRpp * kImgPasses == kImgRows && H % kImgRows == 0 &&
                  kImgCols % kImgKpp == 0 && kImgCols >= H, "tile shape");
constexpr int kImgGroups = H / kImgRows;     // row groups per column tile
__device__ void adam_image_tile(const bgcn_adam_tensor& T, const AdamConst& c, int role, int64_t tile,
                                const WeightImages& im, int64_t F, bool vec) {
  __shared__ float tl[kImgCols][kImgRows + 1];   // [k][o - o_base]
  const bool w1 = role == BGCN_IMAGE_TD_W1 || role == BGCN_IMAGE_BU_W1;
  const int d = (role == BGCN_IMAGE_BU_W1 || role == BGCN_IMAGE_BU_W2) ? 1 : 0;
  const int64_t K = w1 ? F : F + H;
  const int ob = int(tile % kImgGroups) * kImgRows;
  const int64_t k0 = (tile / kImgGroups) * kImgCols;
  const int q = threadIdx.x % kImgTpr, r = threadIdx.x / kImgTpr;
  const int64_t k = k0 + 4 * q;
  const int n = k < K ? int(min<int64_t>(4, K - k)) : 0;
  float u[kImgPasses][4];
  if (vec && n == 4) {
    // every pass's loads issued before the first store
    float4 p[kImgPasses], g[kImgPasses], m[kImgPasses], v[kImgPasses];
#pragma unroll
    for (int t = 0; t < kImgPasses; ++t) {
      const int64_t e = int64_t(ob + r + t * kImgRpp) * K + k;
      p[t] = ld4(T.param + e); g[t] = ld4(T.grad + e); m[t] = ld4(T.exp_avg + e); v[t] = ld4(T.exp_avg_sq + e);
    }
#pragma unroll
    for (int t = 0; t < kImgPasses; ++t) {
      adam_elem(p[t].x, g[t].x, m[t].x, v[t].x, c); adam_elem(p[t].y, g[t].y, m[t].y, v[t].y, c);
      adam_elem(p[t].z, g[t].z, m[t].z, v[t].z, c); adam_elem(p[t].w, g[t].w, m[t].w, v[t].w, c);
      const int64_t e = int64_t(ob + r + t * kImgRpp) * K + k;
      st4(T.param + e, p[t]); st4(T.exp_avg + e, m[t]); st4(T.exp_avg_sq + e, v[t]);
      u[t][0] = p[t].x; u[t][1] = p[t].y; u[t][2] = p[t].z; u[t][3] = p[t].w;
    }
  } else {
#pragma unroll
    for (int t = 0; t < kImgPasses; ++t) adam_quad(T, int64_t(ob + r + t * kImgRpp) * K + k, n, false, c, u[t]);
  }
#pragma unroll
  for (int t = 0; t < kImgPasses; ++t) {
    const int ol = r + t * kImgRpp, o = ob + ol;
#pragma unroll
    for (int j = 0; j < 4; ++j) tl[4 * q + j][ol] = u[t][j];
    if (!w1 && k < H) {   // conv2's split image, row-major like W2 (k < 64 < K: n == 4)
      __bf16* cs = im.w2s + int64_t(d) * 3 * H * kW2sLd + o * kW2sLd + k;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        __bf16 x, y, z;
        split3_bf16(u[t][j], x, y, z);
        cs[j] = x;
        cs[H * kW2sLd + j] = y;
        cs[2 * H * kW2sLd + j] = z;
      }
    }
  }
  __syncthreads();
  // transposed: image rows k0 + kk, outputs [ob + 4qq, ob + 4qq + 4) - kImgRows * 4 contiguous
  // bytes per image row
  const int qq = threadIdx.x % kImgTpk;
#pragma unroll
  for (int kk = threadIdx.x / kImgTpk; kk < kImgCols; kk += kImgKpp) {
    const int64_t kr = k0 + kk;
    if (kr >= K) break;
    const float4 v = make_float4(tl[kk][4 * qq], tl[kk][4 * qq + 1], tl[kk][4 * qq + 2], tl[kk][4 * qq + 3]);
    const int o0 = ob + 4 * qq;
    float* dst = w1 ? im.w1t + kr * (2 * H) + d * H + o0 : im.w2t + (int64_t(d) * K + kr) * H + o0;
    st4(dst, v);
    if (!w1 && kr < H) {   // the middle launch's split image [c][o] (c = kr): hi / mid / lo
      __bf16* ds = im.w2d + int64_t(d) * 3 * H * kW2dLd + kr * kW2dLd + o0;
      const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        __bf16 x, y, z;
        split3_bf16(vv[j], x, y, z);
        ds[j] = x;
        ds[H * kW2dLd + j] = y;
        ds[2 * H * kW2dLd + j] = z;
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_adam(bgcn_adam_args a, WeightImages im) {
  if (a.skip_flag && *a.skip_flag != 0.0f) {   // invalid step (any rank): no update
    if (blockIdx.x == 0 && threadIdx.x == 0 && a.skip_count) atomicAdd(a.skip_count, 1);
    return;
  }
  // locate this block's tensor (at most BGCN_ADAM_MAX_TENSORS, uniform scan)
  int k = 0;
  while (k + 1 < a.count && int64_t(blockIdx.x) >= a.block_start[k + 1]) ++k;
  const bgcn_adam_tensor& T = a.t[k];
  const AdamConst c{a.beta1, a.beta2, a.weight_decay, a.eps, T.lr / a.bias_correction1,
                    1.0f / a.bias_correction2_sqrt, a.grad_scale};
  const int role = a.images ? a.image_role[k] : BGCN_IMAGE_NONE;
  if (role != BGCN_IMAGE_NONE) {
    const bool vec = ((reinterpret_cast<uintptr_t>(T.param) | reinterpret_cast<uintptr_t>(T.grad) |
                       reinterpret_cast<uintptr_t>(T.exp_avg) |
                       reinterpret_cast<uintptr_t>(T.exp_avg_sq)) & 15u) == 0;
    adam_image_tile(T, c, role, int64_t(blockIdx.x) - a.block_start[k], im, a.images_in_feats, vec);
    return;
  }
  const int64_t e0 = (int64_t(blockIdx.x) - a.block_start[k]) * kChunkElems + threadIdx.x * 4;
  const bool vec = ((reinterpret_cast<uintptr_t>(T.param) | reinterpret_cast<uintptr_t>(T.grad) |
                     reinterpret_cast<uintptr_t>(T.exp_avg) |
                     reinterpret_cast<uintptr_t>(T.exp_avg_sq)) & 15u) == 0;
  if (vec && e0 + 4 <= T.numel) {
    float4 p = ld4(T.param + e0), g = ld4(T.grad + e0);
    float4 m = ld4(T.exp_avg + e0), v = ld4(T.exp_avg_sq + e0);
    adam_elem(p.x, g.x, m.x, v.x, c);
    adam_elem(p.y, g.y, m.y, v.y, c);
    adam_elem(p.z, g.z, m.z, v.z, c);
    adam_elem(p.w, g.w, m.w, v.w, c);
    st4(T.param + e0, p);
    st4(T.exp_avg + e0, m);
    st4(T.exp_avg_sq + e0, v);
    return;
  }
  for (int64_t e = e0; e < e0 + 4 && e < T.numel; ++e) {
    float p = T.param[e], m = T.exp_avg[e], v = T.exp_avg_sq[e];
    adam_elem(p, T.grad[e], m, v, c);
    T.param[e] = p;
    T.exp_avg[e] = m;
    T.exp_avg_sq[e] = v;
  }
}

}  // namespace
}  // namespace bgcn

extern "C" int bgcn_adam_step(const bgcn_adam_args* args, bgcn_stream_t stream) {
  using namespace bgcn;
  if (!args || args->count < 1 || args->count > BGCN_ADAM_MAX_TENSORS)
    return fail(BGCN_EINVAL, "adam: 1..BGCN_ADAM_MAX_TENSORS tensors");
  bgcn_adam_args a = *args;
  const int64_t F = a.images_in_feats;
  WeightImages im{};
  if (a.images) {
    if (F <= 0) return fail(BGCN_EINVAL, "adam: images need images_in_feats > 0");
    Carve ci(a.images, bgcn_weight_images_size(F));
    carve_images(ci, F, &im);
  }
  int64_t blocks = 0;
  for (int k = 0; k < a.count; ++k) {
    const bgcn_adam_tensor& T = a.t[k];
    if (T.numel < 0 || (T.numel > 0 && (!T.param || !T.grad || !T.exp_avg || !T.exp_avg_sq)))
      return fail(BGCN_EINVAL, "adam: bad tensor");
    a.block_start[k] = blocks;
    const int role = a.images ? a.image_role[k] : BGCN_IMAGE_NONE;
    if (role != BGCN_IMAGE_NONE) {
      if (role < BGCN_IMAGE_TD_W1 || role > BGCN_IMAGE_BU_W2) return fail(BGCN_EINVAL, "adam: bad image_role");
      const int64_t K = role <= BGCN_IMAGE_BU_W1 ? F : F + H;
      if (T.numel != int64_t(H) * K || F % 4 != 0)
        return fail(BGCN_EINVAL, "adam: an image tensor must be [64][in_feats] (W1) / [64][in_feats + 64] (W2)");
      blocks += kImgGroups * ((K + kImgCols - 1) / kImgCols);
    } else {
      blocks += (T.numel + kChunkElems - 1) / kChunkElems;
    }
  }
  if (blocks == 0) return BGCN_OK;
  hipLaunchKernelGGL(k_adam, dim3(unsigned(blocks)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), a, im);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}
